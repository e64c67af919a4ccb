#!/bin/bash
# Round-end check: GPU suite + smoke + bench, then a rocprof kernel breakdown of the bench step.
bash tools/gpu/round_check.sh r3e || exit $?
O=gpurun_out/r3e_prof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
T=$(find $O -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $O/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $O/breakdown_by_kernel.txt && rm -f $T
S=$(find $O -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats.csv
head -14 $O/breakdown.txt
