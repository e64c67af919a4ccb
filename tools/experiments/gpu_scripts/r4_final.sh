#!/bin/bash
# Round-4 check on the final tree: GPU suite + smoke + bench (round_check.sh), then a rocprof kernel
# breakdown of one bench step (TP=1 halves).
bash tools/gpu/round_check.sh r4b || exit $?
O=gpurun_out/r4b_prof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $O/bench.log 2>&1 || exit $?
T=$(find $O -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $O/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $O/breakdown_by_kernel.txt || exit $?
python tools/stream_timeline.py $T --json > $O/timeline.json || true
rm -f $T
S=$(find $O -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats.csv
find $O -name "*.csv" ! -name kernel_stats.csv -delete
