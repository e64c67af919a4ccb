#!/bin/bash
# Round-4 check on the final tree (after the SPMD test fix): GPU suite + smoke + bench, the SPMD TP=2
# test twice more (stability), then the rocprof breakdown of one bench step.
bash tools/gpu/round_check.sh r4c || exit $?
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_spmd_inference_gpu.py > gpurun_out/r4c_spmd_rerun_$i.log 2>&1 || exit $?
done
O=gpurun_out/r4c_prof; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $O/bench.log 2>&1 || exit $?
T=$(find $O -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $O/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $O/breakdown_by_kernel.txt || exit $?
rm -f $T
S=$(find $O -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats.csv
find $O -name "*.csv" ! -name kernel_stats.csv -delete
