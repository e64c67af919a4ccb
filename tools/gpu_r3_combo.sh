#!/bin/bash
# grouped 256-tile ring-depth / band sweep, wgrad dispatch tests, TP=1 step profile and a 1-GPU bench
set -o pipefail
O=gpurun_out/r3combo; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_wgrad.log 2>&1 || exit $?
NXD_GRG_STAGES=5 timeout -k 10 200 python -u -m pytest tests/test_moe_gpu.py -m gpu -x -q -k grouped_gemm --timeout 120 --timeout-method thread > $O/pytest_s5.log 2>&1 || exit $?
for cfg in "4 4" "5 4" "4 8" "5 8"; do
  set -- $cfg
  NXD_GRG_STAGES=$1 NXD_GRG_BAND=$2 timeout -k 10 200 python -u tools/bench_grouped_gemm.py > $O/grg_s$1_b$2.jsonl 2>&1 || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > $O/prof_bench.log 2>&1 || exit $?
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $O/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $O/breakdown_by_kernel.txt && rm -f $T
timeout -k 10 900 python bench.py --gpus 1 --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit $?
