#!/bin/bash
# wgrad / grouped 256-tile kernel variants (ring depth, band, s_setprio), wgrad dispatch tests,
# TP=1 step profile and a 1-GPU bench.
set -o pipefail
O=gpurun_out/r3combo; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py tests/test_moe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_wgrad.log 2>&1 || exit $?
NXD_GRG_STAGES=5 NXD_GRG_PRIO=1 NXD_WG_PRIO=1 timeout -k 10 200 python -u -m pytest tests/test_moe_gpu.py tests/test_wgrad_gemm_gpu.py -m gpu -x -q -k "grouped_gemm or wgrad" --timeout 120 --timeout-method thread > $O/pytest_variants.log 2>&1 || exit $?
for pr in 0 1 2; do
  NXD_WG_PRIO=$pr timeout -k 10 200 python -u tools/bench_wgrad.py > $O/wg_prio$pr.jsonl 2>&1 || exit $?
done
for cfg in "4 4 0" "4 4 1" "4 4 2" "5 4 0" "5 4 1" "4 8 0"; do
  set -- $cfg
  NXD_GRG_STAGES=$1 NXD_GRG_BAND=$2 NXD_GRG_PRIO=$3 NXD_WG_PRIO=$3 timeout -k 10 200 python -u tools/bench_grouped_gemm.py > $O/grg_s$1_b$2_p$3.jsonl 2>&1 || exit $?
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > $O/prof_bench.log 2>&1 || exit $?
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $O/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $O/breakdown_by_kernel.txt && rm -f $T
timeout -k 10 900 python bench.py --gpus 1 --steps 5 --warmup 2 > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tp8prof -o run --output-format csv -- python tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 2 --mbs 4 > $O/tp8prof.log 2>&1 || exit $?
T=$(find $O/tp8prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T --split emb > $O/tp8_breakdown.txt && python tools/step_breakdown.py $T --split emb --by-kernel > $O/tp8_breakdown_by_kernel.txt && rm -f $T
