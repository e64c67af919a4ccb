#!/bin/bash
# TP=8-shape micro-batch (8 layers, 4 sequences, one GPU): wgrad kernel off vs auto, and a per-kernel breakdown.
set -o pipefail
O=gpurun_out/r3tp8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py tests/test_moe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for k in 0 auto 0 auto; do
  NXD_WGRAD_KERNEL=$k timeout -k 10 300 python -u tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 3 --mbs 4 >> $O/ab_kernel_$k.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 2 --mbs 4 > $O/prof.log 2>&1 || exit $?
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T --split emb::fwd > $O/breakdown.txt && python tools/step_breakdown.py $T --split emb::fwd --by-kernel > $O/breakdown_by_kernel.txt && rm -f $T
timeout -k 10 300 python -u tools/bench_wgrad.py > $O/bench_wgrad.jsonl 2>&1 || exit $?
