#!/bin/bash
# wgrad kernel vs hipBLASLt (PP loop), TP=8-shape micro-batch timing + kernel breakdown, then the real
# TP=8 + SP path's kernel mix (8 gloo-gpu ranks on the one GPU, 2 layers).
set -o pipefail
O=gpurun_out/r3tp8b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_wgrad.py > $O/bench_wgrad_pp.jsonl 2>&1 || exit $?
timeout -k 10 300 python -u tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 3 --mbs 4 > $O/tp8_shapes.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 2 --mbs 4 > $O/prof.log 2>&1 || exit $?
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T --split emb::fwd > $O/breakdown.txt && python tools/step_breakdown.py $T --split emb::fwd --by-kernel > $O/breakdown_by_kernel.txt && rm -f $T
bash tools/gpu_r3_tp8rehearsal.sh || exit $?
