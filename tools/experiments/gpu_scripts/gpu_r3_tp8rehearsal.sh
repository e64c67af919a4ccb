#!/bin/bash
# Kernel mix of the REAL TP=8 + SP code path (bench.py, Llama-3-8B shapes, 2 layers): 8 gloo-gpu ranks
# share the one GPU, each rank's kernels traced (timings inflated by sharing; counts and kinds exact).
set -o pipefail
O=gpurun_out/r3tp8gg; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --gpus 8 --gloo-gpu --layers 2 --steps 1 --warmup 1 > $O/bench.log 2>&1 || exit $?
python tools/rank_kernel_mix.py $O/prof > $O/rank_mix.jsonl || exit $?
find $O/prof -name "*.csv" -size +1M -delete
