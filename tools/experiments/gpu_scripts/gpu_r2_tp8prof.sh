#!/bin/bash
# rocprof kernel stats of one Llama-3-8B micro-batch at TP=8 per-rank shapes (one GPU, no comm)
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/tp8prof -o run --output-format csv -- python tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 2 > gpurun_out/r2/tp8prof.log 2>&1
