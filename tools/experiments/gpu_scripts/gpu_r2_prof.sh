#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2/benchprof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > gpurun_out/r2/benchprof.log 2>&1
