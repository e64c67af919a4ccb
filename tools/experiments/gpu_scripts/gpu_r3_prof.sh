#!/bin/bash
# TP=1 step profile (2 micro-batches) on the current tree: per-category and per-kernel breakdown.
set -o pipefail
D=gpurun_out/r3prof; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > $D/bench.log 2>&1 || exit $?
T=$(find $D -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $D/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $D/breakdown_by_kernel.txt
