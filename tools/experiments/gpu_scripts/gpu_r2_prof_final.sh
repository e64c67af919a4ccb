#!/bin/bash
# rocprof kernel trace of a 2-micro-batch bench step on the final tree (step breakdown).
set -o pipefail
mkdir -p gpurun_out/proff
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/proff/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > gpurun_out/proff/prof.log 2>&1
rc=$?; echo "prof rc=$rc" >> gpurun_out/proff/prof.log
exit $rc
