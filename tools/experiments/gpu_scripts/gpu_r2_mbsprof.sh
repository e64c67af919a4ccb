#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r2/mbs1prof -o run --output-format csv -- python tools/profile_tp_shapes.py --tp 1 --mbs 1 --layers 4 --iters 1 > gpurun_out/r2/mbs1prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r2/mbs2prof -o run --output-format csv -- python tools/profile_tp_shapes.py --tp 1 --mbs 2 --layers 4 --iters 1 > gpurun_out/r2/mbs2prof.log 2>&1
