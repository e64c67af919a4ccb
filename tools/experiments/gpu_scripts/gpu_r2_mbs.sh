#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 500 python tools/profile_tp_shapes.py --tp 8 4 2 --mbs 1 2 4 8 --layers 8 --iters 2 > gpurun_out/r2/mbs_sweep.jsonl 2> gpurun_out/r2/mbs_sweep.err || exit $?
timeout -k 10 300 python tools/profile_tp_shapes.py --tp 1 --mbs 1 2 --layers 8 --iters 2 >> gpurun_out/r2/mbs_sweep.jsonl 2>> gpurun_out/r2/mbs_sweep.err
