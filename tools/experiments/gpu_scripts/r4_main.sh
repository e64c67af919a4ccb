#!/bin/bash
# Round 4: 1-GPU bench through the public API (driver contract), then the k-parts emulation +
# exhaustive-GEMM rehearsal.
set -o pipefail
O=gpurun_out/r4main; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
bash tools/gpu/r4_parts.sh || exit $?
