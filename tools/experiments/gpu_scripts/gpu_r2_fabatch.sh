#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 400 python tools/bench_fa_batch.py --batch 1 2 4 --chunks 0 16 32 64 > gpurun_out/r2/fa_batch.jsonl 2> gpurun_out/r2/fa_batch.err
