#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 400 python tools/bench_fa_batch.py --batch 1 2 4 8 --layouts sbhd --chunks 0 64 96 128 160 224 > gpurun_out/r2/fa_batch2.jsonl 2> gpurun_out/r2/fa_batch2.err
