#!/bin/bash
set -o pipefail
D=gpurun_out/r3wg3; mkdir -p $D
export TMPDIR=/tmp
for ab in 0 1 3 5 7; do timeout -k 10 120 python tools/prof_wgrad.py 8192 28672 4096 10 $ab >> $D/ablate.jsonl 2>&1 || exit $?; done
for ab in 0 1 3 5; do timeout -k 10 120 python tools/prof_wgrad.py 32768 768 4096 20 $ab >> $D/ablate.jsonl 2>&1 || exit $?; done
