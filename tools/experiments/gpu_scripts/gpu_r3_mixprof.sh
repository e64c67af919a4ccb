#!/bin/bash
# Mixtral 4-layer step: kernel stats per MoE backend (grouped vs loop), one timed step after warmup.
set -o pipefail
O=gpurun_out/r3mix; mkdir -p $O
export TMPDIR=/tmp
for b in grouped loop; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$b -o run -- python3 tools/bench_mixtral_train.py --layers 4 --seq 4096 --mbs 2 --accum 4 --steps 1 --warmup 1 --backends $b > $O/$b.log 2>&1 || exit $?
  find $O/$b -name '*kernel_trace*' -delete
done
