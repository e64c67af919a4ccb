#!/bin/bash
# Mixtral (4 full-width layers) training throughput per MoE backend + kernel stats of one step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mixtral; mkdir -p $O
timeout -k 10 600 python -u tools/bench_mixtral_train.py --layers 4 --seq 4096 --mbs 2 --accum 4 --steps 3 > $O/train.jsonl 2> $O/train.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_mixtral_train.py --layers 4 --seq 4096 --mbs 2 --accum 4 --steps 1 --warmup 1 --backends grouped > $O/prof.log 2>&1 || exit $?
find $O/prof -name '*kernel_trace*' -delete
