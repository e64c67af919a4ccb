#!/bin/bash
# Round 4: micro-batch parts on k streams (NXD_SP_STREAMS=k) on the emulated TP rank with the link
# model, k = 1 / 2 / 4 / 8; then the exhaustive-GEMM TP=4 training rehearsal vs the default mode.
set -o pipefail
O=gpurun_out/r4parts; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1"
run() { echo "== $*" >&2; timeout -k 10 300 $E "$@" 2>> $O/emulate.err | grep '^{' >> $O/emulate.jsonl || exit $?; }
for k in 2 4 8 1; do run --tp 8 --link-gbps 400 --sp-streams $k; done
for k in 2 4; do run --tp 8 --sp-streams $k; done
for k in 2 4; do NXD_GEMM_NO_STREAMK=1 run --tp 8 --link-gbps 400 --sp-streams $k; done
for k in 2 4; do run --tp 4 --link-gbps 200 --sp-streams $k; done
for k in 2 4; do run --tp 2 --link-gbps 70 --sp-streams $k; done
timeout -k 10 300 python -u tools/gemm_mode_rehearsal.py > $O/gemm_mode_default.out 2> $O/gemm_mode_default.err || exit $?
NXD_GEMM_TUNE=2 NXD_GEMM_NO_STREAMK=1 timeout -k 10 400 python -u tools/gemm_mode_rehearsal.py > $O/gemm_mode_exh.out 2> $O/gemm_mode_exh.err || exit $?
