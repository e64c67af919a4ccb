#!/bin/bash
# Round 4: SP chunk count (NXD_SP_CHUNKS) with the staggered halves on the emulated ranks.
set -o pipefail
O=gpurun_out/r4chunks; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --sp-streams 2"
run() { echo "== c=$C $*" >&2; NXD_SP_CHUNKS=$C timeout -k 10 300 $E "$@" > $O/run.log 2>> $O/emulate.err || exit $?; grep '^{' $O/run.log >> $O/emulate.jsonl || exit $?; }
for C in 2 8 1 4; do run --tp 8 --link-gbps 400; done
for C in 2 8; do run --tp 4 --link-gbps 200; done
for C in 2 8; do run --tp 2 --link-gbps 70; done
