#!/bin/bash
# Round 4: phase stagger between the two SP halves (NXD_SP_STAGGER) on the emulated ranks.
set -o pipefail
O=gpurun_out/r4stagger; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --sp-streams 2"
run() { echo "== $*" >&2; timeout -k 10 300 $E "$@" > $O/run.log 2>> $O/emulate.err || exit $?; grep '^{' $O/run.log >> $O/emulate.jsonl || exit $?; }
for st in 1 2 3 4 0; do run --tp 8 --link-gbps 400 --sp-stagger $st; done
run --tp 8 --sp-stagger 2
for st in 2 0; do run --tp 4 --link-gbps 200 --sp-stagger $st; done
for st in 2 0; do run --tp 2 --link-gbps 70 --sp-stagger $st; done
