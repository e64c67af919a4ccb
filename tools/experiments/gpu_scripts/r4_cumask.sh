#!/bin/bash
# Round 4: CU-masked compute streams for the SP halves (NXD_SP_RESERVE_CUS CUs left to the collectives)
# on the emulated TP=8 / TP=4 ranks.
set -o pipefail
O=gpurun_out/r4cumask; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --sp-streams 2"
run() { echo "== res=$R $*" >&2; NXD_SP_RESERVE_CUS=$R timeout -k 10 300 $E "$@" > $O/run.log 2>> $O/emulate.err || exit $?; grep '^{' $O/run.log | sed "s/^{/{\"reserve_cus\": $R, /" >> $O/emulate.jsonl || exit $?; }
for R in 8 16 0; do R=$R run --tp 8 --link-gbps 400; done
for R in 16 0; do R=$R run --tp 8 --link-gbps 400 --link-cus 16; done
for R in 8 0; do R=$R run --tp 8; done
for R in 8 0; do R=$R run --tp 4 --link-gbps 200; done
