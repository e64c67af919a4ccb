#!/bin/bash
# Round 4: leave CUs free for the collectives -- hipBLASLt stream-K GEMMs limited to N CUs
# (TENSILE_STREAMK_MAX_CUS) on the emulated TP=8 rank with the link model (1 / 16 link CUs).
set -o pipefail
O=gpurun_out/r4skcus; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --tp 8 --link-gbps 400 --sp-streams 2"
run() { echo "== $*" >&2; timeout -k 10 300 $E "$@" > $O/run.log 2>> $O/emulate.err || exit $?; grep '^{' $O/run.log | sed "s/^{/{\"streamk_max_cus\": \"${TENSILE_STREAMK_MAX_CUS:-all}\", /" >> $O/emulate.jsonl || exit $?; }
for c in all 240 224; do
  for lc in 1 16; do
    if [ $c = all ]; then unset TENSILE_STREAMK_MAX_CUS; else export TENSILE_STREAMK_MAX_CUS=$c; fi
    run --link-cus $lc
  done
done
unset TENSILE_STREAMK_MAX_CUS
export TENSILE_STREAMK_MAX_CUS=240
timeout -k 10 300 python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --tp 8 --sp-streams 2 2>> $O/emulate.err | grep '^{' | sed 's/^{/{"streamk_max_cus": "240", /' >> $O/emulate.jsonl || exit $?
unset TENSILE_STREAMK_MAX_CUS
timeout -k 10 300 python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --tp 8 --sp-streams 2 2>> $O/emulate.err | grep '^{' | sed 's/^{/{"streamk_max_cus": "all", /' >> $O/emulate.jsonl || exit $?
