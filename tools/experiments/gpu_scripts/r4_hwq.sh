#!/bin/bash
# Round 4: hardware queues per process (GPU_MAX_HW_QUEUES; streams beyond it share queues and
# inherit each other's barrier waits) x SP parts on the emulated TP=8 rank, + stream-K CU cap.
set -o pipefail
O=gpurun_out/r4hwq; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1 --tp 8 --link-gbps 400"
for q in 8 16; do
  for k in 2 4; do
    echo "== q=$q k=$k" >&2
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $E --sp-streams $k > $O/run.log 2>> $O/emulate.err || exit $?
    grep '^{' $O/run.log | sed "s/^{/{\"hw_queues\": $q, /" >> $O/emulate.jsonl || exit $?
  done
done
bash tools/gpu/r4_skcus.sh || exit $?
