#!/bin/bash
# Round 4: the emulated TP=2 / TP=4 "slower than serialized" stall -- allocator stats, buffer
# lifetime (record_stream vs stash), link spin (shader-clock sleep vs real-time counter).
set -o pipefail
O=gpurun_out/r4stall; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1"
run() { echo "== $*" >&2; timeout -k 10 300 $E "$@" >> $O/emulate.jsonl 2>> $O/emulate.err || exit $?; }
run --tp 4 --link-gbps 200 --sp-streams 2 --sync record --spin sleep
run --tp 4 --link-gbps 200 --sp-streams 2 --sync record --spin realtime
run --tp 4 --link-gbps 200 --sp-streams 2 --sync stash
run --tp 4 --link-gbps 200 --sp-streams 1 --sync stash
run --tp 4 --sp-streams 2
run --tp 2 --link-gbps 70 --sp-streams 2 --sync stash
run --tp 8 --link-gbps 400 --sp-streams 2 --sync stash
