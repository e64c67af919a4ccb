#!/bin/bash
# Round 4: emulated ranks with the receiving-side writes beside (not behind) the link spin.
set -o pipefail
O=gpurun_out/r4emucopy; mkdir -p $O
export TMPDIR=/tmp
E="python -u tools/emulate_tp_rank.py --steps 3 --warmup 1"
run() { echo "== $*" >&2; timeout -k 10 300 $E "$@" > $O/run.log 2>> $O/emulate.err || exit $?; grep '^{' $O/run.log >> $O/emulate.jsonl || exit $?; }
run --tp 8 --link-gbps 400 --sp-streams 2
run --tp 8 --link-gbps 400 --sp-streams 1
run --tp 4 --link-gbps 200 --sp-streams 2
run --tp 2 --link-gbps 70 --sp-streams 2
run --tp 8 --link-gbps 400 --sp-streams 2 --link-cus 16
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python -u tools/emulate_tp_rank.py --tp 8 --layers 8 --steps 2 --warmup 1 --link-gbps 400 --sp-streams 2 > $O/prof.log 2>&1 || exit $?
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/stream_timeline.py $T --json > $O/timeline.json || exit $?
find $O/prof -name "*.csv" -delete
