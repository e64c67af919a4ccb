#!/bin/bash
# Per-GPU compute floor (no comm) of one bench micro-batch at TP = 1 / 2 / 4 / 8 per-rank shapes, each at the
# micro-batch bench.py uses for that degree (MBS_BY_TP), 8 layers.
set -o pipefail
O=gpurun_out/r3tpfloor; mkdir -p $O
timeout -k 10 200 python -u tools/profile_tp_shapes.py --tp 1 --layers 8 --iters 3 --mbs 1 > $O/tp1.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/profile_tp_shapes.py --tp 2 --layers 8 --iters 3 --mbs 2 > $O/tp2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/profile_tp_shapes.py --tp 4 --layers 8 --iters 3 --mbs 4 > $O/tp4.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/profile_tp_shapes.py --tp 8 --layers 8 --iters 3 --mbs 4 > $O/tp8.log 2>&1 || exit $?
grep -h "{" $O/tp*.log > $O/floor.jsonl
