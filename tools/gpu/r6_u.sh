#!/bin/bash
# projected scaling on the final tree: emulated TP ranks with a link model (per-GPU link bandwidth as
# RCCL would see it on the 7 xGMI links: TP=8 ~400 GB/s, TP=4 ~200, TP=2 ~70) and 16 link workgroups
O=gpurun_out/r6u; mkdir -p $O
for cfg in "8 400" "4 200" "2 70"; do
  set -- $cfg
  timeout -k 10 400 python tools/emulate_tp_rank.py --tp $1 --steps 2 --warmup 2 --link-gbps $2 --link-cus 16 --sp-streams 2 > $O/tp$1.log 2>&1 || { tail -20 $O/tp$1.log; exit 1; }
  echo "tp$1 link $2: $(grep -o '"ms_per_step": [0-9.]*' $O/tp$1.log) $(grep -o '"link_busy_ms_per_step": [0-9.]*' $O/tp$1.log)"
done
