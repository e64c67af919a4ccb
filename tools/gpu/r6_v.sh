#!/bin/bash
# TP=8 emulated rank with the link model: SP parts / stagger sweep on the final tree
O=gpurun_out/r6v; mkdir -p $O
for cfg in "2 2" "2 1" "2 3" "4 2" "4 3"; do
  set -- $cfg
  timeout -k 10 400 python tools/emulate_tp_rank.py --tp 8 --steps 2 --warmup 2 --link-gbps 400 --link-cus 16 --sp-streams $1 --sp-stagger $2 > $O/s$1_g$2.log 2>&1 || { tail -20 $O/s$1_g$2.log; exit 1; }
  echo "streams $1 stagger $2: $(grep -o '"ms_per_step": [0-9.]*' $O/s$1_g$2.log)"
done
