#!/bin/bash
# end of round 6: 1-GPU bench at 10 timed steps, emulated TP ranks (8 / 4 / 2) on the final tree
O=gpurun_out/r6fb; mkdir -p $O
timeout -k 10 900 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | tail -1
for tp in 8 4 2; do
  timeout -k 10 400 python tools/emulate_tp_rank.py --tp $tp --steps 2 --warmup 2 > $O/tp$tp.log 2>&1 || { tail -20 $O/tp$tp.log; exit 1; }
  echo "tp$tp: $(grep -o '"ms_per_step": [0-9.]*' $O/tp$tp.log) $(grep -o '"node_tokens_per_s_comm_free": [0-9.]*' $O/tp$tp.log)"
done
