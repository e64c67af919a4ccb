#!/bin/bash
# Emulated TP=8 rank (full 32-layer Llama-3-8B, GBS 8): dense TN weight-gradient route on / off,
# alternating, then TP=4 once each.
O=gpurun_out/r6emu; mkdir -p $O
for rep in 1 2; do
  for dw in auto 0; do
    NXD_DENSE_WGRAD=$dw timeout -k 10 300 python tools/emulate_tp_rank.py --tp 8 --steps 3 --warmup 2 > $O/tp8_${dw}_$rep.log 2>&1 || { tail -20 $O/tp8_${dw}_$rep.log; exit 1; }
    echo "tp8 dense_wgrad=$dw rep=$rep: $(grep -o '"ms_per_step": [0-9.]*' $O/tp8_${dw}_$rep.log)"
  done
done
for dw in auto 0; do
  NXD_DENSE_WGRAD=$dw timeout -k 10 300 python tools/emulate_tp_rank.py --tp 4 --steps 2 --warmup 2 > $O/tp4_${dw}.log 2>&1 || { tail -20 $O/tp4_${dw}.log; exit 1; }
  echo "tp4 dense_wgrad=$dw: $(grep -o '"ms_per_step": [0-9.]*' $O/tp4_${dw}.log)"
done
