#!/bin/bash
# Two-stream SP halves vs one pass on emulated TP ranks under link models (per-rank ring GB/s).
O=gpurun_out/sts; mkdir -p $O
for cfg in "8 800" "4 200" "4 0" "2 70" "2 0"; do
  set -- $cfg
  for st in 1 2; do
    NXD_SP_STREAMS=$st timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp $1 --steps 2 --warmup 1 --link-gbps $2 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "{\"sp_streams\": $st, \"rec\": $(tail -1 $O/run.log)}" >> $O/emu.jsonl
    tail -1 $O/run.log | cut -c1-40
  done
done
