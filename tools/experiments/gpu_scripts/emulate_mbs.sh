#!/bin/bash
# Micro-batch size per TP degree on the emulated rank (full model, GBS 8).
O=gpurun_out/emum; mkdir -p $O
for cfg in "4 4" "4 8" "2 2" "2 4" "4 4" "2 2"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp $1 --mbs $2 --steps 2 --warmup 1 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  tail -1 $O/run.log | tee -a $O/mbs.jsonl
done
