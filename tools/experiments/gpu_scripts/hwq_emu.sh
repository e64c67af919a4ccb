#!/bin/bash
# HW queue count vs the emulated TP rank with a link model (false dependencies between streams
# that share a hardware queue).
O=gpurun_out/hwq; mkdir -p $O
for q in 4 8; do
  for cfg in "4 200 2" "4 200 1" "8 400 2" "8 400 1" "8 0 2"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$q NXD_SP_STREAMS=$3 timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp $1 --steps 2 --warmup 1 --link-gbps $2 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "{\"hw_queues\": $q, \"sp_streams\": $3, \"rec\": $(tail -1 $O/run.log)}" >> $O/emu.jsonl
    tail -1 $O/run.log | cut -c1-30
  done
done
