#!/bin/bash
# Persistent (stream-K) GEMMs vs a concurrent collective: emulated TP ranks with a link model, NXD_GEMM_NO_STREAMK 0 / 1.
O=gpurun_out/nsk; mkdir -p $O
for cfg in "4 200" "8 400" "4 0" "8 0"; do
  set -- $cfg
  for v in 0 1; do
    NXD_GEMM_LOG_CHOICE=1 NXD_GEMM_NO_STREAMK=$v timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp $1 --steps 2 --warmup 1 --link-gbps $2 > $O/run.log 2> $O/choices_tp$1_$v.txt || { tail -20 $O/choices_tp$1_$v.txt; exit 1; }
    echo "{\"no_streamk\": $v, \"rec\": $(tail -1 $O/run.log)}" >> $O/emu.jsonl
    tail -1 $O/run.log | cut -c1-40
  done
done
