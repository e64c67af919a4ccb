#!/bin/bash
O=gpurun_out/nsk2; mkdir -p $O
for cfg in "4 200 1" "4 200 0" "8 400 1" "8 0 1" "4 0 1"; do
  set -- $cfg
  NXD_GEMM_LOG_CHOICE=1 NXD_GEMM_NO_STREAMK=$3 timeout -k 10 400 python -u tools/emulate_tp_rank.py --tp $1 --steps 2 --warmup 1 --link-gbps $2 > $O/run.log 2> $O/choices_$1_$2_$3.txt || { tail -20 $O/choices_$1_$2_$3.txt; exit 1; }
  echo "{\"no_streamk\": $3, \"rec\": $(tail -1 $O/run.log)}" >> $O/emu.jsonl
  tail -1 $O/run.log | cut -c1-30
done
