#!/bin/bash
# Heuristic-filter stream-K exclusion under the link model, SP halves on (bench settings).
O=gpurun_out/nsk3; mkdir -p $O
for cfg in "8 400 0" "8 400 1" "4 200 0" "4 200 1" "8 0 0" "8 0 1"; do
  set -- $cfg
  NXD_SP_STREAMS=2 NXD_GEMM_NO_STREAMK=$3 timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp $1 --steps 2 --warmup 1 --link-gbps $2 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  echo "{\"no_streamk\": $3, \"rec\": $(tail -1 $O/run.log)}" >> $O/emu.jsonl
done
