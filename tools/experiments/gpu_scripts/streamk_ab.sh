#!/bin/bash
# Stream-K exclusion A/B: GEMM slowdown under a side kernel, and the emulated TP=8 rank with / without a link model.
O=gpurun_out/sk; mkdir -p $O
for v in 0 1; do
  NXD_GEMM_NO_STREAMK=$v timeout -k 10 300 python -u tools/bench_cu_interference.py > $O/interf_$v.jsonl 2>&1 || { tail -20 $O/interf_$v.jsonl; exit 1; }
done
for v in 0 1; do
  for bw in "" 400; do
    NXD_GEMM_NO_STREAMK=$v timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp 8 --steps 2 --warmup 1 ${bw:+--link-gbps $bw} > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "{\"no_streamk\": $v, \"rec\": $(tail -1 $O/run.log)}" | tee -a $O/emu.jsonl
  done
done
