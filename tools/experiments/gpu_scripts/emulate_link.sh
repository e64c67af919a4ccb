#!/bin/bash
# TP=8 rank with a link-time model: SP chunk count vs per-rank ring bandwidth.
O=gpurun_out/emul; mkdir -p $O
run() {
  NXD_SP_CHUNKS=$1 timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp 8 --steps 2 --warmup 1 ${2:+--link-gbps $2} > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  tail -1 $O/run.log | tee -a $O/link.jsonl
}
for bw in 250 400 600; do
  for c in 2 4 8; do run $c $bw; done
done
run 4 ""
