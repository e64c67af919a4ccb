#!/bin/bash
# Llama-2-7B 8-layer long-sequence config at 8k: dense TN wgrad route on / off, FA forward default, alternating
O=gpurun_out/r6r; mkdir -p $O
for rep in 1 2; do
  for dw in auto 0; do
    NXD_DENSE_WGRAD=$dw timeout -k 10 300 python tools/bench_long_seqlen.py --seqs 8192 > $O/ls_${dw}_$rep.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
    echo "dense_wgrad=$dw rep $rep: $(grep -o '"seq_per_s": [0-9.]*' $O/ls_${dw}_$rep.jsonl)"
  done
done
