#!/bin/bash
# notebook-config decode: one-pass fused attention + o_proj with fewer row chunks per kv head (less
# redundant KV traffic) vs the default split attention + merge-in-o_proj
O=gpurun_out/r6o; mkdir -p $O
for rep in 1 2; do
  for cfg in "1024 256" "4096 32" "4096 64" "4096 128"; do
    set -- $cfg
    NXD_DECODE_ATTN_OPROJ_MAXL=$1 NXD_DECODE_OPROJ_WGS=$2 timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 4 --report $O/r_$1_$2_$rep.json > $O/b_$1_$2_$rep.log 2>&1 || { tail -30 $O/b_$1_$2_$rep.log; exit 1; }
    python -c "import json; r=json.load(open('$O/r_$1_$2_$rep.json')); print('maxl $1 oproj_wgs $2 rep $rep', round(r['token_generation']['ms_per_token_p50'],4))"
  done
done
