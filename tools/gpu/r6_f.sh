#!/bin/bash
# decode at the notebook config: fused attention + o_proj past one key split (A/B vs the split path)
O=gpurun_out/r6f; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_inference_gpu.py -k "fused_attention_oproj or fused_decode_matches" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for maxl in 4096 1024; do
    NXD_DECODE_ATTN_OPROJ_MAXL=$maxl timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 6 --report $O/r_${maxl}_$rep.json > $O/b_${maxl}_$rep.log 2>&1 || { tail -30 $O/b_${maxl}_$rep.log; exit 1; }
    python -c "import json; r=json.load(open('$O/r_${maxl}_$rep.json')); print('maxl $maxl rep $rep', r['token_generation'])"
  done
done
