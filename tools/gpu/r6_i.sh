#!/bin/bash
# long-context decode: split attention + (merge + o_proj) launch vs one-pass fused vs split + merge + o_proj
O=gpurun_out/r6i; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_spmd_inference_gpu.py -k "decode or attn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for cfg in "1024 1" "4096 1" "1024 0"; do
    set -- $cfg
    NXD_DECODE_ATTN_OPROJ_MAXL=$1 NXD_DECODE_ATTN_OPROJ=$2 timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 6 --report $O/r_$1_$2_$rep.json > $O/b_$1_$2_$rep.log 2>&1 || { tail -30 $O/b_$1_$2_$rep.log; exit 1; }
    python -c "import json; r=json.load(open('$O/r_$1_$2_$rep.json')); print('maxl $1 fuse $2 rep $rep', r['token_generation'])"
  done
done
