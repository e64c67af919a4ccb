#!/bin/bash
# fused attention+o_proj vs split attention (keys per split filling the GPU) below one 1,024-key split
O=gpurun_out/r6h; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_inference_gpu.py tests/test_kernels_gpu.py -k "decode or attn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for p in 128 512; do
    for maxl in 1024 128; do
      NXD_DECODE_ATTN_OPROJ_MAXL=$maxl timeout -k 10 300 python bench_inference.py --prompt $p --new 256 --batch 1 --runs 6 --report $O/r_${p}_${maxl}_$rep.json > $O/b_${p}_${maxl}_$rep.log 2>&1 || { tail -30 $O/b_${p}_${maxl}_$rep.log; exit 1; }
      python -c "import json; r=json.load(open('$O/r_${p}_${maxl}_$rep.json')); print('prompt $p maxl $maxl rep $rep', r['token_generation'])"
    done
  done
done
timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 6 --report $O/report_p2048.json > $O/p2048.log 2>&1 && python -c "import json; r=json.load(open('$O/report_p2048.json')); print('p2048 default', r['token_generation'])"
