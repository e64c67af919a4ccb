#!/bin/bash
# decode attention V tile swizzle: decode tests, then alternating A/B against the HEAD build (abhead/)
O=gpurun_out/r6q; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_inference_gpu.py tests/test_kernels_gpu.py -k "decode or attn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for p in 128 2048; do
    for v in head new; do
      S=bench_inference.py; [ $v = head ] && S=abhead/bench_inference.py
      timeout -k 10 300 python $S --prompt $p --new 256 --batch 1 --runs 4 --report $O/r_${v}_${p}_$rep.json > $O/b_${v}_${p}_$rep.log 2>&1 || { tail -30 $O/b_${v}_${p}_$rep.log; exit 1; }
      python -c "import json; r=json.load(open('$O/r_${v}_${p}_$rep.json')); print('$v p$p rep $rep', round(r['token_generation']['ms_per_token_p50'],4))"
    done
  done
done
