#!/bin/bash
# FA forward: softmax row sum on the MFMA pipe (MSUM) vs v_add_f32 chain, alternating processes
O=gpurun_out/r6n; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_long_attention_gpu.py tests/test_attention_dropout_gpu.py -k "flash or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for ms in 1 0; do
    NXD_FA_FWD_MSUM=$ms timeout -k 10 300 python tools/bench_fa_fwd_ab.py --root . --tag msum$ms >> $O/ab.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
  done
done
python - <<'PY'
import json,collections,statistics
d=collections.defaultdict(list); e=collections.defaultdict(list)
for l in open('gpurun_out/r6n/ab.jsonl'):
    r=json.loads(l); d[(r['tag'],r['D'],r['H'])].append(r['fwd_ms']); e[(r['tag'],r['D'],r['H'])].append(r['rel_err'])
for k in sorted(d): print(k, round(statistics.median(d[k]),4), max(e[k]))
PY
