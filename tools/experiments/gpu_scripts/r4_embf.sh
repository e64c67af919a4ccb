#!/bin/bash
# Round 4: embedding gather folded into layer 0's QKV decode launch -- decode GPU tests (exactness
# test included), then alternating A/B NXD_DECODE_EMB_FUSED=0|1 and kernel stats of the fused path.
set -o pipefail
O=gpurun_out/r4embf; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for v in 0 1; do
    NXD_DECODE_EMB_FUSED=$v timeout -k 10 120 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/r.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
    python -c "import json;d=json.load(open('$O/r.json'));print('emb_fused=$v rep=$rep', round(d['token_generation']['ms_per_token_p50'],4))" >> $O/summary.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 2 > $O/prof.log 2>&1 || exit $?
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats.csv
find $O/prof -name "*.csv" -delete
cat $O/summary.txt
