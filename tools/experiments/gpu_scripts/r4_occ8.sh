#!/bin/bash
# Round 4: decode GEMVs at 8 waves / SIMD (NXD_DECODE_OCC8) -- decode tests with it on, alternating A/B,
# then rocprof kernel stats of both.
set -o pipefail
O=gpurun_out/r4occ8; mkdir -p $O
export TMPDIR=/tmp
NXD_DECODE_OCC8=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for v in 0 1; do
    NXD_DECODE_OCC8=$v timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_${v}_${rep}.json > $O/bench_${v}_${rep}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('$O/report_${v}_${rep}.json'));print('occ8=$v rep=$rep', d['token_generation'])" >> $O/summary.txt
  done
done
for v in 0 1; do
  NXD_DECODE_OCC8=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 2 > $O/prof$v.log 2>&1 || exit $?
  S=$(find $O/prof$v -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats_occ8_$v.csv
  find $O/prof$v -name "*.csv" -delete
done
