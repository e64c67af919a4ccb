#!/bin/bash
# Round 4: fused attention + o_proj with the layer-0 QKV embedding gather issued ahead of the weights, QKV
# GEMV with whole rows per wave.  Decode tests, two bench runs, rocprof kernel stats.
set -o pipefail
O=gpurun_out/r4dec7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py tests/test_spmd_inference_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_$rep.json > $O/bench_$rep.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/report_$rep.json'));print('rep=$rep', d['token_generation'])" >> $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 2 > $O/prof.log 2>&1 || exit $?
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats.csv
find $O/prof -name "*.csv" -delete
cat $O/summary.txt
