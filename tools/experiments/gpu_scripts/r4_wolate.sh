#!/bin/bash
# Round 4: fused decode attention + o_proj, Wo block issued after (default) / before the attention's
# q / K / V loads (NXD_DECODE_WO_LATE=1|0): decode tests, alternating A/B, kernel stats of both.
set -o pipefail
O=gpurun_out/r4wol; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_inference_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do for v in 0 1; do
  NXD_DECODE_WO_LATE=$v timeout -k 10 120 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/r.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  python -c "import json;d=json.load(open('$O/r.json'));print('wo_late=$v rep=$rep', round(d['token_generation']['ms_per_token_p50'],4))" >> $O/summary.txt
done; done
for v in 0 1; do
  NXD_DECODE_WO_LATE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$v -o run --output-format csv -- python bench_inference.py --prompt 128 --new 256 --runs 2 > $O/prof$v.log 2>&1 || exit $?
  S=$(find $O/prof$v -name "run_kernel_stats.csv" | head -1); [ -n "$S" ] && cp $S $O/kernel_stats_wo_late_$v.csv
  find $O/prof$v -name "*.csv" -delete
done
cat $O/summary.txt
