#!/bin/bash
# Round 4: RMSNorm backward with the next row's loads in flight -- kernel tests, microbench A/B,
# then alternating 1-GPU bench A/B (NXD_RMS_BWD_PIPE=0|1).
set -o pipefail
O=gpurun_out/r4rms; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k rmsnorm > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for v in 0 1; do
  NXD_RMS_BWD_PIPE=$v timeout -k 10 120 python tools/bench_rmsnorm_bwd.py >> $O/micro.jsonl 2>> $O/micro.err || exit $?
done; done
cat $O/micro.jsonl
for rep in 1 2; do for v in 0 1; do
  NXD_RMS_BWD_PIPE=$v timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('pipe=$v rep=$rep', d['ms_per_step'], d['value'], d['loss'])" >> $O/summary.txt
done; done
cat $O/summary.txt
