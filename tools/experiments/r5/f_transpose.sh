#!/bin/bash
# round 5 F: transpose kernel (ds_read_b64_tr_b16) -- exactness tests, microbench A/B, step-level A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "transpose or swiglu or wgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_transpose.py > $O/transpose_ab.jsonl 2> $O/transpose_ab.err || { tail -20 $O/transpose_ab.err; exit 1; }
cat $O/transpose_ab.jsonl
for i in 1 2; do
  for v in 1 0; do
    NXD_TRANSPOSE_TR=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > $O/b_tr${v}_$i.json 2> $O/b_tr${v}_$i.err || { tail -20 $O/b_tr${v}_$i.err; exit 1; }
    grep -h '^{' $O/b_tr${v}_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('NXD_TRANSPOSE_TR=$v run $i', d['ms_per_step'], d['value'])"
  done
done
