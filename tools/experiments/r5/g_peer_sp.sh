#!/bin/bash
# round 5 G: peer sequence-parallel collectives (unit + TP=2/4 training parity on one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g
mkdir -p $O
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"


timeout -k 10 900 $PYT tests/test_bench_gpu.py -k "peer" > $O/pytest_bench.log 2>&1 || { tail -40 $O/pytest_bench.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest_bench.log
