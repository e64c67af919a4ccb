#!/bin/bash
# round 5 I: the whole GPU suite with per-test durations (suite-time budget), then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=60 > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
