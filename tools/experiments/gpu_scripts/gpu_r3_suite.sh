#!/bin/bash
# Full GPU test suite on the current tree (what the driver runs at round end).
set -o pipefail
O=gpurun_out/r3suite; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; exit $rc
