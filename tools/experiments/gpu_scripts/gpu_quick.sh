#!/bin/bash
# One short GPU call: selected GPU tests (pytest -k expression in $1).
set -o pipefail
mkdir -p gpurun_out/quick
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$1" > gpurun_out/quick/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/quick/pytest.log
exit $rc
