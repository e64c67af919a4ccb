#!/bin/bash
# gloo-staged pipeline p2p: multi-rank rehearsal tests, then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/ppfix
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ppfix/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ppfix/pytest_gpu.log
exit $rc
