#!/bin/bash
# Round 4: decode / serving GPU tests on the committed tree (after an abort seen with an
# attention phase-trace build), verbose so a failure names its test.
set -o pipefail
O=gpurun_out/r4infc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py tests/test_spmd_inference_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
