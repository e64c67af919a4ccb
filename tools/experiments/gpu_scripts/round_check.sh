#!/bin/bash
# GPU round check: full GPU suite, smoke, short 1-GPU bench.  Output under gpurun_out/.
mkdir -p gpurun_out
tag=${1:-r3b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
echo rc=$rc >> gpurun_out/${tag}_gpu_tests.log
tail -3 gpurun_out/${tag}_gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_smoke.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/${tag}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_bench.log
