#!/bin/bash
# One GPU call: kernel/numerics tests, smoke, 1-GPU bench, rocprof kernel stats of a short bench.
set -o pipefail
mkdir -p gpurun_out/round
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/round/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/round/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/round/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/round/bench1.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/round/bench1.log; [ $rc -ne 0 ] && exit $rc
if [ "${NXD_PROF:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/round/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > gpurun_out/round/prof.log 2>&1
  rc=$?; echo "prof rc=$rc" >> gpurun_out/round/prof.log
fi
exit $rc
