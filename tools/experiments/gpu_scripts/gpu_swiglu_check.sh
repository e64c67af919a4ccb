set -o pipefail
mkdir -p gpurun_out/sw
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k swiglu --timeout 120 --timeout-method thread > gpurun_out/sw/t.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_kernels.py --only mem > gpurun_out/sw/mem.log 2>&1
