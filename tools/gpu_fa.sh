#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -rf -k "flash or rope_attention" > gpurun_out/fa_t.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/fa_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_kernels.py --only fa > gpurun_out/fa_b.log 2>&1
echo "bench rc=$?" >> gpurun_out/fa_b.log
