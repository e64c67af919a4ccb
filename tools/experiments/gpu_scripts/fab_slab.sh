#!/bin/bash
# FA backward dK/dV slab mode: numerics tests, then the interleaved A/B.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "flash_bwd" > gpurun_out/fab_slab_tests.log 2>&1 || { tail -30 gpurun_out/fab_slab_tests.log; exit 1; }
tail -2 gpurun_out/fab_slab_tests.log
timeout -k 10 300 python -u tools/bench_fab_slab.py > gpurun_out/fab_slab_ab.jsonl 2>&1 || { tail -20 gpurun_out/fab_slab_ab.jsonl; exit 1; }
cat gpurun_out/fab_slab_ab.jsonl
