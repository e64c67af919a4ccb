#!/bin/bash
O=gpurun_out/r6d; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_dense_gemm_gpu.py tests/test_wgrad_gemm_gpu.py tests/test_shard_grad_parity_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | cut -c1-400
