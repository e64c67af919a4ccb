#!/bin/bash
O=gpurun_out/r6b; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_dense_gemm_gpu.py tests/test_peer_allreduce_gpu.py "tests/test_kernels_gpu.py::test_rmsnorm_rows_path_vs_fp32" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
H=8192 timeout -k 10 200 python -u tools/bench_rmsnorm.py > $O/rms8192.jsonl 2>&1 || { tail -20 $O/rms8192.jsonl; exit 1; }
cat $O/rms8192.jsonl
timeout -k 10 400 python -u tools/bench_dense_gemm.py --set tp1 --reps 5 --rounds 3 --pipes 0,1 --shapes qkv,o_proj,gate_up,down > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.jsonl; exit 1; }
cat $O/bench.jsonl
