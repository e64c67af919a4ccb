#!/bin/bash
O=gpurun_out/r6dg2; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gemm_gpu.py > $O/test_p1.log 2>&1 || { tail -40 $O/test_p1.log; exit 1; }
NXD_DG_PIPE=0 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gemm_gpu.py > $O/test_p0.log 2>&1 || { tail -40 $O/test_p0.log; exit 1; }
tail -1 $O/test_p1.log $O/test_p0.log
timeout -k 10 400 python -u tools/bench_dense_gemm.py --set tp1 --reps 5 --rounds 3 --pipes 0,1 --shapes qkv,o_proj,gate_up,down > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.jsonl; exit 1; }
cat $O/bench.jsonl
