#!/bin/bash
O=gpurun_out/r6dg; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dense_gemm_gpu.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 400 python -u tools/bench_dense_gemm.py --set all --reps 5 --rounds 3 > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.jsonl; exit 1; }
cat $O/bench.jsonl
