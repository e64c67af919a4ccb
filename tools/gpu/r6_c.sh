#!/bin/bash
O=gpurun_out/r6c; mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
for pv in 2 1; do
  NXD_DG_PIPE=$pv timeout -k 10 200 $T tests/test_dense_gemm_gpu.py > $O/tests_p$pv.log 2>&1 || { tail -40 $O/tests_p$pv.log; exit 1; }
  tail -1 $O/tests_p$pv.log
done
timeout -k 10 500 python -u tools/bench_dense_gemm.py --set all --reps 5 --rounds 3 --pipes 1,2 > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.jsonl; exit 1; }
cat $O/bench.jsonl
