#!/bin/bash
# FA forward: packed-math softmax + buffer-unrolled tile loop (immediate-offset V reads) vs HEAD build
O=gpurun_out/r6j; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_long_attention_gpu.py tests/test_attention_dropout_gpu.py -k "flash or fa_ or attn or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 300 python tools/bench_fa_fwd_ab.py --root abhead --tag head >> $O/ab.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
  timeout -k 10 300 python tools/bench_fa_fwd_ab.py --root . --tag new >> $O/ab.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
  NXD_FA_FWD_PK=0 timeout -k 10 300 python tools/bench_fa_fwd_ab.py --root . --tag new_nopk >> $O/ab.jsonl 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
done
cat $O/ab.jsonl
