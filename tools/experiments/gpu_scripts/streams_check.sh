#!/bin/bash
# Two-stream SP halves: GPU parity tests, then the emulated TP=8 rank with / without a link model.
O=gpurun_out/st; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_parallel_gpu.py tests/test_emulate_tp.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for st in 1 2; do
  for bw in 0 400; do
    NXD_SP_STREAMS=$st timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp 8 --steps 2 --warmup 1 --link-gbps $bw > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "{\"sp_streams\": $st, \"rec\": $(tail -1 $O/run.log)}" | tee -a $O/emu.jsonl | cut -c1-60
  done
done
