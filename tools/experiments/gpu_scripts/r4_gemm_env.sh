#!/bin/bash
# Round 4: hipBLASLt stream-K grid knobs on the TP=1 training GEMM shapes (16k tokens), each in a
# fresh process (the in-process autotuner re-picks per setting).
set -o pipefail
O=gpurun_out/r4gemmenv; mkdir -p $O
export TMPDIR=/tmp
for e in "NONE=1" "TENSILE_STREAMK_DYNAMIC_GRID=0" "TENSILE_STREAMK_DYNAMIC_GRID=1" "TENSILE_STREAMK_DYNAMIC_GRID=2" "TENSILE_STREAMK_DYNAMIC_GRID=3" "TENSILE_STREAMK_FULL_TILES=1" "TENSILE_STREAMK_GRID_MULTIPLIER=2" "TENSILE_STREAMK_MAX_CUS=240"; do
  echo "== $e" >> $O/gemm_env.jsonl
  env $e timeout -k 10 200 python -u tools/bench_gemm.py --tp 1 --tokens 16384 >> $O/gemm_env.jsonl 2>> $O/gemm_env.err || exit $?
done
