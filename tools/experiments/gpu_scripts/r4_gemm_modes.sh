#!/bin/bash
# Round 4: TP=1 training GEMM shapes (16k tokens = micro-batch 2) under the default top-24 heuristic
# tuning vs the exhaustive validated search (NXD_GEMM_TUNE=2, bounded to 1024 candidates per shape).
set -o pipefail
O=gpurun_out/r4gemm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm.py --tp 1 --tokens 16384 > $O/tune1.jsonl 2> $O/tune1.err || exit $?
NXD_GEMM_TUNE=2 NXD_GEMM_TUNE_MAX_ALGOS=1024 NXD_GEMM_LOG_CHOICE=1 NXD_GEMM_TUNE_FILE=$O/tune2_table.txt timeout -k 10 900 python -u tools/bench_gemm.py --tp 1 --tokens 16384 > $O/tune2.jsonl 2> $O/tune2.err || exit $?
