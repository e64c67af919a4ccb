#!/bin/bash
# GEMM-side cost of SP chunking at the bench's per-TP micro-batch (MBS_BY_TP): TP8/TP4 mbs 4, TP2 mbs 2.
set -o pipefail
O=gpurun_out/r3sp; mkdir -p $O
timeout -k 10 240 python -u tools/bench_sp_chunks.py --tp 8 4 --mbs 4 > $O/sp_chunks_mbs4.jsonl 2>&1 || exit $?
timeout -k 10 240 python -u tools/bench_sp_chunks.py --tp 2 --mbs 2 > $O/sp_chunks_tp2_mbs2.jsonl 2>&1 || exit $?
