#!/bin/bash
# Round 4: emulated-rank stream traces, TP=1 GEMM shapes default vs exhaustive tuning, exhaustive
# mode TP=4 training rehearsal (losses vs the default mode).
set -o pipefail
O=gpurun_out/r4tg; mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/r4_trace.sh || exit $?
timeout -k 10 300 python -u tools/gemm_mode_rehearsal.py > $O/gemm_mode_default.out 2> $O/gemm_mode_default.err || exit $?
NXD_GEMM_TUNE=2 NXD_GEMM_NO_STREAMK=1 timeout -k 10 400 python -u tools/gemm_mode_rehearsal.py > $O/gemm_mode_exh.out 2> $O/gemm_mode_exh.err || exit $?
bash tools/gpu/r4_gemm_modes.sh || exit $?
