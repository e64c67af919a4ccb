#!/bin/bash
# Round 4: TP=1 halves A/B, FA-backward pricing + PMC, hipBLASLt stream-K env sweep.
bash tools/gpu/r4_tp1_halves.sh || exit $?
bash tools/gpu/r4_fa.sh || exit $?
bash tools/gpu/r4_gemm_env.sh || exit $?
