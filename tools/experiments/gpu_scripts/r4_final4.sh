#!/bin/bash
# Round-4 check on the tree with the round-4 decode GEMV changes: GPU suite + smoke + 1-GPU bench.
bash tools/gpu/round_check.sh r4e || exit $?
