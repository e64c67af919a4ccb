#!/bin/bash
# Round-4 check on the final tree (o_proj block ordering in the fused decode attention): GPU suite + smoke + bench.
bash tools/gpu/round_check.sh r4g || exit $?
