#!/bin/bash
# Round-4 check on the final tree (layer-0 gather ahead of the weights): GPU suite + smoke + bench.
bash tools/gpu/round_check.sh r4h || exit $?
