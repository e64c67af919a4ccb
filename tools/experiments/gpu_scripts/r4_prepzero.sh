#!/bin/bash
# Round 4: FA backward dQ-accumulator zeroing in the prep kernel (no memset launch) -- kernel tests,
# then bench A/B (TP=1 halves).
set -o pipefail
O=gpurun_out/r4pz; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_long_attention_gpu.py tests/test_attention_dropout_gpu.py > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for v in 0 1; do
    NXD_FAB_PREP_ZERO=$v timeout -k 10 500 python bench.py --steps 6 --warmup 2 > $O/bench_${v}_${rep}.json 2> $O/bench.err || exit $?
    echo "prep_zero=$v rep=$rep $(tail -n 1 $O/bench_${v}_${rep}.json)" >> $O/summary.txt
  done
done
