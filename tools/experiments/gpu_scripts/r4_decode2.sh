#!/bin/bash
# Round 4: persistent decode GEMV (bit-exactness test + A/B) and per-projection k-slices.
set -o pipefail
O=gpurun_out/r4dec2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_inference_gpu.py -k "persistent or fused_decode_matches or graph_decode" > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for n in 0 1 2 4; do
    NXD_DECODE_PERSIST=$n timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_p${n}_${rep}.json > $O/bench_p${n}_${rep}.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('$O/report_p${n}_${rep}.json'));print('persist=$n rep=$rep', d['token_generation'])" >> $O/summary.txt
  done
done
bash tools/gpu/r4_decode_ks.sh || exit $?
