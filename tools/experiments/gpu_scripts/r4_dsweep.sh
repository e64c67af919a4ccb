#!/bin/bash
# Round 4: decode launch-shape sweep on the refactored GEMVs (Llama-3.2-1B bs=1), alternating with
# the default in each repetition: QKV / down / gate_up k-slices, gate_up row pairs per wave,
# attention + o_proj workgroup target.
set -o pipefail
O=gpurun_out/r4dsw; mkdir -p $O
export TMPDIR=/tmp
VARS="base NXD_DECODE_KS_QKV=1 NXD_DECODE_KS_QKV=4 NXD_DECODE_GLU_PAIRS=2 NXD_DECODE_KS_GLU=2 NXD_DECODE_KS_RESID=2 NXD_DECODE_OPROJ_WGS=512 NXD_DECODE_OPROJ_WGS=128"
for rep in 1 2; do
  for v in $VARS; do
    if [ "$v" = base ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 120 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/r.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
    python -c "import json;d=json.load(open('$O/r.json'));print('$v rep=$rep', round(d['token_generation']['ms_per_token_p50'],4))" >> $O/summary.txt
  done
done
cat $O/summary.txt
