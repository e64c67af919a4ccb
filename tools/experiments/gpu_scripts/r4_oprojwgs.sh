#!/bin/bash
# Round 4: o_proj workgroup target of the fused decode attention launch with the late Wo loads
# (NXD_DECODE_OPROJ_WGS = 256 default / 512 / 1024), alternating.
set -o pipefail
O=gpurun_out/r4owg; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do for v in 256 512 1024; do
  NXD_DECODE_OPROJ_WGS=$v timeout -k 10 120 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/r.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  python -c "import json;d=json.load(open('$O/r.json'));print('oproj_wgs=$v rep=$rep', round(d['token_generation']['ms_per_token_p50'],4))" >> $O/summary.txt
done; done
cat $O/summary.txt
