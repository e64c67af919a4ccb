#!/bin/bash
# Round 4: decode GEMV k-slices per projection (NXD_DECODE_KS_*), per-kernel times from rocprof.
set -o pipefail
O=gpurun_out/r4dks; mkdir -p $O
export TMPDIR=/tmp
for cfg in "0 0 0" "1 4 1" "2 4 1" "4 4 1" "2 2 1" "2 4 2"; do
  set -- $cfg
  NXD_DECODE_KS_QKV=$1 NXD_DECODE_KS_RESID=$2 NXD_DECODE_KS_GLU=$3 timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report $O/report_$1_$2_$3.json > $O/bench_$1_$2_$3.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/report_$1_$2_$3.json'));print('ks qkv=$1 resid=$2 glu=$3', d['token_generation'])" >> $O/summary.txt
done
