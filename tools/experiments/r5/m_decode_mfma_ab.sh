#!/bin/bash
# round 5 M: decode GEMVs at M >= 2 rows on MFMA (dmm_kernel) vs the VALU dot2 body, batch 1 / 2 / 4 / 8
# (Llama-3.2-1B, prompt 128, 128 new tokens, hipGraphs); one process per variant, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name bs env...
  local name=$1 bs=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench_inference.py --prompt 128 --new 128 --batch $bs --runs 3 --report $O/r_${name}_bs$bs.json > $O/${name}_bs$bs.log 2>&1 || { tail -20 $O/${name}_bs$bs.log; exit 1; }
  python -c "import json;r=json.load(open('$O/r_${name}_bs$bs.json'));t=r['token_generation'];print(json.dumps({'variant':'$name','batch':$bs,'ms_per_step':round(t['ms_per_token_p50'],4),'tokens_per_s':round($bs*t['tokens_per_s_per_seq'],1)}))" | tee -a $O/ab.jsonl
}
for rep in 1 2; do
  for bs in 2 4 8; do
    run valu_dot2 $bs NXD_DECODE_MFMA=0
    run mfma $bs NXD_DECODE_MFMA=2
  done
done
true
