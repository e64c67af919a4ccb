#!/bin/bash
# Decode weight prefetch from spare attention workgroups: numerics tests with it on, then an A/B of
# the gate_up prefetch budget (NXD_DECODE_PREFETCH_MB; 0 = off, 1e-4 = o_proj only), alternating.
set -o pipefail
mkdir -p gpurun_out/pf
export TMPDIR=/tmp
NXD_DECODE_PREFETCH_MB=16 timeout -k 10 400 python -u -m pytest tests/test_inference_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pf/pytest.log; [ $rc -ne 0 ] && exit $rc
for mb in 0 0.0001 16 32 64 0 16 32; do
  NXD_DECODE_PREFETCH_MB=$mb timeout -k 10 300 python bench_inference.py --prompt 128 --new 256 --runs 5 --report gpurun_out/pf/report_mb$mb.json > gpurun_out/pf/bench_mb$mb.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "mb=$mb rc=$rc"; exit $rc; }
  python -c "import json;r=json.load(open('gpurun_out/pf/report_mb$mb.json'));print('mb=$mb', r['token_generation']['ms_per_token_p50'])" >> gpurun_out/pf/ab.txt
done
cat gpurun_out/pf/ab.txt
