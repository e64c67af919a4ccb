#!/bin/bash
# Llama-3.2-1B bs=1 decode: end-to-end report + rocprof kernel stats of one generate.
set -o pipefail
mkdir -p gpurun_out/infer
export TMPDIR=/tmp
P=${NXD_PROMPT:-128}
timeout -k 10 400 python -u -m pytest tests/test_inference_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/infer/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/infer/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_inference.py --prompt $P --new 256 --runs 5 --report gpurun_out/infer/report_p$P.json > gpurun_out/infer/bench_p$P.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/infer/bench_p$P.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/infer/prof -o run --output-format csv -- python bench_inference.py --prompt $P --new 256 --runs 1 --report gpurun_out/infer/prof_report.json > gpurun_out/infer/prof.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/infer/prof.log
exit $rc
