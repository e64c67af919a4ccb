#!/bin/bash
# round 5 A: row-per-wave RMSNorm (tests + microbench), fused-decode embedding zero rows + phase trace,
# exhaustive GEMM check, MoE prefill, then the 1-GPU bench through the fallback ladder, then the
# convergence curves
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5a
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k rmsnorm > gpurun_out/r5a/pytest_rms.log 2>&1 || { tail -30 gpurun_out/r5a/pytest_rms.log; exit 1; }
tail -2 gpurun_out/r5a/pytest_rms.log
timeout -k 10 900 $PYT tests/test_inference_gpu.py tests/test_spmd_inference_gpu.py tests/test_gemm_exhaustive_gpu.py \
  tests/test_moe_gpu.py > gpurun_out/r5a/pytest.log 2>&1 || { tail -30 gpurun_out/r5a/pytest.log; exit 1; }
tail -2 gpurun_out/r5a/pytest.log
timeout -k 10 300 python -u tools/bench_rmsnorm.py > gpurun_out/r5a/rmsnorm_ab.jsonl 2>gpurun_out/r5a/rmsnorm_ab.err || exit 1
cat gpurun_out/r5a/rmsnorm_ab.jsonl
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || { tail -30 gpurun_out/r5a/bench.err; exit 1; }
cat gpurun_out/r5a/bench.json
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_convergence_gpu.py \
  > gpurun_out/r5a/convergence.log 2>&1 || { tail -30 gpurun_out/r5a/convergence.log; exit 1; }
grep -E "within rtol|passed|failed" gpurun_out/r5a/convergence.log
