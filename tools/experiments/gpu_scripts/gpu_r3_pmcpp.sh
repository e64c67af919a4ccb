#!/bin/bash
# PMC passes of the ping-pong grouped kernels + the wgrad dispatch test + long-sequence bench (the
# reference's only published throughput config).
set -o pipefail
D=gpurun_out/r3pmcpp; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_wgrad.log 2>&1 || exit $?
for m in 0 1 2; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $D/m${m}_p1 -o run --output-format csv -- python tools/prof_grouped.py $m 3 > $D/m${m}_p1.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $D/m${m}_p2 -o run --output-format csv -- python tools/prof_grouped.py $m 3 > $D/m${m}_p2.log 2>&1 || exit $?
done
timeout -k 10 900 python -u tools/bench_long_seqlen.py > $D/long_seqlen.jsonl 2> $D/long_seqlen.err || exit $?
