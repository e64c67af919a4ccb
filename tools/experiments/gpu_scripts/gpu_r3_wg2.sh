#!/bin/bash
set -o pipefail
D=gpurun_out/r3wg2; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_wgrad.py > $D/bench.jsonl 2>&1 || exit $?
for ab in 0 1; do timeout -k 10 120 python tools/prof_wgrad.py 8192 28672 4096 10 $ab >> $D/ablate.jsonl 2>&1 || exit $?; done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $D/p1 -o run --output-format csv -- python tools/prof_wgrad.py 8192 28672 4096 3 0 > $D/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $D/p2 -o run --output-format csv -- python tools/prof_wgrad.py 8192 28672 4096 3 0 > $D/p2.log 2>&1 || exit $?
