#!/bin/bash
# PMC counters of the grouped-GEMM kernels: one rocprofv3 pass per counter group.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ggpmc; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o run -- python tools/pmc_grouped_gemm.py > $O/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE --output-format csv -d $O/p2 -o run -- python tools/pmc_grouped_gemm.py > $O/p2.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python tools/pmc_grouped_gemm.py > $O/p3.log 2>&1 || exit $?
