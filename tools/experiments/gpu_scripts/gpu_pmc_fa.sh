#!/bin/bash
# PMC counters of the flash-attention forward kernel (one counter pass per run, own process).
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc_fa
cd tools
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d ../gpurun_out/pmc_fa/p1 -o run --output-format csv -- python fa_fwd_ab.py 13 > ../gpurun_out/pmc_fa/p1.log 2>&1
rc=$?; echo "rc=$rc" >> ../gpurun_out/pmc_fa/p1.log; exit $rc
