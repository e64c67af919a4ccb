#!/bin/bash
# PMC counters of the flash-attention backward kernel (own runs: --pmc only with kernel-trace)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python3 $R/tools/fa_bwd_once.py > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> $R/gpurun_out/pmc/status.txt
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
