#!/bin/bash
# PMC passes over the dense GEMM workload (one counter set per run)
O=gpurun_out/r6pmc; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf $O/p$i
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python tools/pmc_dense_gemm.py $@ > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python tools/pmc_avg.py $O/p1 $O/p2 > $O/summary.txt 2>&1 || true
cat $O/summary.txt | head -80
