#!/bin/bash
# round-6 PMC table of the hand-written kernels (tools/pmc_kernels.py workload), one counter set per run
O=gpurun_out/r6pmck; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf $O/p$i
  timeout -s KILL 150 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python tools/pmc_kernels.py > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python tools/pmc_avg.py $O/p1 $O/p2 $O/p3 $O/p4 > $O/summary.txt 2>&1 || true
rm -rf $O/p1 $O/p2 $O/p3 $O/p4
grep -E "^[a-zA-Z_].*|MFMA busy|FETCH_SIZE|WRITE_SIZE" $O/summary.txt | head -60
