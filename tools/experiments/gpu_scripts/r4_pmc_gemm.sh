#!/bin/bash
# Round 4: readable MFMA-busy % (MFMA busy cycles and GPU-active clock from ONE pass) for the
# hand-written weight-gradient kernel (TP=8 shapes at mbs 8 and the TP=1 gate_up half) and the
# grouped MoE kernels (Mixtral gate_up: fwd / dgrad / wgrad).  One rocprofv3 --pmc pass per program.
set -o pipefail
O=gpurun_out/r4pmc; mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
cd /tmp
run() {  # tag, program args...
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR -d $R/$O/$tag -o run --output-format csv -- python3 "$@" > $R/$O/$tag.log 2>&1 || return $?
  local C=$(find $R/$O/$tag -name "*counter_collection.csv" | head -1)
  echo "== $tag: $(tail -1 $R/$O/$tag.log)" >> $R/$O/pmc.txt
  python3 $R/tools/pmc_table.py $C "$KPAT" >> $R/$O/pmc.txt || return $?
  find $R/$O/$tag -name "*.csv" -delete
}
KPAT=wgrad_kernel
run wg_tp8_qkv $R/tools/prof_wgrad.py 65536 768 4096 5 || exit $?
run wg_tp8_o $R/tools/prof_wgrad.py 65536 4096 512 5 || exit $?
run wg_tp8_gateup $R/tools/prof_wgrad.py 65536 3584 4096 5 || exit $?
run wg_tp8_down $R/tools/prof_wgrad.py 65536 4096 1792 5 || exit $?
run wg_tp1_gateup $R/tools/prof_wgrad.py 8192 28672 4096 5 || exit $?
KPAT=""
run grouped_fwd $R/tools/prof_grouped.py 0 3 || exit $?
run grouped_dgrad $R/tools/prof_grouped.py 1 3 || exit $?
run grouped_wgrad $R/tools/prof_grouped.py 2 3 || exit $?
cat $R/$O/pmc.txt | grep -E "^==|MFMA busy|conflict share|^[a-zA-Z_]"
