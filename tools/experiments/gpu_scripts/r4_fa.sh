#!/bin/bash
# Round 4: flash-attention backward -- ablations + the atomic-free dQ (slab + reduce) price, and
# one PMC pass with MFMA busy and the GPU-active clock in the same run (readable MFMA-busy %).
set -o pipefail
O=gpurun_out/r4fa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_fa_ablate.py > $O/ablate.jsonl 2> $O/ablate.err || exit $?
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $R/$O/pmc -o run --output-format csv -- python3 $R/tools/fa_bwd_once.py > $R/$O/pmc.log 2>&1 || exit $?
cd $R
C=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python tools/pmc_table.py $C bwd_kernel > $O/pmc_fab.txt || exit $?
python tools/pmc_table.py $C fwd_kernel > $O/pmc_faf.txt || exit $?
find $O/pmc -name "*.csv" -delete
