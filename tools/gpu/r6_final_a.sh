#!/bin/bash
# smoke, default 1-GPU bench, notebook-config decode kernel stats, FA forward PMC (one counter set per run)
O=gpurun_out/r6fa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | tail -1
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 2 --report $O/report_prof.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $S $O/kernel_stats_p2048.csv; rm -rf $O/prof
head -10 $O/kernel_stats_p2048.csv | cut -c1-160
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf $O/p$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python tools/bench_fa_fwd_ab.py --reps 2 --rounds 1 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python tools/pmc_avg.py $O/p1 $O/p2 > $O/fa_pmc.txt 2>&1 || true
grep -A30 "fa::fwd_kernel" $O/fa_pmc.txt | grep -E "fwd_kernel|MFMA busy|WAIT_ANY/|ACTIVE_INST" | head -20
rm -rf $O/p1 $O/p2
