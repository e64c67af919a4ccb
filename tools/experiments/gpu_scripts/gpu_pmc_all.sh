#!/bin/bash
# PMC counters of every hand-written kernel (tools/pmc_kernels.py): one rocprofv3 run per counter
# pass (capacity limits: <= 8 SQ, <= 4 TCC), plus one kernel-trace run for durations.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_all
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python tools/pmc_kernels.py > $O/trace.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $O/p1 -o run -- python tools/pmc_kernels.py > $O/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p2 -o run -- python tools/pmc_kernels.py > $O/p2.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p3 -o run -- python tools/pmc_kernels.py > $O/p3.log 2>&1 || exit $?
python tools/pmc_summary.py $O/summary.md $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) $(ls $O/p1/*/run_counter_collection.csv $O/p1/run_counter_collection.csv $O/p2/*/run_counter_collection.csv $O/p2/run_counter_collection.csv $O/p3/*/run_counter_collection.csv $O/p3/run_counter_collection.csv 2>/dev/null) > $O/summary.log 2>&1
echo "summary rc=$?"
