#!/bin/bash
# whole-step kernel trace of the default bench configuration (two staggered halves on two streams)
O=gpurun_out/r6sd; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/prof
NXD_BENCH_LADDER=0 timeout -k 10 420 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 2 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T --by-kernel > $O/by_kernel.txt && python tools/step_breakdown.py $T > $O/breakdown.txt
rm -rf $O/prof
head -16 $O/breakdown.txt
grep '"metric"' $O/prof.log | tail -1 | cut -c1-200
