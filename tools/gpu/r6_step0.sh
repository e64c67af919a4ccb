#!/bin/bash
# Round 6 step 0: serialized whole-step split (one stream, no staggered halves), then the default bench.
O=gpurun_out/r6s0; mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/prof
NXD_BENCH_LADDER=0 NXD_SP_STREAMS=1 NXD_SP_STREAMS_NO_SP=0 timeout -k 10 420 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 2 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T --by-kernel > $O/serial_by_kernel.txt && python tools/step_breakdown.py $T > $O/serial_breakdown.txt
gzip -c $T > $O/serial_kernel_trace.csv.gz; rm -rf $O/prof
head -20 $O/serial_breakdown.txt
tail -2 $O/prof.log
