#!/bin/bash
# Kernel durations of the emulated TP=8 rank with and without the link model (which kernels stretch).
O=gpurun_out/emulp; mkdir -p $O
export TMPDIR=/tmp
for bw in 0 400; do
  rm -rf $O/prof$bw
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof$bw -o run --output-format csv -- python tools/emulate_tp_rank.py --tp 8 --steps 1 --warmup 1 --link-gbps $bw > $O/prof$bw.log 2>&1 || { tail -20 $O/prof$bw.log; exit 1; }
  T=$(find $O/prof$bw -name "run_kernel_trace.csv" | head -1)
  python tools/step_breakdown.py $T --by-kernel > $O/by_kernel_$bw.txt && python tools/step_breakdown.py $T > $O/breakdown_$bw.txt && rm -f $T
  head -14 $O/breakdown_$bw.txt
done
