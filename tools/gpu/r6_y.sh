#!/bin/bash
# 1-GPU bench knob A/B on the final tree: stream-K excluded, dense TN wgrad route off, vs defaults (alternating)
O=gpurun_out/r6y; mkdir -p $O
for rep in 1 2; do
  for cfg in "default NXD_X=0" "nosk NXD_GEMM_NO_STREAMK=1" "dw0 NXD_DENSE_WGRAD=0"; do
    set -- $cfg
    env $2 timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $O/$1_$rep.log 2>&1 || { tail -20 $O/$1_$rep.log; exit 1; }
    echo "$1 rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $O/$1_$rep.log | tail -1)"
  done
done
