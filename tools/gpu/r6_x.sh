#!/bin/bash
# 1-GPU bench: weight gradients as bf16-output GEMMs + fp32 add (NXD_WGRAD_BF16=1) vs fp32-output, alternating
O=gpurun_out/r6x; mkdir -p $O
for rep in 1 2; do
  for wb in 1 0; do
    NXD_WGRAD_BF16=$wb timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $O/b_${wb}_$rep.log 2>&1 || { tail -20 $O/b_${wb}_$rep.log; exit 1; }
    echo "wgrad_bf16=$wb rep $rep: $(grep -o '"ms_per_step": [0-9.]*' $O/b_${wb}_$rep.log | tail -1) $(grep -o '"loss": [0-9.]*' $O/b_${wb}_$rep.log | tail -1)"
  done
done
