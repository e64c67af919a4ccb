#!/bin/bash
# Alternating same-box A/B of one env knob on the 1-GPU bench: bench_ab_env.sh VAR A B [rounds] [steps]
mkdir -p gpurun_out
var=$1; a=$2; b=$3; rounds=${4:-2}; steps=${5:-5}
out=gpurun_out/ab_${var}.txt
: > $out
for i in $(seq 1 $rounds); do
  for v in $a $b; do
    env $var=$v timeout -k 10 400 python bench.py --steps $steps --warmup 2 > gpurun_out/ab_tmp.log 2>&1 || { tail -5 gpurun_out/ab_tmp.log; exit 1; }
    echo "$var=$v $(tail -1 gpurun_out/ab_tmp.log)" | tee -a $out
  done
done
