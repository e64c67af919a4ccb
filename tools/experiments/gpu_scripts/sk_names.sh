#!/bin/bash
O=gpurun_out/sk2; mkdir -p $O
for v in 0 1; do
  NXD_GEMM_LOG_CHOICE=1 NXD_GEMM_NO_STREAMK=$v timeout -k 10 300 python -u tools/bench_cu_interference.py > $O/interf_$v.jsonl 2> $O/choices_$v.txt || { tail -20 $O/choices_$v.txt; exit 1; }
done
cat $O/choices_0.txt $O/choices_1.txt | grep "nxd gemm" | cut -c1-250
