#!/bin/bash
# Collect the GEMM keys of a Llama-3-8B training step at TP=1/2/4/8 (gloo, all ranks on cuda:0)
# and tune them exhaustively into the shipped table.
set -o pipefail
mkdir -p gpurun_out/tune
OUT=gpurun_out/tune
export OMP_NUM_THREADS=2
rm -f $OUT/keys.txt
for tp in ${TUNE_TPS:-1 2 4 8}; do
  if [ $tp -eq 1 ]; then
    NXD_GEMM_TUNE=0 NXD_GEMM_LOG_KEYS=$OUT/keys.txt timeout -k 10 300 python tools/collect_gemm_keys.py --tp 1 >> $OUT/collect.log 2>&1 || exit $?
  else
    NXD_GEMM_TUNE=0 NXD_GEMM_LOG_KEYS=$OUT/keys.txt timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $tp \
      --master-addr 127.0.0.1 --master-port 2960$tp tools/collect_gemm_keys.py --tp $tp >> $OUT/collect.log 2>&1 || exit $?
  fi
  echo "tp=$tp keys so far: $(sort -u $OUT/keys.txt | wc -l)"
done
sort -u $OUT/keys.txt > $OUT/keys_uniq.txt
timeout -k 10 ${TUNE_SECONDS:-900} python tools/tune_gemm.py --keys $OUT/keys_uniq.txt --out $OUT/table.txt
