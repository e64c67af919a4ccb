#!/bin/bash
# Llama-3-70B, TP=8 x PP over nodes + ZeRO-1 + SP + selective recompute, seq 8192, Lightning
# (reference: examples/training/llama/lightning/run_llama_70b_tp_pp_ptl.sh).  Per node:
#   NNODES=4 NODE_RANK=<r> MASTER_ADDR=<node0> ./run_llama_70b_tp_pp_ptl.sh
# 288 GB of HBM3E per GPU holds a 70B TP=8/PP=4 stage (10 B params/GPU with fp32 master + Adam
# = 160 GB) with room for 8k-token activations.
set -euo pipefail
cd "$(dirname "$0")"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NNODES=${NNODES:-4}
PP=${PP:-$NNODES}
torchrun --nnodes "$NNODES" --node-rank ${NODE_RANK:-0} --nproc-per-node 8 \
    --master-addr ${MASTER_ADDR:-127.0.0.1} --master-port ${MASTER_PORT:-29542} \
    run_llama_nxd_ptl.py --model llama3-70b --tensor_parallel_size 8 --pipeline_parallel_size "$PP" \
    --num_microbatches ${MICROBATCHES:-32} --use_zero1_optimizer 1 --use_sequence_parallel 1 \
    --activation_checkpoint selective --seq_len 8192 --train_batch_size ${BS:-32} --max_steps ${STEPS:-100} \
    --lr 1.5e-4 --min_lr 1.5e-5 --warmup_steps 100 --num_nodes "$NNODES" --data_path "${DATA_PATH:-}" \
    --checkpoint_dir "${CKPT_DIR:-}" --checkpoint_freq ${CKPT_FREQ:-0} "$@"
