#!/bin/bash
# Llama-2-7B, TP=8 + ZeRO-1 + SP, seq 4096, Lightning on one 8-GPU MI355X node
# (reference: examples/training/llama/lightning/run_llama_7b_tp_ptl.sh).
set -euo pipefail
cd "$(dirname "$0")"
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPUS=${GPUS:-8}
TP=${TP:-8}
torchrun --nnodes 1 --nproc-per-node "$GPUS" --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29541} \
    run_llama_nxd_ptl.py --model llama2-7b --tensor_parallel_size "$TP" --use_zero1_optimizer 1 \
    --use_sequence_parallel 1 --seq_len 4096 --train_batch_size ${BS:-1} --grad_accum_usteps ${ACC:-8} \
    --max_steps ${STEPS:-100} --warmup_steps 10 --lr 3e-4 --data_path "${DATA_PATH:-}" \
    --checkpoint_dir "${CKPT_DIR:-}" --checkpoint_freq ${CKPT_FREQ:-0} "$@"
