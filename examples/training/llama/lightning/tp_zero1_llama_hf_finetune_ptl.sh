#!/bin/bash
# HF Llama instruction fine-tune, TP=8 + ZeRO-1, Lightning (reference:
# examples/training/llama/lightning/tp_zero1_llama2_7b_hf_finetune_ptl.sh).
set -euo pipefail
cd "$(dirname "$0")"
export HSA_ENABLE_IPC_MODE_LEGACY=0
: "${HF_MODEL_DIR:?set HF_MODEL_DIR to a Llama checkpoint directory}"
: "${DATA_FILE:?set DATA_FILE to a JSONL file of instruction/context/response records}"
torchrun --nnodes 1 --nproc-per-node ${GPUS:-8} --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29543} \
    tp_llama_hf_finetune_ptl.py --hf_model_dir "$HF_MODEL_DIR" --data_file "$DATA_FILE" \
    --tensor_parallel_size ${TP:-8} --use_zero_1 --sequence_parallel_enabled --seq_len ${SEQ_LEN:-2048} \
    --batch_size ${BS:-1} --max_steps ${STEPS:-100} --lr ${LR:-5e-6} "$@"
