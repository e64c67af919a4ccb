#!/bin/bash
# Llama-3-8B pre-training, TP=8 + sequence parallel + ZeRO-1, seq 8192, on one 8x MI355X node
# (reference: examples/training/llama/tp_zero1_llama_hf_pretrain/tp_zero1_llama3_8B_hf_pretrain.sh).
# DATA: a flat uint32 token file (native loader) or a packed HF dataset dir; unset = synthetic tokens.
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
NPROC=${NPROC:-8}
TP=${TP:-8}
DIR=$(cd "$(dirname "$0")" && pwd)
torchrun --nproc-per-node $NPROC --master-addr 127.0.0.1 --master-port ${PORT:-29500} \
    $DIR/tp_zero1_llama_hf_pretrain.py --model_path ${MODEL:-llama3-8b} --tensor_parallel_size $TP \
    --seq_len ${SEQ_LEN:-8192} --batch_size 1 --grad_accum_usteps ${GRAD_ACCUM:-8} --max_steps ${STEPS:-1000} \
    --use_zero_1 --sequence_parallel_enabled --lr 1.5e-4 --min_lr 1e-5 --warmup_steps 100 \
    --checkpoint_dir ${CKPT_DIR:-ckpt} --checkpoint_freq ${CKPT_FREQ:-500} --async_checkpoint_saving \
    ${DATA:+--data_dir $DATA} "$@"
