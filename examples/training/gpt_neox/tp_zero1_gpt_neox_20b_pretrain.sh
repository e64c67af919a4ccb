#!/bin/bash
# GPT-NeoX-20B (or MODEL=pythia-6.9b) pre-training, TP=8 + ZeRO-1 on one 8x MI355X node
# (reference: examples/training/tp_dp_gpt_neox_hf_pretrain/tp_dp_gpt_neox_20b_hf_pretrain/).
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
DIR=$(cd "$(dirname "$0")" && pwd)
torchrun --nproc-per-node ${NPROC:-8} --master-addr 127.0.0.1 --master-port ${PORT:-29500} \
    $DIR/../llama/tp_zero1_llama_hf_pretrain.py --model_family gpt_neox --model_path ${MODEL:-gpt-neox-20b} \
    --tensor_parallel_size ${TP:-8} --seq_len ${SEQ_LEN:-2048} --batch_size 1 --grad_accum_usteps ${GRAD_ACCUM:-16} \
    --max_steps ${STEPS:-1000} --use_zero_1 --sequence_parallel_enabled --lr 1e-4 --warmup_steps 50 \
    ${DATA:+--data_dir $DATA} "$@"
