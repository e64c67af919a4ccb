#!/bin/bash
# CodeGen2.5-7B (Llama architecture) training on infilled code, TP=8 + ZeRO-1
# (reference: examples/training/codegen25/tp_zero1_codegen25_7b_hf_pretrain.sh).  Prepare DATA with
#   python examples/training/codegen25/get_dataset_infill.py --input tokens.bin --output infill.bin \
#       --block_size 2048 --mask_ids <ids of <mask_1>..<mask_16>> --eom_id <id> --sep_ids <ids of <|endoftext|><sep>>
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
DIR=$(cd "$(dirname "$0")" && pwd)
torchrun --nproc-per-node ${NPROC:-8} --master-addr 127.0.0.1 --master-port ${PORT:-29500} \
    $DIR/../llama/tp_zero1_llama_hf_pretrain.py --model_path ${MODEL:-codegen25-7b} --tensor_parallel_size ${TP:-8} \
    --seq_len ${SEQ_LEN:-2048} --batch_size 1 --grad_accum_usteps ${GRAD_ACCUM:-16} --max_steps ${STEPS:-1000} \
    --use_zero_1 --sequence_parallel_enabled --lr 3e-5 --warmup_steps 10 ${DATA:+--data_dir $DATA} "$@"
