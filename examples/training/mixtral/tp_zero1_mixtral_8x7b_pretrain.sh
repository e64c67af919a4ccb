#!/bin/bash
# Mixtral-8x7B pre-training on one 8x MI355X node: TP=8 (experts sharded on the intermediate dim,
# dropless MoE) + sequence parallel + ZeRO-1; EP=2 with a capacity factor via EP=2 CF=2.0
# (reference: examples/training/mixtral/ — PTL + NxD MoE).
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
DIR=$(cd "$(dirname "$0")" && pwd)
EP=${EP:-1}
torchrun --nproc-per-node ${NPROC:-8} --master-addr 127.0.0.1 --master-port ${PORT:-29500} \
    $DIR/../llama/tp_zero1_llama_hf_pretrain.py --model_family mixtral --model_path ${MODEL:-mixtral-8x7b} \
    --tensor_parallel_size ${TP:-8} --expert_parallel_size $EP ${CF:+--capacity_factor $CF} \
    --seq_len ${SEQ_LEN:-4096} --batch_size 1 --grad_accum_usteps ${GRAD_ACCUM:-8} --max_steps ${STEPS:-1000} \
    --use_zero_1 --sequence_parallel_enabled --lr 1e-4 --warmup_steps 50 \
    --checkpoint_dir ${CKPT_DIR:-ckpt_mixtral} --checkpoint_freq ${CKPT_FREQ:-500} ${DATA:+--data_dir $DATA} "$@"
