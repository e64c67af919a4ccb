#!/bin/bash
# Llama-3-70B TP=8 x PP=N pre-training (reference: tp_pp_llama_hf_pretrain/run_llama3_70B_tp_pp.sh).
# One process per MI355X; NNODES/NODE_RANK/MASTER_ADDR for multi-node, RCCL over xGMI inside a node.
set -euo pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPUS_PER_NODE=${GPUS_PER_NODE:-8}
NNODES=${NNODES:-1}
NODE_RANK=${NODE_RANK:-0}
MASTER_ADDR=${MASTER_ADDR:-127.0.0.1}
TP_DEGREE=${TP_DEGREE:-8}
PP_DEGREE=${PP_DEGREE:-$NNODES}
GBS=${GBS:-1024}
SEQ_LEN=${SEQ_LEN:-8192}
NUM_MICROBATCHES=${NUM_MICROBATCHES:-32}
WORLD=$((GPUS_PER_NODE * NNODES))
DP=$((WORLD / TP_DEGREE / PP_DEGREE))
BS=$((GBS / DP))
cd "$(dirname "$0")"
python -m torch.distributed.run --nproc-per-node "$GPUS_PER_NODE" --nnodes "$NNODES" --node-rank "$NODE_RANK" \
  --master-addr "$MASTER_ADDR" --master-port "${MASTER_PORT:-29533}" tp_pp_llama_hf_pretrain.py \
  --model_path "${MODEL_PATH:-llama3-70b}" --tensor_parallel_size "$TP_DEGREE" \
  --pipeline_parallel_size "$PP_DEGREE" --num_microbatches "$NUM_MICROBATCHES" --train_batch_size "$BS" \
  --seq_len "$SEQ_LEN" --use_zero_1 --sequence_parallel_enabled --selective_checkpoint_enabled \
  --max_steps "${MAX_STEPS:-1000}" --warmup_steps 100 --lr 1.5e-4 --min_lr 1e-5 \
  --checkpoint_dir "${CKPT_DIR:-ckpt_70b}" --checkpoint_freq "${CKPT_FREQ:-100}" --num_kept_checkpoint 2 \
  --async_checkpoint_saving --watchdog_timeout "${WATCHDOG:-1800}" ${DATA_DIR:+--data_dir "$DATA_DIR"} "$@"
