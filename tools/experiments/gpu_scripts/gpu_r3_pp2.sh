#!/bin/bash
# PP default on: dense + MoE A/B, Mixtral 4-layer training bench, SP chunk bench, smoke + default bench.
set -o pipefail
O=gpurun_out/r3pp2; mkdir -p $O
timeout -k 10 300 python -u tools/bench_pp_ab.py > $O/pp_ab.jsonl 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_mixtral_train.py --layers 4 --seq 4096 --mbs 2 --accum 4 --steps 3 > $O/mixtral_train.jsonl 2> $O/mixtral_train.err || exit $?
bash tools/gpu_r3_spchunks.sh || exit $?
bash tools/gpu_r3_final.sh || exit $?
