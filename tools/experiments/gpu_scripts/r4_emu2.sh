#!/bin/bash
# Round 4 (2): exhaustive GEMM in place, Llama-3-70B TP=8 emulated rank, RCCL-like link CU footprint.
set -o pipefail
O=gpurun_out/r4emu2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_exhaustive_gpu.py > $O/gemm_exhaustive_test.log 2>&1 || exit $?
NXD_GEMM_TUNE=2 NXD_GEMM_NO_STREAMK=1 NXD_GEMM_TUNE_MAX_ALGOS=1024 NXD_GEMM_LOG_CHOICE=1 timeout -k 10 200 python -u tools/check_gemm_exhaustive.py --tokens 16384 > $O/gemm_exhaustive_16k.jsonl 2>$O/gemm_exhaustive_16k.err || exit $?
E="python -u tools/emulate_tp_rank.py --steps 2 --warmup 1"
run() { echo "== $*" >&2; timeout -k 10 400 $E "$@" 2>> $O/emulate.err | grep '^{' >> $O/emulate.jsonl || exit $?; }
run --tp 8 --model llama3-70b --mbs 1 --gbs 8 --link-gbps 400
run --tp 8 --model llama3-70b --mbs 2 --gbs 8 --link-gbps 400
run --tp 8 --model llama3-70b --mbs 2 --gbs 8 --ckpt selective --link-gbps 400
run --tp 8 --model llama3-70b --mbs 1 --gbs 8
run --tp 8 --link-gbps 400 --link-cus 16 --sp-streams 2
NXD_GEMM_NO_STREAMK=1 run --tp 8 --link-gbps 400 --link-cus 16 --sp-streams 2
run --tp 8 --link-gbps 400 --link-cus 16 --sp-streams 1
