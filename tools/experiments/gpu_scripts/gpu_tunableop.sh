#!/bin/bash
# Tune hipBLASLt/rocBLAS GEMM solutions for the bench shapes with PyTorch TunableOp; results CSV is
# written under gpurun_out/ and copied into the repo (configs/) so later runs only read it.
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=15 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
timeout -k 10 900 python bench.py --gpus 1 --steps 2 --warmup 1 --gbs 2 > gpurun_out/tune/tune.log 2>&1
rc=$?; echo "tune rc=$rc" >> gpurun_out/tune/tune.log; [ $rc -ne 0 ] && exit $rc
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/tune/bench_tuned.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/tune/bench_tuned.log
exit $rc
