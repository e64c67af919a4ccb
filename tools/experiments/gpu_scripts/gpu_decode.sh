#!/bin/bash
mkdir -p gpurun_out/decode
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "decode or argmax" > gpurun_out/decode/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/decode/pytest.log; [ $rc -ne 0 ] && exit $rc
NXD_DECODE_FUSED_MERGE=1 timeout -k 10 300 python tools/bench_decode.py > gpurun_out/decode/fused.json 2>gpurun_out/decode/err1.log
rc=$?; [ $rc -ne 0 ] && exit $rc
NXD_DECODE_FUSED_MERGE=0 timeout -k 10 300 python tools/bench_decode.py > gpurun_out/decode/split.json 2>gpurun_out/decode/err0.log
rc=$?; [ $rc -ne 0 ] && exit $rc
NXD_DECODE_FUSED_MERGE=0 timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "decode" >> gpurun_out/decode/pytest.log 2>&1
exit $?
