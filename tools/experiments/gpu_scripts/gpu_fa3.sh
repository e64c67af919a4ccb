#!/bin/bash
mkdir -p gpurun_out/fa
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "flash or rope_attention" > gpurun_out/fa/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/fa/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only fa > gpurun_out/fa/bench.jsonl 2>gpurun_out/fa/bench.err || exit $?
timeout -k 10 300 python tools/bench_kernels.py --only fa_tp > gpurun_out/fa/bench_tp.jsonl 2>>gpurun_out/fa/bench.err || exit $?
timeout -k 10 300 python tools/bench_fa_ablate.py > gpurun_out/fa/ablate.jsonl 2>gpurun_out/fa/ablate.err
