#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --gpus 1 --steps 1 --warmup 1 --gbs 2 > gpurun_out/prof1/bench.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/prof1/bench.log
find gpurun_out/prof1 -name "*stats*" | head
exit $rc
