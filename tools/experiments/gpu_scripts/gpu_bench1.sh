#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench1.log
exit $rc
