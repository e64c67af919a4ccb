#!/bin/bash
# round 5 D: whole-step kernel trace of the 1-GPU bench (ladder off: the profiler wraps the rank
# process itself), per-category split of the last step; MoE prefill timing print
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5d
mkdir -p $O
export PYTHONUNBUFFERED=1 NXD_BENCH_LADDER=0
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/step_breakdown.py "$T" > $O/step_breakdown.txt && python tools/step_breakdown.py "$T" --by-kernel > $O/step_breakdown_by_kernel.txt
head -25 $O/step_breakdown.txt
head -30 $O/step_breakdown_by_kernel.txt
unset NXD_BENCH_LADDER
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_moe_gpu.py -k prefill > $O/moe.log 2>&1 || { tail -30 $O/moe.log; exit 1; }
grep -E "moe prefill|passed|failed" $O/moe.log
