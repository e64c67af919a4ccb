#!/bin/bash
# round 5 B: one-shot peer all-reduce (IPC, ranks sharing the GPU), TP=2 decode on the fused kernels,
# decode timings TP=1 (graphs / eager) and the TP=2 one-GPU rehearsal, kernel trace of a TP=2 rank
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5b
mkdir -p $O
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_peer_allreduce_gpu.py -k "2" > $O/pytest_par.log 2>&1 || { tail -40 $O/pytest_par.log; exit 1; }
grep -E "checks|passed|failed" $O/pytest_par.log
timeout -k 10 300 $PYT tests/test_graph_capture_gpu.py > $O/pytest_gc.log 2>&1 || { tail -40 $O/pytest_gc.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest_gc.log
timeout -k 10 900 $PYT tests/test_spmd_inference_gpu.py tests/test_inference_gpu.py > $O/pytest_inf.log 2>&1 || { tail -40 $O/pytest_inf.log; exit 1; }
grep -E "near-tie|passed|failed" $O/pytest_inf.log
A="--prompt 128 --new 256 --runs 5"
timeout -k 10 300 python -u bench_inference.py $A --report $O/tp1_graphs.json > $O/tp1_graphs.log 2>&1 || { tail -20 $O/tp1_graphs.log; exit 1; }
timeout -k 10 300 python -u bench_inference.py $A --no-graphs --report $O/tp1_eager.json > $O/tp1_eager.log 2>&1 || { tail -20 $O/tp1_eager.log; exit 1; }
timeout -k 10 400 python -u tools/experiments/r5/launch_ranks.py 2 -- python -u bench_inference.py $A --gloo-gpu --report $O/tp2_gloo_gpu.json > $O/tp2.log 2>&1 || { tail -20 $O/tp2.log; exit 1; }
python - <<'PY'
import json
for k in ("tp1_graphs", "tp1_eager", "tp2_gloo_gpu"):
    d = json.load(open(f"gpurun_out/r5b/{k}.json"))
    print(k, round(d["token_generation"]["ms_per_token_p50"], 4), "ms/token", d["config"]["tp"], d["config"]["hip_graphs"])
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/experiments/r5/launch_ranks.py 2 -- rocprofv3 --kernel-trace --stats -d $O/prof_r{rank} -o run -- python -u bench_inference.py --prompt 128 --new 32 --runs 1 --gloo-gpu --report $O/tp2_prof.json > $O/tp2_prof.log 2>&1 || { tail -20 $O/tp2_prof.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -4
