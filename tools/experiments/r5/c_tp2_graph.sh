#!/bin/bash
# round 5 C: peer gather + TP=2 decode in hipGraphs over the peer kernels; TP=2 rehearsal timing with graphs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c
mkdir -p $O
export PYTHONUNBUFFERED=1
PYT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_peer_allreduce_gpu.py > $O/pytest_par.log 2>&1 || { tail -40 $O/pytest_par.log; exit 1; }
grep -E "checks|passed|failed" $O/pytest_par.log
timeout -k 10 600 $PYT tests/test_spmd_inference_gpu.py > $O/pytest_spmd.log 2>&1 || { tail -40 $O/pytest_spmd.log; exit 1; }
grep -E "TP=|near-tie|first differing|passed|failed" $O/pytest_spmd.log
A="--prompt 128 --new 256 --runs 5"
timeout -k 10 400 python -u tools/experiments/r5/launch_ranks.py 2 -- python -u bench_inference.py $A --gloo-gpu --report $O/tp2_gloo_gpu_graphs.json > $O/tp2.log 2>&1 || { tail -20 $O/tp2.log; exit 1; }
python -c "import json; d=json.load(open('$O/tp2_gloo_gpu_graphs.json')); print('tp2 graphs', d['token_generation'], d['config']['hip_graphs'])"
timeout -k 10 300 python -u tools/bench_dense_vs_hipblaslt.py > $O/dense_vs_hipblaslt.jsonl 2>$O/dense.err || { tail -20 $O/dense.err; exit 1; }
cat $O/dense_vs_hipblaslt.jsonl
