"""tools/emulate_tp_rank.py: one TP rank of the N-GPU bench on the in-process "fake" process group
(world size = TP, this process rank 0; collectives replaced by their local HBM work).  CPU plumbing
check here; the GPU suite runs it on the HIP kernels at real TP=8 shard shapes (few layers)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "tools/emulate_tp_rank.py", *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(recs) == 1, r.stdout
    return recs[0]


@pytest.mark.parametrize("tp", [2, 8])
def test_emulated_tp_rank_cpu(tp):
    rec = _run("--tp", str(tp), "--cpu", "--layers", "1", "--hidden", "1024", "--seq", "128", "--gbs", "8",
               "--steps", "1", "--warmup", "1")
    assert rec["tp"] == tp and rec["sp"] is True
    assert rec["grad_accum"] * rec["mbs"] == 8
    # the TP shard of every weight: 1/tp of the full layer (+ replicated norms)
    assert rec["params_per_rank"] > 0 and rec["ms_per_step"] > 0


@pytest.mark.gpu
def test_emulated_tp8_rank_gpu():
    # real Llama-3-8B TP=8 shard shapes on the HIP kernels (2 layers): runs end to end
    rec = _run("--tp", "8", "--layers", "2", "--steps", "1", "--warmup", "1", timeout=300)
    assert rec["tp"] == 8 and rec["mbs"] == 8 and rec["peak_mem_gib"] > 0   # bench.MBS_BY_TP[8]
