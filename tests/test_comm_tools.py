"""RCCL tooling on CPU/gloo: the collective benchmark runs end to end on N ranks and records the
communication environment; library RCCL defaults never override a user's setting."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_collectives_gloo():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", NXD_RCCL_CHANNELS="16")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "tools/bench_collectives.py", "--gpus", "3", "--cpu", "--sizes", "1",
                        "--iters", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert {x["op"] for x in recs} == {"all_gather", "reduce_scatter", "all_reduce", "p2p_neighbours"}
    for x in recs:
        assert x["ranks"] == 3 and x["busbw_gbs"] > 0
        assert x["env"]["NCCL_MAX_NCHANNELS"] == "16"


def test_apply_rccl_env_respects_user(monkeypatch):
    from neuronx_distributed_llama3_2_amd.parallel import rccl_env

    monkeypatch.setenv("TORCH_NCCL_AVOID_RECORD_STREAMS", "0")
    monkeypatch.delenv("NXD_RCCL_CHANNELS", raising=False)
    applied = rccl_env.apply_rccl_env({"NCCL_DEBUG": "WARN"})
    assert os.environ["TORCH_NCCL_AVOID_RECORD_STREAMS"] == "0"
    assert "TORCH_NCCL_AVOID_RECORD_STREAMS" not in applied
    cfg = rccl_env.log_comm_config(force=True)
    assert cfg["TORCH_NCCL_AVOID_RECORD_STREAMS"] == "0"
    if "NCCL_DEBUG" in applied:
        monkeypatch.delenv("NCCL_DEBUG")


def test_default_channel_cap_logged(monkeypatch):
    """The measured default (16 channels max, profiles/r3_cu_interference.jsonl) is applied unless the
    user set NCCL_MAX_NCHANNELS or NXD_RCCL_CHANNELS=auto, and appears in the logged config."""
    from neuronx_distributed_llama3_2_amd.parallel import rccl_env

    monkeypatch.delenv("NXD_RCCL_CHANNELS", raising=False)
    monkeypatch.delenv("NCCL_MAX_NCHANNELS", raising=False)
    applied = rccl_env.apply_rccl_env()
    assert applied.get("NCCL_MAX_NCHANNELS") == str(rccl_env.DEFAULT_CHANNELS)
    assert rccl_env.log_comm_config(force=True)["NCCL_MAX_NCHANNELS"] == "16"
    monkeypatch.delenv("NCCL_MAX_NCHANNELS")
    monkeypatch.setenv("NXD_RCCL_CHANNELS", "auto")
    assert "NCCL_MAX_NCHANNELS" not in rccl_env.apply_rccl_env()
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "40")
    monkeypatch.delenv("NXD_RCCL_CHANNELS")
    rccl_env.apply_rccl_env()
    assert os.environ["NCCL_MAX_NCHANNELS"] == "40"


def test_comm_cu_reservation_only_for_multi_rank(monkeypatch):
    from neuronx_distributed_llama3_2_amd.parallel import rccl_env

    monkeypatch.delenv("TENSILE_STREAMK_MAX_CUS", raising=False)
    monkeypatch.setenv("NXD_COMM_RESERVE_CUS", "16")
    monkeypatch.setattr(rccl_env, "_num_cus", lambda: 256)
    applied = rccl_env.apply_rccl_env(world_size=1)
    assert "TENSILE_STREAMK_MAX_CUS" not in applied
    applied = rccl_env.apply_rccl_env(world_size=8)
    assert applied["TENSILE_STREAMK_MAX_CUS"] == "240"
    monkeypatch.delenv("TENSILE_STREAMK_MAX_CUS", raising=False)
