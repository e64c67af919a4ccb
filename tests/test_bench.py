"""bench.py contract on CPU/gloo: `python bench.py --gpus N` spawns its own N ranks (no launcher),
the torch.distributed.run form still works, and rank 0 prints exactly one well-formed JSON line."""

import json
import math
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "tiny", "--seq", "128", "--gbs", "4", "--steps", "1", "--warmup", "1", "--cpu"]


def _env():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(rec, n):
    assert rec["n_gpus"] == n and rec["comm_world_size"] == n
    assert rec["steps"] == 1 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == (f"tp{n}_sp" if n > 1 else "tp1")
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    # fresh random tokens every micro-step: loss stays near ln(V) (no memorisation)
    assert abs(rec["loss"] - math.log(1024)) < 0.5, rec["loss"]
    for k in ("metric", "unit", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert k in rec


@pytest.mark.parametrize("n", [1, 4])
def test_bench_self_spawn(n):
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), *ARGS], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    _check(recs[0], n)


def test_bench_torchrun():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29631", "bench.py", "--gpus", "2", *ARGS],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    _check(recs[0], 2)


def test_bench_rank_failure_propagates():
    # a launcher whose world size disagrees with --gpus must fail loudly, not hang
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_PORT="29632")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", *ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_bench_pipeline_mode():
    """--pp: TP = N / P x PP = P through NxDPPModel 1F1B (the BASELINE's TP=2 x PP=4 config shape)."""
    args = ["--model", "tiny", "--seq", "128", "--gbs", "8", "--steps", "1", "--warmup", "1", "--cpu", "--pp", "2"]
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", *args], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["config"]["parallelism"] == "tp2_sp_pp2_1f1b" and rec["config"]["grad_accum"] == 4
    assert rec["n_gpus"] == 4 and rec["value"] > 0
    assert abs(rec["loss"] - math.log(1024)) < 0.5, rec["loss"]


def test_bench_hung_rank_exits_through_watchdog():
    """A rank that stops making progress (injected hang before its 2nd micro-step; the other rank
    then blocks in a collective) ends the job with exit code 124 and each live rank's last
    collectives on stderr, well inside the driver's limit -- not a silent hang."""
    env = _env()
    env["NXD_FAULT_INJECT"] = "bench_microstep@1#2:hang"
    env["NXD_BENCH_WATCHDOG_S"] = "20"
    env["NXD_BENCH_STEP_WATCHDOG_S"] = "20"
    env["NXD_BENCH_LADDER"] = "0"    # this test: the watchdog exit path of one rung
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 124, (r.returncode, r.stderr[-3000:])
    assert "step watchdog: no progress" in r.stderr
    assert "last collectives issued" in r.stderr and "#" in r.stderr.split("last collectives issued")[1]
    assert not _json_lines(r.stdout)


def _ladder_env(**kw):
    env = _env()
    # rung 1: rank 1 hangs before its 2nd micro-step (the first timed one) -> step watchdog, exit 124;
    # rung 2: rank 0 dies at its first micro-step (exit 43); rung 3 must produce the result
    env["NXD_BENCH_LADDER_FAULTS"] = "1=bench_microstep@1#2:hang;2=bench_microstep@0#1:exit"
    env["NXD_BENCH_WATCHDOG_S"] = "60"
    env["NXD_BENCH_STEP_WATCHDOG_S"] = "15"
    env.update(kw)
    return env


def _check_ladder(r, n, budget_s):
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    _check(rec, n)
    assert rec["attempt"] == 3 and rec["ladder_rung"] == "conservative"
    assert rec["ladder_knobs"]["NXD_SP_STREAMS"] == "1" and rec["sp_streams"] == 1
    failed = rec["ladder_failed"]
    assert [f["rung"] for f in failed] == [1, 2]
    assert failed[0]["rc"] == 124 and "last collectives issued" in failed[0]["stderr_tail"], failed[0]
    assert failed[1]["rc"] == 43 and "injected fault" in failed[1]["stderr_tail"], failed[1]
    assert sum(f["s"] for f in failed) < budget_s
    # step-0 sanity: the initial loss is the random-init expectation
    assert abs(rec["loss_step0"] - math.log(1024)) < 0.5


def test_bench_ladder_recovers_self_spawn():
    """Fallback ladder, no launcher: a hang in rung 1 and a crash in rung 2 still give one valid
    JSON line from rung 3 (fresh child processes each rung), recording both failures."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, env=_ladder_env(),
                       capture_output=True, text=True, timeout=400)
    _check_ladder(r, 2, 400)


def test_bench_ladder_recovers_under_torchrun():
    """The same under torch.distributed.run (the driver's N-GPU launch): each launched process is
    its rank's supervisor; they agree on failure and on each rung's port over the launcher's store."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29633", "bench.py", "--gpus", "2", *ARGS],
                       cwd=ROOT, env=_ladder_env(), capture_output=True, text=True, timeout=400)
    _check_ladder(r, 2, 400)


def test_bench_ladder_rung_budget_kills_silent_hang():
    """With the step watchdog off, a hung rung is ended by its wall budget (the supervisor kills the
    rank processes) and the next rung still fits in the total budget."""
    env = _env()
    env.update(NXD_BENCH_LADDER_FAULTS="1=bench_microstep@1#2:hang", NXD_BENCH_WATCHDOG_S="0",
               NXD_BENCH_LADDER_BUDGET_S="150", NXD_BENCH_LADDER_MIN_RUNG_S="50")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["attempt"] == 2 and rec["ladder_failed"][0]["rc"] == 124
    assert "wall budget" in rec["ladder_failed"][0]["why"]


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_bench_ladder_names_the_hung_rank(launcher):
    """Rank 1 hangs and its own (short) step watchdog ends it; rank 0, blocked in a collective with a
    long watchdog, is killed by the supervisor.  The history must blame rank 1 -- its tail carries the
    watchdog's flight-recorder dump -- and list rank 0 as collateral, not as the failure."""
    env = _env()
    env.update(NXD_BENCH_LADDER_FAULTS="1=bench_microstep@1#2:hang", NXD_BENCH_WATCHDOG_S="60",
               NXD_BENCH_STEP_WATCHDOG_S="120,15")
    cmd = [sys.executable, "bench.py", "--gpus", "2", *ARGS]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", "29634", "bench.py", "--gpus", "2", *ARGS]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["attempt"] == 2
    f = rec["ladder_failed"][0]
    assert f["failed_rank"] == 1 and f["rc"] == 124, f
    assert "last collectives issued" in f["stderr_tail"], f
    assert f["killed_by_supervisor"] == [0], f
    assert "0" in f["killed_tails"]
