"""Fault injection / resume: a rank killed mid-save leaves an incomplete tag that
is never picked for resume and is garbage-collected by the next save; async-save failures re-raise;
the step watchdog fires on a hung loop; the restart supervisor resumes a crashed job to completion."""

import os
import subprocess
import sys
import tempfile
import textwrap

import pytest
import torch

from neuronx_distributed_llama3_2_amd.utils import resilience

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# A tiny "training job": resumes from the latest complete checkpoint, trains to step 6, saving
# every 2 steps.  Faults are armed through NXD_FAULT_INJECT by the test.
JOB = textwrap.dedent("""
    import os, sys, torch
    sys.path.insert(0, {repo!r})
    from neuronx_distributed_llama3_2_amd.trainer import checkpoint as ck
    from neuronx_distributed_llama3_2_amd.utils.resilience import fault_point
    d = sys.argv[1]
    torch.manual_seed(0)
    m = torch.nn.Linear(4, 4)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    step = 0
    if ck.has_checkpoint(d):
        step = ck.load_checkpoint(d, model=m, optimizer=opt)["step"]
        print("resumed", step, flush=True)
    x = torch.ones(2, 4)
    while step < 6:
        fault_point("train_step_%d" % step)
        opt.zero_grad(); m(x).square().sum().backward(); opt.step(); step += 1
        if step % 2 == 0:
            ck.save_checkpoint(d, tag=str(step), model=m, optimizer=opt, user_content={{"step": step}},
                               num_kept_ckpts=2, async_save=bool(int(os.environ.get("ASYNC", "0"))))
    ck.finalize_checkpoint()
    print("final", step, float(m.weight.sum()), flush=True)
""")


def _job_file(d):
    p = os.path.join(d, "job.py")
    with open(p, "w") as f:
        f.write(JOB.format(repo=REPO))
    return p


def _run(job, ckdir, fault="", asyn=False):
    env = dict(os.environ, NXD_FAULT_INJECT=fault, ASYNC="1" if asyn else "0")
    return subprocess.run([sys.executable, job, ckdir], capture_output=True, text=True, env=env, timeout=300)


def _reference_final(tmp):
    r = _run(_job_file(tmp), os.path.join(tmp, "clean"))
    assert r.returncode == 0, r.stderr
    return [ln for ln in r.stdout.splitlines() if ln.startswith("final")][0]


@pytest.mark.parametrize("asyn", [False, True])
def test_kill_before_done_marker_then_resume(asyn):
    tmp = tempfile.mkdtemp()
    job, ck = _job_file(tmp), os.path.join(tmp, "ck")
    # rank dies after writing tag 4's shards but before its `done` marker
    r = _run(job, ck, fault="ckpt_before_done#2:exit" if not asyn else "train_step_5:exit", asyn=asyn)
    assert r.returncode == resilience.FAULT_EXIT_CODE, r.stderr
    tags = sorted(os.listdir(ck))
    assert "2" in tags
    if not asyn:
        assert "4" in tags and not os.path.exists(os.path.join(ck, "4", "done"))
    from neuronx_distributed_llama3_2_amd.trainer.checkpoint_storage import create_checkpoint_storage

    latest = create_checkpoint_storage(ck).get_latest_tag()
    assert latest == "2"   # async: tag 4's marker is only written at the next save / finalize
    # restart: resumes from the last complete tag, finishes, and matches an uninterrupted run
    r2 = _run(job, ck, asyn=asyn)
    assert r2.returncode == 0, r2.stderr
    assert f"resumed {latest}" in r2.stdout
    final = [ln for ln in r2.stdout.splitlines() if ln.startswith("final")][0]
    assert final == _reference_final(tmp)
    tags = sorted(os.listdir(ck))
    assert tags == ["4", "6"]   # incomplete tag removed, keep-2 GC
    assert all(os.path.exists(os.path.join(ck, t, "done")) for t in tags)


def test_kill_mid_shard_write_never_resumed():
    tmp = tempfile.mkdtemp()
    job, ck = _job_file(tmp), os.path.join(tmp, "ck")
    r = _run(job, ck, fault="ckpt_after_shard_write:exit")
    assert r.returncode == resilience.FAULT_EXIT_CODE
    from neuronx_distributed_llama3_2_amd.trainer import checkpoint as ckm

    assert not ckm.has_checkpoint(ck)   # tag 2 began but never completed
    r2 = _run(job, ck)
    assert r2.returncode == 0 and "resumed" not in r2.stdout


def test_async_save_failure_reraises(tmp_path, monkeypatch):
    from neuronx_distributed_llama3_2_amd.trainer import checkpoint as ckm

    monkeypatch.setenv("NXD_FAULT_INJECT", "ckpt_after_shard_write:raise")
    m = torch.nn.Linear(2, 2)
    ckm.save_checkpoint(str(tmp_path), tag="1", model=m, async_save=True)
    with pytest.raises(resilience.InjectedFault):
        ckm.finalize_checkpoint()
    monkeypatch.setenv("NXD_FAULT_INJECT", "")
    assert not ckm.has_checkpoint(str(tmp_path))
    ckm.save_checkpoint(str(tmp_path), tag="2", model=m, async_save=True)
    ckm.finalize_checkpoint()
    assert sorted(os.listdir(tmp_path)) == ["2"]


def test_fault_point_rank_filter_and_raise(monkeypatch):
    monkeypatch.setenv("NXD_FAULT_INJECT", "a@3:raise,b:raise")
    monkeypatch.setenv("RANK", "0")
    resilience.fault_point("a")        # armed for rank 3 only
    resilience.fault_point("zzz")      # not armed
    with pytest.raises(resilience.InjectedFault):
        resilience.fault_point("b")
    monkeypatch.setenv("NXD_FAULT_INJECT", "d#2:raise")
    resilience.fault_point("d")
    with pytest.raises(resilience.InjectedFault):
        resilience.fault_point("d")
    resilience.fault_point("d")
    monkeypatch.setenv("NXD_FAULT_INJECT", "c:explode")
    with pytest.raises(ValueError):
        resilience.fault_point("c")


def test_step_watchdog_fires_and_stays_quiet():
    fired = []
    with resilience.StepWatchdog(0.3, on_timeout=lambda: fired.append(1), poll_s=0.05) as wd:
        for _ in range(6):
            wd.kick()
            import time

            time.sleep(0.05)
        assert not wd.fired
        time.sleep(0.8)
        assert wd.fired and fired == [1]


def test_restart_supervisor_resumes_to_completion():
    tmp = tempfile.mkdtemp()
    job, ck = _job_file(tmp), os.path.join(tmp, "ck")
    env = dict(os.environ, NXD_FAULT_INJECT="train_step_3:exit", ASYNC="0")
    rc = resilience.run_with_restarts([sys.executable, job, ck], max_restarts=2, env=env, backoff_s=0.0,
                                      on_restart=lambda a, rc: {"NXD_FAULT_INJECT": ""})
    assert rc == 0
    assert sorted(os.listdir(ck)) == ["4", "6"]
