"""One-shot peer all-reduce (csrc/peer_allreduce.hip, parallel/peer_allreduce.py) with W processes
sharing the box's GPU through IPC handles: sum / residual-fold / residual-set modes bitwise against a
rank-order fp32 recomputation, the vocab-parallel gather, the sequence-parallel all-gather /
reduce-scatter (async handles, region growth), inside replayed hipGraphs too, and no peer ever missing its flag."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return str(p)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_peer_allreduce_ranks_on_one_gpu(world):
    out = os.path.join(tempfile.mkdtemp(), "par.json")
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   NXD_PEER_AR_SPIN_LIMIT="4000000")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "peer_ar_worker.py"), out], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-2000:] for l in logs)
    with open(out) as f:
        rec = json.load(f)
    print(rec)
    assert rec["errors"] == 0 and rec["checks"] == 61


@pytest.mark.timeout(200)
def test_peer_allreduce_lost_peer_raises():
    """A rank that skips a call: its peer's call times out, writes NaN and raises on check(); the
    skipping rank's next call reads the poisoned flags and raises too -- nobody gets a plausible sum."""
    out = os.path.join(tempfile.mkdtemp(), "lost")
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                   NXD_PEER_AR_SPIN_LIMIT="20000", NXD_PEER_AR_DROP="1:3")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "peer_ar_lost_worker.py"), out],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = [p.communicate(timeout=150)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-2000:] for l in logs)
    r0 = json.load(open(out + ".0"))
    r1 = json.load(open(out + ".1"))
    print(r0, r1)
    assert r0["raised_at"] == 3 and r0["calls_ok"] == 2 and r0["nan_output"], r0
    assert r1["raised_at"] == 4 and r1["calls_ok"] == 3 and r1["nan_output"], r1
