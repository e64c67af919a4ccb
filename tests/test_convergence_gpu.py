"""Long-horizon convergence parity on the GPU kernels (reference:
test/integration/combinatorial_tests/common/compare_gpu_trn1_metrics.py:34-75 -- rtol 0.05 on >= 95 %
of the steps after warm-up -- and test/integration/llama3_70B_4layers_PP/logger.py:50-55).

A 4-layer Llama (hidden 1024, 8 / 4 heads of 128, vocabulary 2048) trains for 500 steps at seq 2048 on
an in-repo Markov-chain corpus (tools/convergence.py) through the public training API with fp32-master
AdamW, as four runs in fresh processes:
  * the HIP kernels (bf16 copy-out round-to-nearest),
  * the HIP kernels with stochastic rounding of the bf16 weight copy-out,
  * every op on its plain-PyTorch reference (NXD_FORCE_REFERENCE=1) on the same GPU,
  * TP = 2 + sequence parallel on the HIP kernels, two ranks sharing the GPU (gloo group, SP
    collectives on the direct-peer IPC kernels).
Each must agree with the reference run at rtol 0.05 on >= 95 % of the steps after step 100, and the
loss must end far below ln V (near the chain's 1.13-nat entropy).  The curves are written under
gpurun_out/convergence/ (copied to profiles/ by hand)."""

import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
OUT = os.environ.get("NXD_CONVERGENCE_DIR", os.path.join(ROOT, "gpurun_out", "convergence"))
STEPS = int(os.environ.get("NXD_CONVERGENCE_STEPS", "500"))
START = 100

VARIANTS = {
    "hip": ({}, []),
    "hip_sr": ({"NXD_STOCHASTIC_ROUNDING": "1"}, []),
    "reference": ({"NXD_FORCE_REFERENCE": "1"}, []),
    # SP all-gathers / reduce-scatters on the peer kernels (host-staged gloo SP collectives made this
    # variant 240 s of the GPU suite); the remaining collectives (grad norm, CE stats) stay on gloo
    "tp2_sp_gloo": ({"NXD_SP_PEER": "1"}, ["--tp", "2", "--gloo-gpu"]),
}
_curves = {}


def _run(name):
    if name in _curves:
        return _curves[name]
    env_over, args = VARIANTS[name]
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, f"{name}.json")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", **env_over)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "convergence.py"), "--steps", str(STEPS),
                        "--out", out, *args], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    with open(out) as f:
        rec = json.load(f)
    assert rec["done"] and len(rec["losses"]) == STEPS
    _curves[name] = rec
    return rec


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["reference", "hip", "hip_sr", "tp2_sp_gloo"])
def test_convergence_curve(name):
    rec = _run(name)
    losses = rec["losses"]
    assert all(math.isfinite(x) for x in losses)
    assert abs(losses[0] - math.log(rec["config"]["vocab"])) < 0.5
    # learned: the tail sits far below ln V, near the chain's entropy
    tail = sum(losses[-20:]) / 20
    assert tail < 0.5 * rec["ln_vocab"] and tail < rec["chain_entropy"] + 0.6, tail
    if name != "reference":
        from convergence import agreement

        ref = _run("reference")["losses"]
        frac = agreement(losses, ref, START, 0.05)
        worst = max(abs(a - b) / b for a, b in zip(losses[START:], ref[START:]))
        print(f"{name}: {frac:.3f} of steps >= {START} within rtol 0.05 of the reference (worst {worst:.4f}); "
              f"final {losses[-1]:.4f} vs {ref[-1]:.4f}")
        assert frac >= 0.95, (frac, worst)
