"""xser checkpoints in torch_xla's format (reference trainer/checkpoint.py:308-470): records pickled
as torch_xla.utils.serialization.TensorReference, `.info.pt` tensor metadata, DP-deduplicated
bin-packed tensor writes and round-robin read + broadcast loading.

torch_xla is not installed here: a throwaway subprocess registers a stand-in module under that
name with the same class definition as torch_xla's, so it pickles exactly what the reference's
xser writer pickles -- that subprocess produces the "reference" checkpoint we read, and reads ours.
"""

import os
import subprocess
import sys
import tempfile
import textwrap

import torch

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.utils import serialization as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_FAKE_XLA = textwrap.dedent("""
    import sys, types, os, torch
    m = types.ModuleType("torch_xla.utils.serialization")
    class TensorReference(object):          # torch_xla/utils/serialization.py
        def __init__(self, tid):
            self.tid = tid
    TensorReference.__module__ = "torch_xla.utils.serialization"
    m.TensorReference = TensorReference
    for name in ("torch_xla", "torch_xla.utils"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["torch_xla.utils.serialization"] = m
""")


def _run(code: str):
    r = subprocess.run([sys.executable, "-c", _FAKE_XLA + textwrap.dedent(code)], capture_output=True, text=True,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_reads_reference_written_xser():
    d = tempfile.mkdtemp()
    path = os.path.join(d, "dp_rank_00_tp_rank_00_pp_rank_00.pt")
    _run(f"""
        path = {path!r}
        torch.manual_seed(0)
        sd = {{"w": torch.randn(4, 8), "b": torch.arange(3), "nested": {{"m": torch.ones(2, dtype=torch.bfloat16)}},
              "step": 7}}
        os.makedirs(path + ".tensors")
        refs, info = {{}}, {{}}
        tid = 0
        def strip(o):
            global tid
            if isinstance(o, torch.Tensor):
                torch.save(o, os.path.join(path + ".tensors", "tensor_%d.pt" % tid))
                info[tid] = {{"dtype": o.dtype, "shape": o.shape, "expert_model_parallel": False}}
                tid += 1
                return TensorReference(tid - 1)
            if isinstance(o, dict):
                return {{k: strip(v) for k, v in o.items()}}
            return o
        torch.save(strip(sd), path)
        torch.save(info, path + ".info.pt")
        torch.save(sd, path + ".expected")
    """)
    got = S.xser_load(path)
    exp = torch.load(path + ".expected", weights_only=True)
    assert torch.equal(got["w"], exp["w"]) and torch.equal(got["b"], exp["b"])
    assert torch.equal(got["nested"]["m"], exp["nested"]["m"]) and got["step"] == 7
    assert S.xser_load_info(path)[0]["shape"] == (4, 8)


def test_reference_reads_our_xser():
    d = tempfile.mkdtemp()
    path = os.path.join(d, "m.pt")
    sd = {"a": torch.randn(3, 5), "l": [torch.arange(4), "x"], "k": 1}
    S.xser_save(sd, path)
    out = _run(f"""
        path = {path!r}
        ref = torch.load(path, weights_only=False)   # a file this test wrote
        from torch_xla.utils.serialization import TensorReference
        assert isinstance(ref["a"], TensorReference) and ref["a"].tid == 0 and ref["l"][0].tid == 1, ref
        t = torch.load(os.path.join(path + ".tensors", "tensor_%d.pt" % ref["a"].tid))
        info = torch.load(path + ".info.pt")
        print(tuple(t.shape), info[1]["dtype"], ref["l"][1], ref["k"])
    """)
    assert out.strip() == "(3, 5) torch.int64 x 1"


def _dedup(rank, world, ckpt, out):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    ps.initialize_model_parallel(1)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 32), torch.nn.Linear(32, 8))
    nxd.save_checkpoint(ckpt, "t1", model=model, use_xser=True)
    nxd.finalize_checkpoint()
    torch.manual_seed(1)
    fresh = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 32), torch.nn.Linear(32, 8))
    nxd.load_checkpoint(ckpt, "t1", model=fresh)
    for a, b in zip(model.parameters(), fresh.parameters()):
        assert torch.equal(a, b)
    if rank == 0:
        torch.save(True, out)


def test_dp2_dedup_xser_save_and_broadcast_load(monkeypatch):
    d = tempfile.mkdtemp()
    ck = os.path.join(d, "ck")
    run_distributed(_dedup, 2, ck, os.path.join(d, "ok.pt"))
    assert torch.load(os.path.join(d, "ok.pt"))
    base = os.path.join(ck, "t1", "model", "dp_rank_00_tp_rank_00_pp_rank_00.pt")
    files = sorted(os.listdir(base + ".tensors"))
    assert files == [f"tensor_{i}.pt" for i in range(6)], files
    assert os.path.exists(base + ".info.pt")
    # the bins split the bytes between the two replicas: the largest tensor alone vs the rest
    sizes = [os.path.getsize(os.path.join(base + ".tensors", f)) for f in files]
    bins = S.assign_tensors_to_bins([torch.empty(64 * 128), torch.empty(128), torch.empty(128 * 32), torch.empty(32),
                                     torch.empty(32 * 8), torch.empty(8)], 2)
    assert sorted(len(b) for b in bins) == [1, 5] and len(sizes) == 6
