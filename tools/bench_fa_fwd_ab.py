"""FA forward TFLOP/s at the bench's attention shapes, for A/B of kernel builds: --root picks the
directory the package is imported from (e.g. a copy built from another commit).  One JSON line per
shape: median over rounds of the mean of `reps` launches."""
import argparse
import json
import os
import statistics
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--root", default=".")
ap.add_argument("--tag", default="")
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
sys.path.insert(0, os.path.abspath(a.root))
import torch  # noqa: E402

import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402

assert os.path.abspath(ops.__file__).startswith(os.path.abspath(a.root)), ops.__file__


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


# (B, S, Hq, Hkv, D): the TP=1 bench micro-step (2 x 8192, 32 / 8 heads), the TP=8 rank (8 x 8192, 4 / 1),
# Llama-3.2-1B prefill (D = 64)
for (B, S, H, Hkv, D) in [(2, 8192, 32, 8, 128), (8, 8192, 4, 1, 128), (1, 8192, 32, 8, 64)]:
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * B * H * S * S * D * 0.5
    o = ops.flash_attn_fwd_lse(q, k, v, causal=True)[0].float()
    ref_rows = slice(S - 64, S)   # fp32 check of the last 64 query rows (the longest sweeps)
    qr, kr, vr = q[:, ref_rows].float(), k.float(), v.float()
    kr = kr.repeat_interleave(H // Hkv, dim=2)
    vr = vr.repeat_interleave(H // Hkv, dim=2)
    sc = torch.einsum("bqhd,bkhd->bhqk", qr, kr) * D ** -0.5
    pos_q = torch.arange(S - 64, S, device="cuda")[:, None]
    sc = sc.masked_fill(torch.arange(S, device="cuda")[None, :] > pos_q, float("-inf"))
    ref = torch.einsum("bhqk,bkhd->bqhd", sc.softmax(-1), vr)
    err = ((o[:, ref_rows] - ref).abs().max() / ref.abs().max()).item()
    ts = [timed(lambda: ops.flash_attn_fwd_lse(q, k, v, causal=True), a.reps) for _ in range(a.rounds)]
    ms = statistics.median(ts)
    print(json.dumps({"tag": a.tag, "B": B, "S": S, "H": H, "Hkv": Hkv, "D": D, "fwd_ms": round(ms, 4),
                      "fwd_tf": round(fl / ms / 1e9, 1), "rel_err": round(err, 5)}), flush=True)
