"""Flash attention fwd/bwd time vs micro-batch and memory layout, at the Llama-3-8B TP=1 and TP=8
per-rank head counts (S = 8192, D = 128, causal), on random data.

  layout "bshd": contiguous [B, S, H, D] (batch-major)
  layout "sbhd": the training model's layout, views of a fused [S, B, (Hq+2Hkv)*D] QKV buffer
Optionally sweeps the backward work-item chunk (--chunks) to check the host's chunk chooser.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import ops  # noqa: E402


def tm(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--heads", default="32:8,4:1")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--layouts", nargs="+", default=["bshd", "sbhd"])
    ap.add_argument("--chunks", type=int, nargs="*", default=[0])
    a = ap.parse_args()
    ext = ops.ext()
    D, S = 128, a.seq
    for hs in a.heads.split(","):
        Hq, Hkv = map(int, hs.split(":"))
        for B in a.batch:
            for lay in a.layouts:
                if lay == "bshd":
                    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
                    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
                    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
                else:
                    qkv = torch.randn(S, B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
                    q = qkv[..., :Hq * D].view(S, B, Hq, D).transpose(0, 1)
                    k = qkv[..., Hq * D:(Hq + Hkv) * D].view(S, B, Hkv, D).transpose(0, 1)
                    v = qkv[..., (Hq + Hkv) * D:].view(S, B, Hkv, D).transpose(0, 1)
                o = torch.empty(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
                lse = torch.empty(B, Hq, S, device="cuda", dtype=torch.float32)
                scale = D ** -0.5
                fl = 4.0 * B * Hq * S * S * D / 2   # causal fwd FLOPs
                tf = tm(lambda: ext.flash_attn_fwd(q, k, v, o, lse, scale, True, 0))
                do = torch.randn_like(o)
                dq, dk, dv = torch.empty_like(o), torch.empty(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16), \
                    torch.empty(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
                for ch in a.chunks:
                    ext.flash_attn_set_knob(1, ch)
                    tb = tm(lambda: ext.flash_attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True, 0))
                    print(json.dumps({"Hq": Hq, "Hkv": Hkv, "B": B, "S": S, "layout": lay, "bwd_chunk": ch or "auto",
                                      "fwd_ms": round(tf, 3), "fwd_tf": round(fl / tf / 1e9, 1),
                                      "bwd_ms": round(tb, 3), "bwd_tf": round(2.5 * fl / tb / 1e9, 1)}), flush=True)
                ext.flash_attn_set_knob(1, 0)
                del q, k, v, o, lse, do, dq, dk, dv
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
