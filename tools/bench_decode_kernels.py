"""Decode-step kernel A/B on one MI355X (bs = 1): fused GEMVs (csrc/decode_fused.hip) against the
plain skinny GEMM (csrc/gemv.hip) on Llama-3.2-1B / Llama-3-8B projection shapes, with the GLU
row-pair and k-slice knobs; MFMA decode attention (decode_attn.hip) against the 128-key-chunk
kernel (inference.hip) at several cache lengths.  One JSON line per measurement."""
import json
import sys

import torch

sys.path.insert(0, ".")
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops.gemv import skinny_linear  # noqa: E402


def timed(fn, reps=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0   # us


def out(rec):
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in rec.items()}), flush=True)


def gemvs(C, model, H, I, nq, nkv, D, V):
    dev = "cuda"
    x = torch.randn(1, H, device=dev, dtype=torch.bfloat16)
    nw = torch.randn(H, device=dev, dtype=torch.bfloat16)
    shapes = {"qkv": ((nq + 2 * nkv) * D, H, 0), "o": (H, nq * D, 1), "gate_up": (2 * I, H, 2), "down": (H, I, 1),
              "lm_head": (V, H, 0)}
    for name, (Nw, K, epi) in shapes.items():
        w = torch.randn(Nw, K, device=dev, dtype=torch.bfloat16) * 0.02
        xi = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        N = Nw // 2 if epi == 2 else Nw
        y = torch.zeros(1, N, device=dev, dtype=torch.bfloat16)
        nbytes = Nw * K * 2
        norm = nw if K == H and name in ("qkv", "gate_up", "lm_head") else None
        t_old = timed(lambda: skinny_linear(xi, w, glu=(epi == 2)))
        out({"model": model, "op": name, "kernel": "gemv.hip", "us": t_old, "TBps": nbytes / t_old / 1e6})
        for ks in ([0] if epi == 2 else [0, 1, 2, 4]):
            for pairs in ([1, 2] if epi == 2 else [1]):
                C.decode_set_knob(0, pairs)
                C.decode_set_knob(1, ks)
                t = timed(lambda: C.dgemv(epi, xi, norm, 1e-5, w, y, 0, 0, 0, None, None, None, 1, None, None, None))
                out({"model": model, "op": name, "kernel": "decode_fused", "norm": norm is not None, "ks": ks,
                     "glu_pairs": pairs, "us": t, "TBps": nbytes / t / 1e6})
        C.decode_set_knob(0, 1)
        C.decode_set_knob(1, 0)
        del w
    # QKV with RoPE + KV-cache write epilogue
    Nw = (nq + 2 * nkv) * D
    w = torch.randn(Nw, H, device=dev, dtype=torch.bfloat16) * 0.02
    qkv = torch.empty(1, Nw, device=dev, dtype=torch.bfloat16)
    kc = torch.zeros(1, nkv, 4096, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    cos = torch.randn(8192, D // 2, device=dev)
    sin = torch.randn(8192, D // 2, device=dev)
    pos = torch.tensor([777], device=dev, dtype=torch.int64)
    t = timed(lambda: C.dgemv(3, x, nw, 1e-5, w, qkv, nq, nkv, D, cos, sin, pos, 1, kc, vc, None))
    out({"model": model, "op": "qkv_rope_kv", "kernel": "decode_fused", "us": t, "TBps": Nw * H * 2 / t / 1e6})


def attention(C, model, nq, nkv, D):
    dev = "cuda"
    for L in (384, 1024, 2048, 8192):
        kc = torch.randn(1, nkv, L, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(1, 1, nq, D, device=dev, dtype=torch.bfloat16)
        seq = torch.tensor([L], device=dev, dtype=torch.int32)
        o = torch.empty_like(q)
        for v2 in (0, 1):
            C.decode_set_knob(2, v2)
            t = timed(lambda: ops.decode_attention(q, kc, vc, seq, out=o))
            out({"model": model, "op": "decode_attention", "L": L, "kernel": "mfma_v2" if v2 else "chunk128",
                 "us": t, "TBps": 2 * kc.numel() * 2 / t / 1e6})
    C.decode_set_knob(2, 1)


def main():
    C = ops.ext()
    gemvs(C, "llama3.2-1b", 2048, 8192, 32, 8, 64, 128256)
    attention(C, "llama3.2-1b", 32, 8, 64)
    gemvs(C, "llama3-8b", 4096, 14336, 32, 8, 128, 128256)
    attention(C, "llama3-8b", 32, 8, 128)


if __name__ == "__main__":
    main()
