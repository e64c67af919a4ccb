"""Exhaustive hipBLASLt search (NXD_GEMM_TUNE=2) on the production layouts of the TP=8 linear
layers, checked against fp32 PyTorch.

The weight gradients accumulate IN PLACE into fp32 main_grad views that sit at offsets of one flat
buffer (parallel/grad_buffer.py), twice (two micro-batches); forward / dgrad GEMMs write into the
chunk views of the sequence-parallel pipelines (parallel_layers/sp.py).  Run in a fresh process with
the tuning mode set in the environment (the tuner reads it once):

    NXD_GEMM_TUNE=2 NXD_GEMM_NO_STREAMK=1 python tools/check_gemm_exhaustive.py --tokens 8192

Prints one JSON line per GEMM with the relative max error; exits 1 if any exceeds the tolerance.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuronx_distributed_llama3_2_amd.ops import gemm as G  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops._ext import ext  # noqa: E402

# Llama-3-8B at TP=8: (name, out features N, in features K) of each linear shard
SHAPES = [("qkv", 768, 4096), ("o_proj", 4096, 512), ("gate_up", 3584, 4096), ("down", 4096, 1792)]


def rel_err(got, ref):
    return float((got.double() - ref.double()).abs().max() / ref.double().abs().max().clamp(min=1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--tol", type=float, default=1e-2)
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    T = a.tokens
    # flat fp32 grad buffer, every main_grad view 64 B aligned (16 floats) but not 256 B
    sizes = [n * k for _, n, k in SHAPES]
    offs, o = [], 16
    for sz in sizes:
        offs.append(o)
        o += (sz + 15) // 16 * 16 + 16
    flat = torch.zeros(o, dtype=torch.float32, device=dev)
    C = ext()
    bad = 0
    for (name, N, K), off in zip(SHAPES, offs):
        mg = flat[off:off + N * K].view(N, K)
        mg.normal_()
        mg0 = mg.clone()
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        go = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        # weight gradient, in place: main_grad += go^T x, both production layouts (NT and the TN of
        # the transposed operands), two micro-batches
        gt, xt = go.t().contiguous(), x.t().contiguous()
        for _ in range(2):
            C.gemm(go.t(), x, mg, None, 1.0, 1.0)
        ref = mg0 + 2 * (go.float().t() @ x.float())
        e_nt = rel_err(mg, ref)
        mg.copy_(mg0)
        for _ in range(2):
            C.gemm(gt, xt.t(), mg, None, 1.0, 1.0)
        e_tn = rel_err(mg, ref)
        # forward into a chunk view of a larger output (sp.py gather_linear) and dgrad
        out = torch.empty(2 * T, N, device=dev, dtype=torch.bfloat16)
        G.linear(x, w, out=out[T:])
        e_fwd = rel_err(out[T:], x.float() @ w.float().t())
        dx = torch.empty(2 * T, K, device=dev, dtype=torch.bfloat16)
        C.gemm(go, w, dx[T:], None, 1.0, 0.0)
        e_dg = rel_err(dx[T:], go.float() @ w.float())
        torch.cuda.synchronize()
        errs = {"wgrad_nt": e_nt, "wgrad_tn": e_tn, "fwd": e_fwd, "dgrad": e_dg}
        ok = all(v <= a.tol for v in errs.values())
        bad += not ok
        print(json.dumps({"gemm": name, "tokens": T, "N": N, "K": K, "tune": os.environ.get("NXD_GEMM_TUNE", "1"),
                          "no_streamk": os.environ.get("NXD_GEMM_NO_STREAMK", "0"), "ok": ok,
                          **{k: round(v, 6) for k, v in errs.items()}}), flush=True)
    if os.environ.get("NXD_GEMM_LOG_TABLE"):
        for k, ms in C.gemm_tuned_entries():
            print(json.dumps({"key": k, "ms": ms}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
