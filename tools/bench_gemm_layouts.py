"""Which operand layouts does hipBLASLt run fastest for the three GEMMs of a linear layer?

For each Llama-3-8B TP=1 shape (8192 tokens) time, on random data, in one process:
  fwd    Y = X W^T                 (X [T,K], W [N,K]: both K-contiguous)
  dgrad  dX = dY W                 (as trained: W contraction dim is its row dim)
  dgradT dX = dY (W^T)^T           (with a K-major copy Wt [K,N] of the weight)
  wgrad  mg += dY^T X              (as trained: contraction over T = rows of both)
  wgradT mg += (dY^T) (X^T)^T      (with T-contiguous copies dYt [N,T], Xt [K,T])
  transpose costs of dY and X (what wgradT has to pay per micro-batch).
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from neuronx_distributed_llama3_2_amd.ops import ext  # noqa: E402


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


T = 8192
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096), "tp8_qkv": (768, 4096), "tp8_down": (4096, 1792), "tp8_gate_up": (3584, 4096)}
E = ext()
for name, (N, K) in shapes.items():
    x = torch.rand(T, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
    w = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
    g = torch.rand(T, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
    mg = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
    wt = w.t().contiguous()
    gt = g.t().contiguous()
    xt = x.t().contiguous()
    fl = 2.0 * T * N * K
    r = {"name": name, "N": N, "K": K}
    r["fwd_tf"] = fl / t(lambda: E.gemm(x, w.t(), y, None, 1.0, 0.0)) / 1e9
    r["dgrad_tf"] = fl / t(lambda: E.gemm(g, w, dx, None, 1.0, 0.0)) / 1e9
    r["dgradT_tf"] = fl / t(lambda: E.gemm(g, wt.t(), dx, None, 1.0, 0.0)) / 1e9
    r["wgrad_tf"] = fl / t(lambda: E.gemm(g.t(), x, mg, None, 1.0, 1.0)) / 1e9
    r["wgradT_tf"] = fl / t(lambda: E.gemm(gt, xt.t(), mg, None, 1.0, 1.0)) / 1e9
    r["wgrad_ms"] = fl / r["wgrad_tf"] / 1e9
    r["wgradT_ms"] = fl / r["wgradT_tf"] / 1e9
    r["transpose_g_ms_torch"] = t(lambda: gt.copy_(g.t()))
    r["transpose_g_ms"] = t(lambda: E.transpose_bf16(g, gt))
    r["transpose_x_ms"] = t(lambda: E.transpose_bf16(x, xt))
    r["transpose_g_tbs"] = 2 * g.numel() * 2 / r["transpose_g_ms"] / 1e9
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    del x, w, g, mg, y, dx, wt, gt, xt
    torch.cuda.empty_cache()
