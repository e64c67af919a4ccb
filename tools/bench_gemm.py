"""Tuned hipBLASLt GEMM (csrc/gemm.cpp) vs torch for the Llama-3-8B training shapes at TP=N per-rank
shapes (N, K divided by TP; tokens = micro-batch x 8192 after the sequence-parallel all-gather).

    python tools/bench_gemm.py [--tp 8 --tokens 32768]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from neuronx_distributed_llama3_2_amd.ops import gemm  # noqa: E402


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


ap = argparse.ArgumentParser()
ap.add_argument("--tp", type=int, default=1)
ap.add_argument("--tokens", type=int, default=8192)
a = ap.parse_args()
T, tp = a.tokens, a.tp
shapes = {"qkv": (6144 // tp, 4096), "o": (4096, 4096 // tp), "gate_up": (28672 // tp, 4096),
          "down": (4096, 14336 // tp), "lm_head": (128256 // tp, 4096)}
for name, (N, K) in shapes.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    mg = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    fl = 2.0 * T * N * K
    r = {"name": name, "tp": tp, "tokens": T, "N": N, "K": K}
    r["fwd_torch"] = fl / t(lambda: torch.matmul(x, w.t())) / 1e9
    r["fwd_tuned"] = fl / t(lambda: gemm.linear(x, w)) / 1e9
    r["dgrad_torch"] = fl / t(lambda: torch.matmul(g, w)) / 1e9
    r["dgrad_tuned"] = fl / t(lambda: gemm.matmul(g, w)) / 1e9
    r["dgrad_path"] = fl / t(lambda: gemm.dgrad(g, w)) / 1e9
    r["wgrad_torch"] = fl / t(lambda: torch.addmm(mg, g.t(), x, out_dtype=torch.float32, out=mg)) / 1e9
    r["wgrad_tuned"] = fl / t(lambda: gemm.wgrad_accumulate_(mg, g, x)) / 1e9
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    del x, w, g, mg
