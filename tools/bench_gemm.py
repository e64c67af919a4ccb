"""Tuned hipBLASLt GEMM (csrc/gemm.cpp) vs torch for the Llama-3-8B training shapes (TP=1, 8192 tokens)."""
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


T = 8192
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
for name, (N, K) in shapes.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    mg = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    fl = 2.0 * T * N * K
    r = {"name": name}
    r["fwd_torch"] = fl / t(lambda: torch.matmul(x, w.t())) / 1e9
    r["fwd_tuned"] = fl / t(lambda: gemm.linear(x, w)) / 1e9
    r["dgrad_torch"] = fl / t(lambda: torch.matmul(g, w)) / 1e9
    r["dgrad_tuned"] = fl / t(lambda: gemm.matmul(g, w)) / 1e9
    r["wgrad_torch"] = fl / t(lambda: torch.addmm(mg, g.t(), x, out_dtype=torch.float32, out=mg)) / 1e9
    r["wgrad_tuned"] = fl / t(lambda: gemm.wgrad_accumulate_(mg, g, x)) / 1e9
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    del x, w, g, mg
