"""Prefill-sized GEMMs (M = 32..512 tokens) of Llama-3.2-1B through the tuned hipBLASLt path:
time, TFLOP/s and effective weight-stream bandwidth (weights are read once per GEMM at best)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from neuronx_distributed_llama3_2_amd.ops import gemm  # noqa: E402


def t(fn, reps=50):
    """GPU time per call: `reps` calls captured in one hipGraph (eager back-to-back calls of these
    ~10 us GEMMs measure the host dispatch, ~28 us, not the GPU)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * reps)


shapes = {"qkv": (3072, 2048), "o": (2048, 2048), "gate_up": (16384, 2048), "down": (2048, 8192)}
for M in (32, 128, 512):
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ms = t(lambda: gemm.linear(x, w, out=y))
        print(json.dumps({"M": M, "proj": name, "N": N, "K": K, "us": round(ms * 1000, 2),
                          "tflops": round(2 * M * N * K / ms / 1e9, 1),
                          "weight_tb_s": round(N * K * 2 / ms / 1e9, 2)}), flush=True)
