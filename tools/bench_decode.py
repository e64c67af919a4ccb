"""Decode-attention microbenchmark: per-call time inside a captured hipGraph (launch overhead out)."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from neuronx_distributed_llama3_2_amd import ops  # noqa: E402


def main():
    res = {"fused_merge": os.environ.get("NXD_DECODE_FUSED_MERGE", "1")}
    for (B, Hq, Hkv, D, L) in [(1, 32, 8, 64, 2320), (1, 32, 8, 64, 8192), (8, 32, 8, 64, 2320), (1, 32, 8, 128, 8192)]:
        kc = torch.randn(B, Hkv, L, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        q = torch.randn(B, 1, Hq, D, device="cuda", dtype=torch.bfloat16)
        seq = torch.full((B,), L - 20, device="cuda", dtype=torch.int32)
        out = torch.empty_like(q)
        ops.decode_attention(q, kc, vc, seq, out=out)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        N = 50
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g):
                for _ in range(N):
                    ops.decode_attention(q, kc, vc, seq, out=out)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / (5 * N)
        kv_bytes = 2 * B * Hkv * (L - 20) * D * 2
        res[f"B{B}_D{D}_L{L}"] = {"us": round(us, 2), "GBps": round(kv_bytes / us / 1e3, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
