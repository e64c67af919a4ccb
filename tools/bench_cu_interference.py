"""How much does a concurrent collective slow the GEMMs it overlaps with?  One MI355X: a hipBLASLt
GEMM of the TP=8 sequence-parallel shapes on the compute stream while a copy kernel occupying K
workgroups (RCCL runs one workgroup per channel, streaming HBM) runs on a side stream for longer
than the GEMM.  Prints the GEMM time per K relative to K = 0 (JSON lines).

    python tools/bench_cu_interference.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.ops._ext import ext  # noqa: E402

C = ext()
SHAPES = [("gate_up_fwd_tp8", 32768, 4096, 3584), ("o_fwd_tp8", 32768, 512, 4096), ("qkv_fwd_tp8", 32768, 4096, 768),
          ("wgrad_kernel_gate_up_tp8", 32768, 4096, 3584), ("flash_attn_fwd_tp8", 4, 8192, 4)]
BLOCKS = [0, 4, 16, 64, 128]


def main():
    side = torch.cuda.Stream()
    hog_bytes = 1 << 30
    src = torch.empty(hog_bytes // 4, dtype=torch.float32, device="cuda").uniform_()
    dst = torch.empty_like(src)
    for name, M, K, N in SHAPES:
        if name.startswith("flash"):
            from neuronx_distributed_llama3_2_amd import ops

            q = torch.randn(M, K, N, 128, device="cuda", dtype=torch.bfloat16)
            kv = torch.randn(M, K, 1, 128, device="cuda", dtype=torch.bfloat16)
            gemm = lambda: ops.flash_attn_fwd_lse(q, kv, kv, causal=True)  # noqa: E731
        elif name.startswith("wgrad"):
            dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            mg = torch.zeros(N, K, device="cuda", dtype=torch.float32)
            gemm = lambda: C.wgrad_gemm(mg, dy, x, 0)  # noqa: E731
        else:
            a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            gemm = lambda: C.gemm(a, w.t(), y, None, 1.0, 0.0)  # noqa: E731
        for _ in range(3):
            gemm()
        torch.cuda.synchronize()
        base = None
        for blocks in BLOCKS:
            times = []
            for _ in range(5):
                if blocks:
                    # copy kernel for ~3x the GEMM reps' time (100 MHz ticks), started first
                    ticks = int(max(base or 1.0, 0.2) * 5 * 3 * 1e5)
                    with torch.cuda.stream(side):
                        C.cu_stream(src, dst, min(hog_bytes // blocks, 8 << 20) // 16 * 16, blocks, ticks)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    gemm()
                e.record()
                torch.cuda.synchronize()
                times.append(s.elapsed_time(e) / 5)
            t = sorted(times)[len(times) // 2]
            base = base or t
            print(json.dumps({"kernel": name, "M": M, "K": K, "N": N, "side_workgroups": blocks, "ms": round(t, 4),
                              "slowdown": round(t / base, 3)}), flush=True)
        # the side kernel alone for the same number of workgroups: bytes/s it moved
        del gemm


if __name__ == "__main__":
    main()
