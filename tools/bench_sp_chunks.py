"""GEMM-side cost of sequence-parallel chunking (parallel_layers/sp.py) at the per-rank Llama-3-8B
shapes of TP = 2 / 4 / 8: per-layer time of the chunked column/row forward GEMMs and backward dgrad
GEMMs for c = 1, 2, 4, 8 chunks (wgrad GEMMs are unchunked and excluded).  The communication side
of the trade-off needs the multi-GPU run; this isolates what chunking costs the matrix cores.

    python tools/bench_sp_chunks.py [--tp 8 --mbs 4]   (rows per rank-GEMM = mbs * 8192)"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from neuronx_distributed_llama3_2_amd.ops import gemm  # noqa: E402


def timed(fn, reps=20):
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
ap.add_argument("--tp", type=int, nargs="+", default=[2, 4, 8])
ap.add_argument("--mbs", type=int, default=1, help="sequences per micro-batch (GEMM rows = mbs * 8192)")
a = ap.parse_args()
S, H, I, Q, KV = 8192 * a.mbs, 4096, 14336, 4096, 1024
for tp in a.tp:
    # (name, N_out, K_in) of the per-rank weight [N, K]
    col = [("qkv", (Q + 2 * KV) // tp, H), ("gate_up", 2 * I // tp, H)]
    row = [("o", H, Q // tp), ("down", H, I // tp)]
    ws = {n: torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for n, N, K in col + row}
    for c in (1, 2, 4, 8):
        m = S // c
        tot = 0.0
        for n, N, K in col + row:
            x = torch.randn(S, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(S, N, device="cuda", dtype=torch.bfloat16)
            xv, ov = x.view(c, m, K), out.view(c, m, N)
            fwd = timed(lambda: [gemm.linear(xv[j], ws[n], out=ov[j]) for j in range(c)])
            gy = torch.randn(S, N, device="cuda", dtype=torch.bfloat16)
            gx = torch.empty(S, K, device="cuda", dtype=torch.bfloat16)
            gv, gxv = gy.view(c, m, N), gx.view(c, m, K)
            bwd = timed(lambda: [gemm.matmul(gv[j], ws[n], out=gxv[j]) for j in range(c)])
            tot += fwd + bwd
            print(json.dumps({"tp": tp, "chunks": c, "gemm": n, "fwd_ms": round(fwd, 4), "dgrad_ms": round(bwd, 4)}),
                  flush=True)
        print(json.dumps({"tp": tp, "mbs": a.mbs, "chunks": c, "layer_fwd_dgrad_ms": round(tot, 4)}), flush=True)
