"""GEMM-side cost of sequence-parallel chunking (parallel_layers/sp.py) at the per-rank Llama-3-8B
shapes of TP = 2 / 4 / 8: per-layer time of the chunked column/row forward GEMMs and backward dgrad
GEMMs for c = 1, 2, 4, 8 chunks (wgrad GEMMs are unchunked and excluded).  The communication side
of the trade-off needs the multi-GPU run; this isolates what chunking costs the matrix cores."""
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


S, H, I, Q, KV = 8192, 4096, 14336, 4096, 1024
for tp in (2, 4, 8):
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
        print(json.dumps({"tp": tp, "chunks": c, "layer_fwd_dgrad_ms": round(tot, 4)}), flush=True)
