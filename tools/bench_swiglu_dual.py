"""Time the dual-layout SwiGLU backward vs the plain backward + separate transpose at the
Llama-3-8B gate_up shape (T=8192, I=14336) and the TP=8 shard (I=1792).  One JSON line per shape.
NXD_SWIGLU_DUAL_ROWS (64 | 128) picks the tile height of the dual kernel (read once per process)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuronx_distributed_llama3_2_amd.ops._ext import ext  # noqa: E402


def _time(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3   # us


def main():
    C = ext()
    for T, I in ((8192, 14336), (8192, 1792), (32768, 1792)):
        gu = torch.randn(T, 2 * I, device="cuda", dtype=torch.bfloat16)
        dh = torch.randn(T, I, device="cuda", dtype=torch.bfloat16)
        dgu = torch.empty_like(gu)
        dgu_t = torch.empty(2 * I, T, device="cuda", dtype=torch.bfloat16)
        dual = _time(lambda: C.swiglu_bwd_dual(gu, dh, dgu, dgu_t))
        plain = _time(lambda: C.swiglu_bwd(gu, dh, dgu))
        tr = _time(lambda: C.transpose_bf16(dgu, dgu_t))
        h = torch.empty_like(dh)
        h_t = torch.empty(I, T, device="cuda", dtype=torch.bfloat16)
        fdual = _time(lambda: C.swiglu_fwd_dual(gu, h, h_t))
        fplain = _time(lambda: C.swiglu_fwd(gu, h))
        ftr = _time(lambda: C.transpose_bf16(h, h_t))
        gb = (gu.numel() + dh.numel() + 2 * dgu.numel()) * 2 / 1e9
        print(json.dumps({"T": T, "I": I, "rows_tile": int(os.environ.get("NXD_SWIGLU_DUAL_ROWS", "128")),
                          "dual_us": round(dual, 1), "dual_TBps": round(gb / dual * 1e6 / 1e3, 2),
                          "plain_bwd_us": round(plain, 1), "transpose_us": round(tr, 1),
                          "saved_us": round(plain + tr - dual, 1), "fwd_dual_us": round(fdual, 1),
                          "fwd_plain_us": round(fplain, 1), "fwd_transpose_us": round(ftr, 1),
                          "fwd_saved_us": round(fplain + ftr - fdual, 1)}), flush=True)


if __name__ == "__main__":
    main()
