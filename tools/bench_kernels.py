"""Micro-benchmarks of the hand-written kernels at the headline (Llama-3-8B) shapes.

Prints one JSON line per kernel: time, achieved TFLOP/s or TB/s.  Used for the profiles/ summaries.
    python tools/bench_kernels.py [--only fa]
"""

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def emit(**kw):
    print(json.dumps(kw), flush=True)


def bench_fa(S=8192, B=1, Hq=32, Hkv=8, D=128, sdpa=True):
    dev = "cuda"
    q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
    flops_f = 4 * B * Hq * S * S * D / 2  # causal
    t = timeit(lambda: ops.flash_attn_fwd_lse(q, k, v, causal=True))
    emit(kernel="flash_fwd", S=S, Hq=Hq, Hkv=Hkv, D=D, ms=t, tflops=flops_f / t / 1e9)
    qg, kg, vg = (x.clone().requires_grad_(True) for x in (q, k, v))
    o = ops.flash_attn_func(qg, kg, vg, causal=True)
    do = torch.randn_like(o)

    def bwd():
        torch.autograd.grad(o, (qg, kg, vg), do, retain_graph=True)

    t = timeit(bwd, iters=10)
    emit(kernel="flash_bwd", S=S, Hq=Hq, Hkv=Hkv, D=D, ms=t, tflops=2.5 * flops_f / t / 1e9)
    # vendor SDPA for context (not used by the framework)
    if not sdpa:
        return
    try:
        qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2).repeat_interleave(Hq // Hkv, 1), v.transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
        t = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True))
        emit(kernel="torch_sdpa_fwd_reference_only", S=S, ms=t, tflops=flops_f / t / 1e9)
    except Exception as ex:  # pragma: no cover
        emit(kernel="torch_sdpa_fwd_reference_only", error=str(ex)[:200])


def bench_fa_fused_layout(S=8192, B=1, Hq=32, Hkv=8, D=128):
    """FA on strided views of a fused [S, B, (Hq+2Hkv)*D] QKV buffer (the training model's layout)."""
    from neuronx_distributed_llama3_2_amd.ops.flash_attn import _views

    qkv = torch.randn(S, B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = _views(qkv, Hq, Hkv, D)
    flops_f = 4 * B * Hq * S * S * D / 2
    t = timeit(lambda: ops.flash_attn_fwd_lse(q, k, v, causal=True))
    emit(kernel="flash_fwd_fused_qkv_layout", S=S, D=D, ms=t, tflops=flops_f / t / 1e9)
    qg, kg, vg = (x.detach().requires_grad_(True) for x in (q, k, v))
    o = ops.flash_attn_func(qg, kg, vg, causal=True)
    do = torch.randn_like(o)
    t = timeit(lambda: torch.autograd.grad(o, (qg, kg, vg), do, retain_graph=True), iters=10)
    emit(kernel="flash_bwd_fused_qkv_layout", S=S, D=D, ms=t, tflops=2.5 * flops_f / t / 1e9)


def bench_gemm():
    dev = "cuda"
    for (M, K, N, name) in [(8192, 4096, 6144, "qkv"), (8192, 4096, 4096, "o_proj"), (8192, 4096, 28672, "gate_up"),
                            (8192, 14336, 4096, "down"), (8192, 4096, 128256, "lm_head")]:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: torch.matmul(a, w.t()), iters=10)
        emit(kernel="hipblaslt_gemm", name=name, M=M, K=K, N=N, ms=t, tflops=2 * M * K * N / t / 1e9)
    # fp32-accumulating weight-grad GEMM (main_grad fusion)
    a = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(8192, 6144, device=dev, dtype=torch.bfloat16)
    mg = torch.zeros(6144, 4096, device=dev)
    try:
        t = timeit(lambda: torch.addmm(mg, dy.t(), a, out_dtype=torch.float32, out=mg), iters=10)
        emit(kernel="wgrad_addmm_fp32acc", ms=t, tflops=2 * 8192 * 4096 * 6144 / t / 1e9)
    except Exception as ex:
        emit(kernel="wgrad_addmm_fp32acc", error=str(ex)[:300])


def bench_mem():
    dev = "cuda"
    N, H = 8192, 4096
    x = torch.randn(N, H, device=dev, dtype=torch.bfloat16)
    r = torch.randn(N, H, device=dev, dtype=torch.bfloat16)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.rms_norm(x, w, 1e-5, residual=r))
    emit(kernel="rmsnorm_fwd_residual", ms=t, tbps=4 * N * H * 2 / t / 1e9)
    gu = torch.randn(N, 2 * 14336, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.swiglu(gu))
    emit(kernel="swiglu_fwd", ms=t, tbps=3 * N * 14336 * 2 / t / 1e9)
    logits = torch.randn(N, 128256, device=dev, dtype=torch.bfloat16)
    labels = torch.randint(0, 128256, (N,), device=dev)
    t = timeit(lambda: ops.vocab_parallel_cross_entropy(logits, labels), iters=5)
    emit(kernel="xent_fwd", ms=t, tbps=N * 128256 * 2 / t / 1e9)
    n = 8_030_000_000 // 8
    p = torch.zeros(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    g = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    p16 = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.adamw_flat_(p, g, m, v, p16, 1e-4, 0.9, 0.95, 1e-8, 0.1, 1), iters=5)
    emit(kernel="adamw_flat_1B", ms=t, tbps=n * (2 + 12 + 12 + 2) / t / 1e9)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="all")
    a = ap.parse_args()
    torch.manual_seed(0)
    if a.only in ("all", "fa"):
        bench_fa()
        bench_fa_fused_layout()
        bench_fa(S=4096, Hq=32, Hkv=8, D=64)
    if a.only in ("all", "fa", "fa_tp"):
        # per-GPU attention shapes of Llama-3-8B under TP = 2 / 4 / 8 (heads sharded)
        for tp in (2, 4, 8):
            bench_fa(Hq=32 // tp, Hkv=8 // tp, sdpa=False)
    if a.only in ("all", "gemm"):
        bench_gemm()
    if a.only in ("all", "mem"):
        bench_mem()
