"""GEMM entry points of the linear layers (csrc/gemm.cpp: hipBLASLt with per-shape autotuning).

`linear(x, w)` = x @ w^T, `matmul(a, b)` = a @ b, `wgrad_accumulate_(mg, go, x)` does
mg += go^T @ x with bf16 operands accumulating into the fp32 `main_grad` in place (one GEMM with
beta = 1, no bf16 temporary).  On CPU, or with NXD_TUNED_GEMM=0, they fall back to torch.
"""

from __future__ import annotations

import os

import torch

from ._ext import ext, use_native

_ENABLED = os.environ.get("NXD_TUNED_GEMM", "1") == "1"


def set_overlap_safe(enabled: bool) -> None:
    """Select GEMM solutions without stream-K (csrc/gemm.cpp `no_streamk`): a persistent stream-K
    GEMM stalls while a concurrent collective holds one of its CUs.  Multi-rank training turns it
    on with NXD_GEMM_NO_STREAMK=1 (parallel_state.initialize_model_parallel)."""
    if not torch.cuda.is_available():
        return
    try:
        ext().gemm_set_no_streamk(1 if enabled else 0)
    except Exception:  # extension not built (CPU-only environments)
        pass


def _native(*t: torch.Tensor) -> bool:
    return _ENABLED and use_native(*t) and all(x.dtype in (torch.bfloat16, torch.float16) for x in t)


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, out: torch.Tensor = None) -> torch.Tensor:
    """x [..., K] @ w[N, K]^T -> [..., N] (written into `out` if given: contiguous [..., N])."""
    shape = x.shape[:-1] + (w.shape[0],)
    if _native(x, w) and x.stride(-1) == 1:
        x2 = x.reshape(-1, x.shape[-1])
        y = out if out is not None else torch.empty(shape, dtype=x.dtype, device=x.device)
        ext().gemm(x2, w.t(), y.view(-1, w.shape[0]), None, 1.0, 0.0)
        return y + bias if bias is not None else y
    y = torch.nn.functional.linear(x, w, bias)
    if out is not None:
        out.copy_(y)
        return out
    return y


def matmul(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """a [..., K] @ b [K, N] -> [..., N] (written into `out` if given: contiguous [..., N])."""
    shape = a.shape[:-1] + (b.shape[1],)
    if _native(a, b) and a.stride(-1) == 1:
        a2 = a.reshape(-1, a.shape[-1])
        y = out if out is not None else torch.empty(shape, dtype=a.dtype, device=a.device)
        ext().gemm(a2, b, y.view(-1, b.shape[1]), None, 1.0, 0.0)
        return y
    y = torch.matmul(a, b)
    if out is not None:
        out.copy_(y)
        return out
    return y


_WGRAD_BF16 = os.environ.get("NXD_WGRAD_BF16", "0") == "1"
_scratch = {}


# wgrad through transposed operands pays when the GEMM time saved beats the two transposes
# (~0.8e-12 * T*(N+K) s): measured, N*K/(N+K) above ~1200 -- Llama-3-8B gate_up, down, qkv and
# lm_head at TP=1; gate_up (975 -> 1116 TF/s), down (920 -> 944) and lm_head at TP=8, but not the
# TP=8 qkv / o shards (798 -> 566, 742 -> 440; profiles/r2_gemm_tp8_wgrad_layouts.jsonl).
# NXD_WGRAD_T=0 disables, =2 forces.
_WGRAD_T = os.environ.get("NXD_WGRAD_T", "1")


def _use_wgrad_t(go2: torch.Tensor, x2: torch.Tensor = None, K: int = None) -> bool:
    """TN layout for this wgrad?  x2 = None: the caller holds a contiguous token-major copy of x
    with K rows (only go2's strides matter)."""
    if _WGRAD_T == "0" or _WGRAD_BF16:
        return False
    T, N = go2.shape[0], go2.shape[1]
    K = x2.shape[1] if x2 is not None else K
    if T % 8 or N % 8 or K % 8 or go2.stride(-1) != 1 or go2.stride(0) % 8:
        return False
    if x2 is not None and (x2.stride(-1) != 1 or x2.stride(0) % 8):
        return False
    return _WGRAD_T == "2" or N * K / (N + K) > 1200


# Hand-written weight-gradient kernel (csrc/wgrad_gemm.hip): reads both token-major operands with
# the hardware transpose read and splits the token range over workgroups.  Measured against this
# module's hipBLASLt path (profiles/r3_wgrad_kernel_vs_hipblaslt.jsonl): faster on the skinny
# tensor-parallel shards -- TP=8 qkv 984 vs 743 TF/s, o 880 vs 717 (M*N/(M+N) < 1100) -- and
# 5-13 % slower than the bare TN GEMM on the large TP=1 shapes.  Counting the TN path's two operand
# transposes the isolated kernel should also win TP=1 qkv / o_proj, but inside the TP=1 step that
# routing measured +4.6 ms per 2 micro-batches (GEMM + wgrad kernel + transposes 531.9 vs 527.3 ms,
# profiles/r3_step_breakdown_wgrad_all_nocopy_rejected.txt), so `auto` keeps the skinny rule.  With
# the ping-pong main loop (profiles/r3_wgrad_pp_vs_hipblaslt.jsonl) the kernel also takes the
# vocabulary-sized output (lm_head) when no producer wrote a feature-major copy: TP=8 1201 vs 1074
# TF/s for the hipBLASLt path and its two transposes (the 1 GiB logits gradient), TP=1 a tie.
# NXD_WGRAD_KERNEL = auto | 1 (whenever the shapes allow) | 0.
_WG_KERNEL = os.environ.get("NXD_WGRAD_KERNEL", "auto")
_WG_SKINNY = 1100.0
_WG_WIDE = 16000


def _use_wgrad_kernel(mg: torch.Tensor, go2: torch.Tensor, x2: torch.Tensor, has_copy: bool = False) -> bool:
    if _WG_KERNEL == "0" or x2 is None or not _native(go2, x2) or mg.dtype != torch.float32:
        return False
    T, M = go2.shape
    N = x2.shape[1]
    if T % 32 or M % 8 or N % 8 or go2.stride(1) != 1 or x2.stride(1) != 1 or mg.stride(1) != 1:
        return False
    if go2.stride(0) % 8 or x2.stride(0) % 8 or go2.data_ptr() % 16 or x2.data_ptr() % 16:
        return False
    return _WG_KERNEL == "1" or M * N / (M + N) < _WG_SKINNY or (not has_copy and max(M, N) >= _WG_WIDE)


# The hand-written dense GEMM (csrc/dense_gemm.hip) in its TN form reads the token-major dy / x
# directly (no transposes) and adds into the fp32 main_grad: one read-modify-write per element when
# a single K split fills the chip, split-K float atomics otherwise.  Measured against this module's
# other routes at the Llama-3-8B shapes (profiles/r6_dense_gemm_pipes_vs_hipblaslt.jsonl, T = 8192 /
# 65536): it wins every TP=8 shard -- qkv 1018 vs 880 TF/s, o_proj 1005 vs 904, gate_up 1180 vs 1164,
# down 1073 vs 961 -- and the TP=1 o_proj (1236 vs 1092, whose hipBLASLt route transposes both
# operands), and loses the wide TP=1 shapes to hipBLASLt's TN GEMM on producer-written copies
# (qkv 955 vs 1070, gate_up 1130 vs 1195, down 1063 vs 1152).  Rule: no producer copy, and
# M N / (M + N) < 2200.  NXD_DENSE_WGRAD = auto | 1 (whenever the shapes allow) | 0.
_DENSE_WG = os.environ.get("NXD_DENSE_WGRAD", "auto")
_DENSE_WG_SKINNY = 2200.0


def _use_dense_wgrad(mg: torch.Tensor, go2: torch.Tensor, x2, has_copy: bool) -> bool:
    if _DENSE_WG == "0" or x2 is None or not _native(go2, x2) or mg.dtype != torch.float32:
        return False
    T, M = go2.shape
    N = x2.shape[1]
    if T % 64 or M % 8 or N % 8 or go2.stride(1) != 1 or x2.stride(1) != 1 or mg.stride(1) != 1:
        return False
    if go2.stride(0) % 8 or x2.stride(0) % 8 or mg.stride(0) % 4:
        return False
    if go2.data_ptr() % 16 or x2.data_ptr() % 16 or mg.data_ptr() % 16:
        return False
    return _DENSE_WG == "1" or (not has_copy and M * N / (M + N) < _DENSE_WG_SKINNY)


def _dense_wgrad(mg: torch.Tensor, go2: torch.Tensor, x2: torch.Tensor) -> None:
    C = ext()
    T, M = go2.shape
    splits = C.dense_gemm_splits(M, x2.shape[1], T)
    C.dense_gemm(1, 1 if splits == 1 else 2, go2, x2, mg, splits)


def _wgrad_scratch(n: int, dtype, device, tag: str = "") -> torch.Tensor:
    # one buffer per stream: the two halves of parallel_layers/stream_split.py transpose concurrently
    sid = torch.cuda.current_stream(device).stream_id if torch.device(device).type == "cuda" else 0
    key = (dtype, str(device), tag, sid)
    t = _scratch.get(key)
    if t is None or t.numel() < n:
        t = _scratch[key] = torch.empty(n, dtype=dtype, device=device)
    return t[:n]


def wgrad_accumulate_(mg: torch.Tensor, go2: torch.Tensor, x2, go_t: torch.Tensor = None,
                      x_t: torch.Tensor = None) -> None:
    """mg [N, K] (fp32) += go2[T, N]^T @ x2[T, K].

    `go_t` / `x_t`: optional contiguous [N, T] / [K, T] copies of go2 / x2 already written by their
    producers (the SwiGLU backward / forward), used instead of transposing when the TN layout is
    taken.  x2 may be None when only x_t was kept.

    Default: one hipBLASLt GEMM with fp32 C/D and beta = 1.  NXD_WGRAD_BF16=1: bf16-output GEMM
    into a reused scratch, then an fp32 add (the per-micro-batch weight gradient is rounded to
    bf16 before the fp32 accumulation — the precision of the reference's XLA matmul + fp32
    grad accumulation; hipBLASLt's bf16-output solutions run faster than its fp32-output ones)."""
    has_copy = go_t is not None or x_t is not None
    if _use_dense_wgrad(mg, go2, x2, has_copy):
        _dense_wgrad(mg, go2, x2)
        return
    if _use_wgrad_kernel(mg, go2, x2, has_copy=has_copy):
        ext().wgrad_gemm(mg, go2, x2, 0)
        return
    if x_t is not None and not (x_t.dim() == 2 and x_t.is_contiguous() and x_t.shape[1] == go2.shape[0]):
        x_t = None
    if x2 is None and not (x_t is not None and _native(go2, x_t) and mg.is_contiguous()
                           and _use_wgrad_t(go2, K=x_t.shape[0])):
        x2 = x_t.t().contiguous()   # only the token-major copy was kept and the TN path is off
        x_t = None
    if x2 is None or (_native(go2, x2) and mg.is_contiguous()):
        if x2 is None or _use_wgrad_t(go2, x2):
            # T-contiguous operands: both transposed by the HIP kernel (~5 TB/s) into scratch, then
            # the TN GEMM (1.30-1.44 vs 1.06-1.16 PF/s on the NT layout, profiles/r2_gemm_layouts)
            T, N = go2.shape[0], go2.shape[1]
            K = x_t.shape[0] if x_t is not None else x2.shape[1]
            if go_t is not None and go_t.shape == (N, T) and go_t.is_contiguous() and go_t.dtype == go2.dtype:
                gt = go_t
            else:
                gt = transpose(go2, out=_wgrad_scratch(N * T, go2.dtype, go2.device, "gt").view(N, T))
            xt = x_t if x_t is not None else transpose(x2, out=_wgrad_scratch(K * T, x2.dtype, x2.device, "xt").view(K, T))
            ext().gemm(gt, xt.t(), mg, None, 1.0, 1.0)
            return
        if _WGRAD_BF16:
            tmp = _wgrad_scratch(mg.numel(), go2.dtype, go2.device).view(mg.shape)
            ext().gemm(go2.t(), x2, tmp, None, 1.0, 0.0)
            mg.add_(tmp)
            return
        ext().gemm(go2.t(), x2, mg, None, 1.0, 1.0)
        return
    if go2.is_cuda:
        torch.addmm(mg, go2.t(), x2, out_dtype=torch.float32, out=mg)
    else:
        mg.add_(go2.t().float().matmul(x2.float()))


# ----------------------------------------------------------------------------- dgrad layout
# hipBLASLt runs dX = dY W (W [N, K] row-major: the contraction dim is W's row dim) at 1.31-1.44
# PF/s on the Llama-3-8B shapes but at 1.56-1.69 PF/s when W is stored K-major (W^T [K, N]
# contiguous; profiles/r2_gemm_layouts.jsonl).  Training therefore keeps a K-major copy of every
# weight it back-propagates through, refreshed lazily by the first backward after the weights
# changed (one transpose per weight per optimizer step, HBM-bound, vs a faster dgrad in every
# micro-batch).  Staleness is detected by the optimizer's weight epoch (bumped by every optimizer
# step and checkpoint load that writes the weights outside autograd) plus the tensor's own
# version counter and storage pointer (any in-place torch write).  NXD_DGRAD_WT=0 disables it.
_DGRAD_WT = os.environ.get("NXD_DGRAD_WT", "1") == "1"
_weight_epoch = [0]


def weights_updated() -> None:
    """Tell the GEMM layer that weights were rewritten behind autograd's back (optimizer step)."""
    _weight_epoch[0] += 1


def transpose(src: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """[R, C] -> contiguous [C, R] (HIP tiled transpose for bf16; torch elsewhere)."""
    dst = out if out is not None else torch.empty((src.shape[1], src.shape[0]), dtype=src.dtype, device=src.device)
    if use_native(src) and src.dtype == torch.bfloat16 and src.stride(-1) == 1 and src.shape[0] % 8 == 0 \
            and src.shape[1] % 8 == 0 and src.stride(0) % 8 == 0:
        ext().transpose_bf16(src, dst)
    else:
        dst.copy_(src.t())
    return dst


def _kmajor(weight: torch.Tensor) -> torch.Tensor:
    key = (_weight_epoch[0], weight._version, weight.data_ptr())
    wt = getattr(weight, "_nxd_wt", None)
    cur = torch.cuda.current_stream(weight.device)
    if wt is None or getattr(weight, "_nxd_wt_key", None) != key:
        if wt is None or wt.shape != (weight.shape[1], weight.shape[0]):
            wt = torch.empty((weight.shape[1], weight.shape[0]), dtype=weight.dtype, device=weight.device)
        transpose(weight.detach(), out=wt)
        weight._nxd_wt = wt
        weight._nxd_wt_key = key
        weight._nxd_wt_ev = torch.cuda.Event()
        weight._nxd_wt_ev.record(cur)
        weight._nxd_wt_stream = cur.stream_id
    elif getattr(weight, "_nxd_wt_stream", cur.stream_id) != cur.stream_id:
        # written on another stream (the other half of stream_split): wait for the transpose
        cur.wait_event(weight._nxd_wt_ev)
        wt.record_stream(cur)
    return wt


def dgrad(go: torch.Tensor, weight: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """dX = go [..., N] @ weight [N, K] -> [..., K] (the input gradient of y = x W^T)."""
    if _DGRAD_WT and _native(go, weight) and go.stride(-1) == 1 and weight.dim() == 2 and weight.shape[0] % 8 == 0 \
            and weight.shape[1] % 8 == 0 and weight.is_contiguous():
        wt = _kmajor(weight)
        return matmul(go, wt.t(), out=out)
    return matmul(go, weight, out=out)
