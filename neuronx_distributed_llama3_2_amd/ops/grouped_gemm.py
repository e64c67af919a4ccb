"""Grouped (ragged-M) expert GEMMs for dropless MoE (csrc/grouped_gemm.hip) and the device-side
token permutation around them.

Tokens are sorted by their chosen expert on the device; expert e owns rows offs[e]:offs[e+1] of
the sorted activations.  Nothing here reads a group size on the host, so a dropless MoE layer has
no device->host sync (reference: modules/moe/expert_mlps.py:169-265, utils/tensor_utils.py:4-62).

GPU tensors run the HIP kernels (forward, input gradient and the fp32 weight gradient, which is
accumulated straight into `main_grad` when the flat gradient buffer provides one); CPU tensors run
the plain-PyTorch reference (per-expert matmuls over the host-known offsets).
"""

from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch

from ._ext import ext, use_native

# "grouped" (default): the device-side grouped kernel, no host sync (hipGraph-capturable).
# "loop": one hipBLASLt GEMM per expert (torch.matmul: its first heuristic -- the group sizes change
# every step, so the in-process tuner of ops/gemm.py would re-time every call) over host-read group
# sizes: one device->host sync per MoE layer, not capturable, but hipBLASLt's large-M tiles
# (Mixtral shapes, TP=1: fwd 1.08 vs 0.55 PF/s, dgrad 0.85 vs 0.65 / 1.33 vs 0.58, wgrad 0.58 vs 0.40;
# profiles/r2_moe_grouped_gemm_v1.jsonl; whole layer 37.0 vs 60.5 ms at 16k tokens,
# profiles/r2_moe_layer_v1.md).
# "auto": the loop, except while a hipGraph is being captured (no host read possible).
# Default "grouped": the MoE forward stays free of device->host syncs unless the user opts in.
MOE_GEMM = os.environ.get("NXD_MOE_GEMM", "grouped")


def host_group_bounds(offs: torch.Tensor) -> Optional[List[int]]:
    """Host copy of the group boundaries when the per-expert loop backend is selected, else None."""
    if not offs.is_cuda or MOE_GEMM == "grouped":
        return None
    if MOE_GEMM == "auto" and torch.cuda.is_current_stream_capturing():
        return None
    return offs.tolist()


def moe_permutation(expert_index: torch.Tensor, num_experts: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Stable sort of the T*k (token, choice) slots by expert, all on the device.

    Returns (order, inverse, offs): sorted slot s holds flat slot order[s] (token order[s] // k),
    flat slot i sits at sorted row inverse[i], and offs int32 [E + 1] are the group boundaries.
    """
    flat = expert_index.reshape(-1)
    order = torch.argsort(flat, stable=True)
    inverse = torch.empty_like(order)
    inverse.scatter_(0, order, torch.arange(order.numel(), device=order.device, dtype=order.dtype))
    counts = torch.zeros(num_experts, dtype=torch.int32, device=flat.device)
    counts.scatter_add_(0, flat.long(), torch.ones_like(flat, dtype=torch.int32))
    offs = torch.zeros(num_experts + 1, dtype=torch.int32, device=flat.device)
    offs[1:] = torch.cumsum(counts, 0, dtype=torch.int32)
    return order, inverse, offs


def grouped_linear_reference(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """y[offs[e]:offs[e+1]] = x[offs[e]:offs[e+1]] @ w[e] (fp32 accumulate), differentiable."""
    bounds = offs.tolist()
    outs = []
    for e in range(w.shape[0]):
        lo, hi = bounds[e], bounds[e + 1]
        if hi > lo:
            outs.append((x[lo:hi].float() @ w[e].float()).to(x.dtype))
    if not outs:
        return x.new_zeros(x.shape[0], w.shape[2]) + 0 * x.sum() * w.sum()
    y = torch.cat(outs, 0)
    if y.shape[0] < x.shape[0]:   # rows past offs[E] (none in a well-formed permutation)
        y = torch.cat([y, y.new_zeros(x.shape[0] - y.shape[0], y.shape[1])], 0)
    return y


def _loop_fwd(x, w, bounds, y):
    for e in range(w.shape[0]):
        lo, hi = bounds[e], bounds[e + 1]
        if hi > lo:
            torch.matmul(x[lo:hi], w[e], out=y[lo:hi])


def _loop_dgrad(dy, w, bounds, dx):
    dx[bounds[-1]:].zero_()
    for e in range(w.shape[0]):
        lo, hi = bounds[e], bounds[e + 1]
        if hi > lo:
            torch.matmul(dy[lo:hi], w[e].t(), out=dx[lo:hi])


def _loop_wgrad(x, dy, bounds, g, accumulate):
    if not accumulate:
        g.zero_()
    for e in range(g.shape[0]):
        lo, hi = bounds[e], bounds[e + 1]
        if hi > lo:
            torch.addmm(g[e], x[lo:hi].t(), dy[lo:hi], out_dtype=torch.float32, out=g[e])   # += x_e^T dy_e


class GroupedLinearFunc(torch.autograd.Function):
    """y = x @ W[e] per expert group; dx = dy @ W[e]^T; dW[e] = x_e^T dy_e (fp32)."""

    @staticmethod
    def forward(ctx, x, w, offs, bounds: Optional[List[int]] = None):
        x = x.contiguous()
        y = torch.empty(x.shape[0], w.shape[2], dtype=x.dtype, device=x.device)
        if bounds is not None:
            y[bounds[-1]:].zero_()
            _loop_fwd(x, w, bounds, y)
        else:
            ext().grouped_gemm(0, x, w, offs, y, False)
        ctx.bounds = bounds
        ctx.save_for_backward(x, w, offs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, offs = ctx.saved_tensors
        bounds = ctx.bounds
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            if bounds is not None:
                _loop_dgrad(dy, w, bounds, dx)
            else:
                ext().grouped_gemm(1, dy, w, offs, dx, False)

        def wgrad(g, accumulate):
            if bounds is not None:
                _loop_wgrad(x, dy, bounds, g, accumulate)
            else:
                ext().grouped_gemm(2, x, dy, offs, g, accumulate)

        dw = None
        if ctx.needs_input_grad[1]:
            mg = getattr(w, "main_grad", None)
            if mg is not None and mg.dtype == torch.float32 and mg.is_contiguous():
                wgrad(mg, True)
                cb = getattr(w, "_nxd_grad_ready", None)
                if cb is not None:
                    cb(w)
            else:
                g = torch.empty(w.shape, dtype=torch.float32, device=w.device)
                wgrad(g, False)
                if mg is not None:
                    mg.add_(g.to(mg.dtype))
                    cb = getattr(w, "_nxd_grad_ready", None)
                    if cb is not None:
                        cb(w)
                else:
                    dw = g.to(w.dtype)
        return dx, dw, None, None


def grouped_linear(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor,
                   bounds: Optional[List[int]] = None) -> torch.Tensor:
    """Expert-grouped linear over expert-sorted rows: x [M, K], w [E, K, N], offs int32 [E + 1].
    `bounds` (host list of offs) selects the per-expert hipBLASLt loop (NXD_MOE_GEMM=loop)."""
    if use_native(x, w, offs):
        if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
            raise TypeError("grouped_linear: the HIP kernel takes bf16 activations and weights")
        return GroupedLinearFunc.apply(x, w, offs, bounds)
    return grouped_linear_reference(x, w, offs)


# ---------------------------------------------------------------------------------------------
# dispatch gather / un-permute + combine around the expert GEMMs (csrc/moe_combine.hip)

class MoEDispatchFunc(torch.autograd.Function):
    """x_sorted = x[order // k]; backward dx[t] = sum_j dxs[inverse[t*k + j]] (gather-sum, no atomics)."""

    @staticmethod
    def forward(ctx, x, order, inverse, k):
        ctx.save_for_backward(inverse)
        ctx.k = k
        return x.index_select(0, order // k)

    @staticmethod
    def backward(ctx, dxs):
        (inverse,) = ctx.saved_tensors
        dxs = dxs.contiguous()
        dx = torch.empty(inverse.numel() // ctx.k, dxs.shape[1], dtype=dxs.dtype, device=dxs.device)
        ext().moe_combine_fwd(dxs, inverse, None, dx)
        return dx, None, None, None


class MoECombineFunc(torch.autograd.Function):
    """out[t] = sum_j aff[t, j] * ys[inverse[t*k + j]]; aff fp32 [T, k]."""

    @staticmethod
    def forward(ctx, ys, inverse, aff):
        ys = ys.contiguous()
        aff = aff.float().contiguous()
        T = aff.shape[0]
        out = torch.empty(T, ys.shape[1], dtype=ys.dtype, device=ys.device)
        ext().moe_combine_fwd(ys, inverse, aff, out)
        ctx.save_for_backward(ys, inverse, aff)
        return out

    @staticmethod
    def backward(ctx, dout):
        ys, inverse, aff = ctx.saved_tensors
        dys = torch.empty_like(ys)
        daff = torch.empty_like(aff)
        ext().moe_combine_bwd(dout.contiguous(), ys, inverse, aff, dys, daff)
        return dys, None, daff


def moe_dispatch(x: torch.Tensor, order: torch.Tensor, inverse: torch.Tensor, k: int) -> torch.Tensor:
    """Rows of x [T, H] in expert-sorted slot order (x[order // k]), [T*k, H]."""
    if use_native(x, order, inverse) and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0 and k <= 8:
        return MoEDispatchFunc.apply(x, order, inverse, k)
    return x.index_select(0, order // k)


def moe_unpermute_combine(ys: torch.Tensor, inverse: torch.Tensor, aff: torch.Tensor) -> torch.Tensor:
    """Un-permute the expert outputs ys [T*k, H] (sorted) and take the affinity-weighted sum over the
    k choices: out [T, H].  GPU: one fused kernel each way (the einsum it replaces ran as a batch-T
    batched GEMM); CPU: gather + einsum in the activation dtype."""
    T, k = aff.shape
    if use_native(ys, inverse, aff) and ys.dtype == torch.bfloat16 and ys.shape[1] % 8 == 0 and k <= 8:
        return MoECombineFunc.apply(ys, inverse, aff)
    y = ys.index_select(0, inverse).view(T, k, ys.shape[1])
    return torch.einsum("tkh,tk->th", y, aff.to(y.dtype))
