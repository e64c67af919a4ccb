"""Sparse-MoE causal LM inference (Mixtral, DBRX) on the shared decoder inference forward
(reference: examples/inference/mixtral/neuron_modeling_mixtral.py, examples/inference/dbrx/
neuron_modeling_dbrx.py — both built on the MoE module with RouterTopK + ExpertMLPs).

The module IS the training `MixtralForCausalLM` (attention identical to Llama, MoE block from
modules/moe), so training checkpoints and converted HF weights load directly.  The MoE block picks
its dispatch per call, all with experts TP-sharded on the intermediate dim (one all-reduce after
the down projection, like a dense MLP):

* few (token, expert) pairs (T * top_k <= E: token generation) — *selective loading*: the
  expert-mode skinny GEMM (csrc/gemv.hip) reads only the chosen experts' weights, SwiGLU fused in
  its epilogue; static shapes, no host sync, captured in the decode hipGraph;
* small T under graph capture (batched decode / speculation) — every token through every expert
  as two batched GEMMs (each expert's weights read once, static shapes);
* prefill — tokens sorted by expert on the device, each expert multiplies only its own rows (the
  training path's grouped GEMM kernels, top_k / E of the dense work, no host sync).

To feed the skinny-GEMM kernel, the expert weights are stored output-major ([E, out, in] in
memory) while keeping their logical [E, in, out] parameter shapes (`post_load`).
DBRX differences handled here: LayerNorm without bias instead of RMSNorm (`norm_type`), QKV
clamped to +-clip_qkv, optional top-k renormalisation (models/mixtral/convert.py translates its
config and weights).
"""

from __future__ import annotations

import copy

import torch
import torch.nn.functional as F

from ..models.mixtral.modeling_mixtral import MixtralForCausalLM
from ..ops._ext import ext, use_native
from ..ops.gemv import expert_linear
from ..ops.grouped_gemm import moe_dispatch, moe_permutation, moe_unpermute_combine
from ..ops import swiglu
from .model_base import DecoderInferenceMixin

# below this many tokens a capture-safe dense all-experts dispatch is used outside selective loading
_DENSE_MAX_TOKENS = 64


class MoEInferenceModel(DecoderInferenceMixin, MixtralForCausalLM):
    def __init__(self, config, dtype=torch.bfloat16, device=None):
        cfg = copy.copy(config)
        cfg.sequence_parallel_enabled = False
        cfg.capacity_factor = None
        MixtralForCausalLM.__init__(self, cfg, dtype=dtype, device=device)
        self._init_inference(config)
        self.norm_type = getattr(config, "norm_type", "rmsnorm")
        self.clip_qkv = getattr(config, "clip_qkv", None)
        self.top_k = int(config.num_experts_per_tok)
        self.num_experts = int(config.num_local_experts)
        self.normalize_top_k = bool(getattr(config, "normalize_top_k_affinities", self.top_k > 1))
        if next(self.parameters()).device.type != "meta":
            self.post_load()

    # ------------------------------------------------------------------ weights
    def _expert_weights(self, layer):
        mo = layer.block_sparse_moe.expert_mlps.mlp_op
        return mo.gate_up_proj.weight, mo.down_proj.weight   # [E, H, 2I/tp], [E, I/tp, H]

    @torch.no_grad()
    def post_load(self) -> None:
        """Re-lay the expert weights output-major in memory (logical shapes unchanged)."""
        for layer in self.model.layers:
            for w in self._expert_weights(layer):
                if w.stride(-1) == 1 and w.shape[-1] > 1:
                    w.data = w.data.transpose(1, 2).contiguous().transpose(1, 2)

    # ------------------------------------------------------------------ block pieces
    def _qkv_hook(self, qkv: torch.Tensor) -> torch.Tensor:
        if self.clip_qkv is not None:
            qkv.clamp_(-float(self.clip_qkv), float(self.clip_qkv))
        return qkv

    def _norm(self, x, w, residual):
        if self.norm_type == "rmsnorm":
            return DecoderInferenceMixin._norm(self, x, w, residual)
        r = x if residual is None else x + residual
        y = F.layer_norm(r.float(), (r.shape[-1],), w.float(), None, self.eps).to(r.dtype)
        return y, r

    def _route(self, layer, x: torch.Tensor):
        router = layer.block_sparse_moe.router.linear_router
        logits = F.linear(x, router.weight.to(x.dtype))
        probs = torch.softmax(logits.float(), dim=-1)
        top_w, top_i = torch.topk(probs, self.top_k, dim=-1)
        if self.normalize_top_k:
            top_w = top_w / top_w.sum(-1, keepdim=True)
        return top_w, top_i

    def _ffn(self, layer, h: torch.Tensor) -> torch.Tensor:
        shape = h.shape
        x = h.reshape(-1, shape[-1])
        n, k, E = x.shape[0], self.top_k, self.num_experts
        top_w, top_i = self._route(layer, x)
        w_gu, w_d = self._expert_weights(layer)
        if n * k <= E:
            out = self._selective(x, top_w, top_i, w_gu, w_d)
        elif n <= _DENSE_MAX_TOKENS or (x.is_cuda and torch.cuda.is_current_stream_capturing()):
            out = self._all_experts(x, top_w, top_i, w_gu, w_d)
        else:
            out = self._grouped(x, top_w, top_i, w_gu, w_d)
        return self._all_reduce(out).view(shape)

    def _selective(self, x, top_w, top_i, w_gu, w_d):
        n, k = top_i.shape
        eidx = top_i.reshape(-1).to(torch.int32)
        a = expert_linear(x, w_gu.transpose(1, 2), eidx, xdiv=k, glu=True)   # [n*k, I/tp]
        y = expert_linear(a, w_d.transpose(1, 2), eidx, xdiv=1)             # [n*k, H] partial over TP
        return (y.view(n, k, -1).float() * top_w.unsqueeze(-1)).sum(1).to(x.dtype)

    def _all_experts(self, x, top_w, top_i, w_gu, w_d):
        E = self.num_experts
        gu = torch.matmul(x.unsqueeze(0), w_gu)                              # [E, n, 2I/tp]
        y = torch.matmul(swiglu(gu), w_d)                                    # [E, n, H]
        dense_w = torch.zeros(x.shape[0], E, dtype=torch.float32, device=x.device).scatter_(1, top_i, top_w)
        return torch.einsum("enh,ne->nh", y.float(), dense_w).to(x.dtype)

    def _grouped(self, x, top_w, top_i, w_gu, w_d):
        """Prefill: (token, choice) slots sorted by expert on the device, each expert multiplying only
        its own rows.  GPU bf16: the training path's sync-free kernels -- device-side permutation,
        dispatch gather, the grouped GEMMs (csrc/grouped_rowgemm.hip / grouped_gemm.hip) with the
        expert weights read output-major in place, SwiGLU, and the fused un-permute + affinity
        combine (csrc/moe_combine.hip); no host read of the group sizes, so a prefill graph can
        capture it.  Otherwise (CPU, fp32): per-expert matmuls over host-read group sizes.
        Reference: src/neuronx_distributed/modules/moe/expert_mlps.py:169-265."""
        if x.is_cuda and x.dtype == torch.bfloat16 and use_native(x) and x.shape[1] % 8 == 0 \
                and w_gu.shape[2] % 8 == 0 and top_i.shape[1] <= 8:
            return self._grouped_device(x, top_w, top_i, w_gu, w_d)
        n, k = top_i.shape
        flat = top_i.reshape(-1)
        order = torch.argsort(flat, stable=True)
        tok = order // k
        counts = torch.bincount(flat, minlength=self.num_experts).tolist()   # one host sync (prefill)
        xs = x.index_select(0, tok)
        ys = torch.empty((n * k, x.shape[1]), dtype=x.dtype, device=x.device)
        start = 0
        for e, c in enumerate(counts):
            if c:
                seg = xs[start:start + c]
                ys[start:start + c] = torch.matmul(swiglu(torch.matmul(seg, w_gu[e])), w_d[e])
                start += c
        ys = ys.float() * top_w.reshape(-1)[order].unsqueeze(1)
        out = torch.zeros((n, x.shape[1]), dtype=torch.float32, device=x.device)
        out.index_add_(0, tok, ys)
        return out.to(x.dtype)

    def _grouped_device(self, x, top_w, top_i, w_gu, w_d):
        n, k = top_i.shape
        order, inverse, offs = moe_permutation(top_i, self.num_experts)
        xs = moe_dispatch(x, order, inverse, k)                       # [n*k, H], expert-sorted rows
        gu = _grouped_mm(xs, w_gu, offs)                              # [n*k, 2I/tp]
        ys = _grouped_mm(swiglu(gu), w_d, offs)                       # [n*k, H] partial over TP
        return moe_unpermute_combine(ys, inverse, top_w.float())      # [n, H]


def _grouped_mm(x: torch.Tensor, w: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """y[rows of e] = x[rows of e] @ w[e] for logical w [E, K, N], read in its stored layout: the
    grouped kernel's forward mode for [E, K, N]-contiguous weights, its input-gradient mode (x @ W^T)
    for the output-major [E, N, K] storage `post_load` gives the expert weights."""
    y = torch.empty(x.shape[0], w.shape[2], dtype=x.dtype, device=x.device)
    if w.is_contiguous():
        ext().grouped_gemm(0, x.contiguous(), w, offs, y, False)
    else:
        ext().grouped_gemm(1, x.contiguous(), w.transpose(1, 2).contiguous(), offs, y, False)
    return y
