"""Shared inference forward for decoder-only causal LMs on the framework's training modules
(reference: examples/inference/modules/model_base.py:334-451 `NeuronBaseModel.forward`).

* context encoding (prefill, T tokens per sequence): fused residual+RMSNorm kernel -> one fused
  QKV GEMM -> in-place RoPE on the q/k columns of that buffer (one launch for both) -> in-place
  KV-cache write -> causal flash attention (flash_attn_fwd.hip) on strided views -> o_proj
  (+ TP all-reduce) -> add+norm -> feed-forward block (dense SwiGLU or MoE) -> final norm and
  lm_head on the last valid position of every sequence only;
* token generation (T = 1, or T = speculation length): same block with the flash-decoding
  kernel (inference.hip) reading the KV cache up to a per-sequence DEVICE length, so a decode
  step has static shapes and no host sync — it is captured into hipGraphs (inference/graphs.py).

Decode fast path (TP = 1, bf16 weights, <= 8 new tokens): each projection is one fused GEMV
(csrc/decode_fused.hip) that also does the surrounding element-wise work -- RMSNorm prologues,
RoPE + KV-cache write after QKV, residual adds after o_proj / down -- so a layer is 5 launches
(QKV, attention, o_proj, gate_up, down) instead of 10 (`NXD_DECODE_FUSED=0` disables it).

KV cache: ONE allocation [layers, 2, max_batch, kv_heads_local, max_len, head_dim] (bf16);
`seq_ids` selects cache rows (continuous batching).
"""

from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops
from ..ops.gemm import linear as _linear
from ..ops.gemv import skinny_linear
from ..parallel_layers import parallel_state as ps
from ..parallel_layers.parallel_state import get_tensor_model_parallel_size

# Fused decode: MiB of the gate_up weight (after all of o_proj) that the attention launch streams
# into the Infinity Cache from spare workgroups (0 disables), and how many workgroups do it.
_PREFETCH_MB = float(os.environ.get("NXD_DECODE_PREFETCH_MB", "0"))
_PREFETCH_WGS = int(os.environ.get("NXD_DECODE_PREFETCH_WGS", "256"))
# decode attention + o_proj in one launch (csrc/decode_attn.hip FUSE); the o_proj sum reaches the
# residual stream through the next two fused GEMVs (xadd / yadd side inputs).  Its rows are summed
# with fp32 atomics, so the low bits of a token's logits -- and rarely a greedy near-tie -- can vary
# from run to run; InferenceConfig(deterministic=True) or NXD_DECODE_ATTN_OPROJ=0 takes the
# two-launch path (bitwise-reproducible decode, ~5 % slower per token).
_ATTN_OPROJ = os.environ.get("NXD_DECODE_ATTN_OPROJ", "1") == "1"
# ... up to this many sequences per step: every (sequence, kv head) workgroup group of the fused
# launch streams its own copy of the o_proj block, so at batch B it reads Wo B times; above the cap
# the attention and the o_proj GEMV (one read of Wo for all rows) run as two launches.  Llama-3.2-1B
# ms per step fused / two launches: B=2 0.760 / 0.802, B=4 1.096 / 1.083, B=8 1.91 / 1.76
# (profiles/r5l_decode_dot2_batch_ab.jsonl)
_ATTN_OPROJ_MAXB = int(os.environ.get("NXD_DECODE_ATTN_OPROJ_MAXB", "2"))
# The token-embedding gather folded into the first layer's QKV launch (its RMSNorm prologue reads the
# embedding row of each token id and workgroup 0 writes it to the residual stream): one launch less
# per decode step.  NXD_DECODE_EMB_FUSED=0 keeps the separate embedding kernel (A/B).
_EMB_FUSED = os.environ.get("NXD_DECODE_EMB_FUSED", "1") == "1"


class DecoderInferenceMixin:
    """Inference forward of a decoder-only causal LM whose modules follow the framework's training
    layout (`model.embed_tokens / layers[i].{input_layernorm, self_attn.qkv_proj, self_attn.o_proj,
    post_attention_layernorm} / norm`, `lm_head`).  Subclasses provide the feed-forward block
    (`_ffn`) and may override the norm (`_norm`) and the QKV post-processing (`_qkv_hook`)."""

    def _init_inference(self, config) -> None:
        attn0 = self.model.layers[0].self_attn
        self.nq, self.nkv, self.head_dim = attn0.num_heads_local, attn0.num_kv_heads_local, attn0.head_dim
        self.tp = get_tensor_model_parallel_size()
        self.kv_cache: Optional[torch.Tensor] = None
        self.eps = float(config.rms_norm_eps)
        self.eval()
        for p in self.parameters():
            p.requires_grad_(False)

    # ------------------------------------------------------------------ KV cache
    def setup_kv_cache(self, max_batch: int, max_len: int, device=None) -> torch.Tensor:
        emb = self.model.embed_tokens.weight   # activation dtype (lm_head may be int8-quantized)
        device = device or emb.device
        L = len(self.model.layers)
        shape = (L, 2, max_batch, self.nkv, max_len, self.head_dim)
        if self.kv_cache is None or tuple(self.kv_cache.shape) != shape or self.kv_cache.device != torch.device(device):
            self.kv_cache = torch.zeros(shape, dtype=emb.dtype, device=device)
        return self.kv_cache

    def reset_kv_cache(self) -> None:
        if self.kv_cache is not None:
            self.kv_cache.zero_()

    # ------------------------------------------------------------------ collectives
    def _all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.tp > 1:
            dist.all_reduce(x, group=ps.get_tensor_model_parallel_group())
        return x

    def _gather_vocab(self, logits: torch.Tensor) -> torch.Tensor:
        if self.tp == 1:
            return logits
        from ..parallel import comm

        out = torch.empty((self.tp,) + tuple(logits.shape), dtype=logits.dtype, device=logits.device)
        comm.all_gather_into_tensor(out, logits.contiguous(), group=ps.get_tensor_model_parallel_group())
        return torch.movedim(out, 0, -2).reshape(logits.shape[:-1] + (self.tp * logits.shape[-1],))

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward_tokens(self, input_ids: torch.Tensor, positions: torch.Tensor, seq_ids: Optional[torch.Tensor] = None,
                       cache_len: Optional[torch.Tensor] = None, last_index: Optional[torch.Tensor] = None,
                       prefill: bool = False, return_hidden: bool = False):
        """input_ids [B, T]; positions [B, T] (int64) absolute positions of the new tokens;
        seq_ids [B] cache rows; cache_len [B] int32 valid cache length AFTER this step (decode);
        last_index [B] -> logits [B, V] of that token per sequence, else logits [B, T, V].
        prefill=True: the new tokens start at position 0 (causal flash attention over them)."""
        assert self.kv_cache is not None, "call setup_kv_cache() first"
        B, T = input_ids.shape
        if not prefill and self._decode_fusable(input_ids):
            return self._forward_decode_fused(input_ids, positions, seq_ids, cache_len, last_index, return_hidden)
        nq, nkv, D = self.nq, self.nkv, self.head_dim
        W = (nq + 2 * nkv) * D
        cos_t, sin_t = self.model.rope_cache.tables(input_ids.device)
        pos_flat = positions.reshape(-1)
        pos0 = positions[:, 0].to(torch.int32)
        sid32 = seq_ids.to(torch.int32) if seq_ids is not None else None   # once per step, not per layer
        emb = self.model.embed_tokens
        x = ops.vocab_parallel_embedding(input_ids, emb.weight, emb.start_index)
        x = self._all_reduce(x)
        residual = None
        for i, layer in enumerate(self.model.layers):
            attn = layer.self_attn
            h, residual = self._norm(x, layer.input_layernorm.weight, residual)
            qkv = self._qkv_hook(self._proj(attn.qkv_proj, h))  # [B, T, W]
            ops.rope_inplace_(qkv.view(B * T, W), 0, nq + nkv, D, cos_t, sin_t, pos_flat)
            q = qkv.view(B, T, nq + 2 * nkv, D)[:, :, :nq]
            k = qkv.view(B, T, nq + 2 * nkv, D)[:, :, nq:nq + nkv]
            v = qkv.view(B, T, nq + 2 * nkv, D)[:, :, nq + nkv:]
            kc, vc = self.kv_cache[i, 0], self.kv_cache[i, 1]
            ops.kv_cache_write(k, v, kc, vc, pos0, sid32)
            if prefill:
                o, _ = ops.flash_attn_fwd_lse(q, k, v, causal=True)
            else:
                o = ops.decode_attention(q, kc, vc, cache_len, sid32)
            x = self._row(attn.o_proj, o.reshape(B, T, nq * D))
            h, residual = self._norm(x, layer.post_attention_layernorm.weight, residual)
            x = self._ffn(layer, h)
        if last_index is not None:
            rows = torch.arange(B, device=x.device)
            x = x[rows, last_index]
            residual = residual[rows, last_index]
        h, _ = self._norm(x, self.model.norm.weight, residual)
        logits = self._gather_vocab(self._proj(self.lm_head, h))
        return (logits, h) if return_hidden else logits

    # ------------------------------------------------------------------ fused decode path
    def _fused_ffn_weights(self, layer):
        """(post-attention norm weight, fused gate/up [2I, H], down [H, I]) when the feed-forward
        block is a dense bias-free SwiGLU MLP the fused decode kernels can run, else None."""
        return None

    def _decode_fusable(self, input_ids: torch.Tensor) -> bool:
        ok = getattr(self, "_decode_fused_ok", None)
        if ok is None:
            ok = self._check_decode_fusable()
            self._decode_fused_ok = ok
        M = input_ids.numel()
        return ok and input_ids.is_cuda and M <= 8 and M * self.config.hidden_size <= 32768

    def _check_decode_fusable(self) -> bool:
        if os.environ.get("NXD_DECODE_FUSED", "1") == "0":
            return False
        if self.tp > 1 and os.environ.get("NXD_DECODE_FUSED_TP", "1") == "0":
            return False
        if type(self)._qkv_hook is not DecoderInferenceMixin._qkv_hook or type(self)._norm is not DecoderInferenceMixin._norm:
            return False
        if self.head_dim % 2 or self.head_dim > 256:
            return False
        for layer in self.model.layers:
            attn = layer.self_attn
            w, b = attn.qkv_proj._fused_weight_bias() if hasattr(attn.qkv_proj, "_fused_weight_bias") \
                else (attn.qkv_proj.weight, getattr(attn.qkv_proj, "bias", None))
            if b is not None or w.dtype != torch.bfloat16 or getattr(attn.o_proj, "bias", None) is not None:
                return False
            if attn.o_proj.weight.dtype != torch.bfloat16 or self._fused_ffn_weights(layer) is None:
                return False
        lm = self.lm_head.weight
        return lm.dtype == torch.bfloat16 and getattr(self.lm_head, "bias", None) is None

    def _decode_oacc(self, M: int, res: torch.Tensor) -> torch.Tensor:
        """fp32 [8, H] o_proj accumulator of the fused attention + o_proj decode launch: zero between
        uses (the down projection's epilogue re-zeroes the rows it consumed)."""
        buf = getattr(self, "_oacc_buf", None)
        if buf is None or buf.device != res.device or buf.shape[1] != res.shape[1]:
            buf = self._oacc_buf = torch.zeros((8, res.shape[1]), dtype=torch.float32, device=res.device)
        return buf

    def _forward_decode_fused(self, input_ids, positions, seq_ids, cache_len, last_index, return_hidden):
        if self.tp > 1:
            return self._forward_decode_fused_tp(input_ids, positions, seq_ids, cache_len, last_index, return_hidden)
        C = ops.ext()
        B, T = input_ids.shape
        M = B * T
        nq, nkv, D = self.nq, self.nkv, self.head_dim
        W = (nq + 2 * nkv) * D
        cos_t, sin_t = self.model.rope_cache.tables(input_ids.device)
        pos = positions.reshape(-1).to(torch.int64).contiguous()
        sid32 = seq_ids.to(torch.int32).contiguous() if seq_ids is not None else None
        emb = self.model.embed_tokens
        ew = emb.weight
        emb_fused = (_EMB_FUSED and emb.start_index == 0 and ew.dtype == torch.bfloat16 and ew.is_contiguous()
                     and input_ids.dtype == torch.int64)
        if emb_fused:
            ids = input_ids.reshape(-1).contiguous()
            res = torch.empty((M, ew.shape[1]), dtype=ew.dtype, device=ew.device)   # written by layer 0's QKV
        else:
            res = ops.vocab_parallel_embedding(input_ids, ew, emb.start_index).reshape(M, -1).contiguous()
        qkv = torch.empty((M, W), dtype=res.dtype, device=res.device)
        for i, layer in enumerate(self.model.layers):
            attn = layer.self_attn
            w_qkv = attn.qkv_proj._fused_weight_bias()[0] if hasattr(attn.qkv_proj, "_fused_weight_bias") \
                else attn.qkv_proj.weight
            kc, vc = self.kv_cache[i, 0], self.kv_cache[i, 1]
            # RMSNorm -> QKV -> RoPE -> k/v into the cache, one launch (layer 0: + the embedding gather)
            if i == 0 and emb_fused:
                C.dgemv(3, ew, layer.input_layernorm.weight, self.eps, w_qkv, qkv, nq, nkv, D, cos_t, sin_t, pos, T,
                        kc, vc, sid32, xidx=ids, xcopy=res)
            else:
                C.dgemv(3, res, layer.input_layernorm.weight, self.eps, w_qkv, qkv, nq, nkv, D, cos_t, sin_t, pos, T,
                        kc, vc, sid32)
            q = qkv.view(B, T, nq + 2 * nkv, D)[:, :, :nq]
            ln2, w_gu, w_d = self._fused_ffn_weights(layer)
            if _PREFETCH_MB > 0:
                # spare workgroups of the attention launch pull o_proj and the head of gate_up into
                # the Infinity Cache while the (latency-bound) attention leaves HBM idle
                C.decode_attn_prefetch(attn.o_proj.weight, -1, w_gu, int(_PREFETCH_MB * 2**20), _PREFETCH_WGS)
            fuse_o = (_ATTN_OPROJ and _PREFETCH_MB <= 0 and B <= _ATTN_OPROJ_MAXB
                      and not getattr(self, "_decode_deterministic", False))
            oacc = self._decode_oacc(M, res) if fuse_o else None
            if oacc is not None and C.decode_attn_oproj(q, kc, vc, sid32, cache_len.to(torch.int32), attn.o_proj.weight,
                                                        oacc, 1.0 / math.sqrt(D)):
                # oacc += o_proj(attention) (one launch); the GLU prologue sees res + oacc, the down
                # epilogue folds it into res with the unfused rounding and zeroes it
                a = torch.empty((M, w_d.shape[1]), dtype=res.dtype, device=res.device)
                C.dgemv(2, res, ln2, self.eps, w_gu, a, 0, 0, 0, None, None, None, 1, None, None, None, oacc, None)
                C.dgemv(1, a, None, 0.0, w_d, res, 0, 0, 0, None, None, None, 1, None, None, None, None, oacc)
                continue
            o = ops.decode_attention(q, kc, vc, cache_len, sid32)
            C.dgemv(1, o.reshape(M, nq * D), None, 0.0, attn.o_proj.weight, res, 0, 0, 0, None, None, None, 1,
                    None, None, None)                                   # res += o_proj(o)
            a = torch.empty((M, w_d.shape[1]), dtype=res.dtype, device=res.device)
            C.dgemv(2, res, ln2, self.eps, w_gu, a, 0, 0, 0, None, None, None, 1, None, None, None)  # norm+SwiGLU
            C.dgemv(1, a, None, 0.0, w_d, res, 0, 0, 0, None, None, None, 1, None, None, None)   # res += down(a)
        h = res.view(B, T, -1)
        if last_index is not None:
            h = h[torch.arange(B, device=h.device), last_index]
        h2 = h.reshape(-1, h.shape[-1]).contiguous()
        logits = torch.empty((h2.shape[0], self.lm_head.weight.shape[0]), dtype=res.dtype, device=res.device)
        C.dgemv(0, h2, self.model.norm.weight, self.eps, self.lm_head.weight, logits, 0, 0, 0, None, None, None, 1,
                None, None, None)                                       # final norm + lm_head
        logits = logits.view(h.shape[:-1] + (logits.shape[-1],))
        if return_hidden:
            return logits, ops.rms_norm(h, self.model.norm.weight, self.eps)[0]
        return logits

    def peer_decode_ready(self) -> bool:
        """True when decode at TP > 1 runs entirely on the one-shot peer kernels (fused path, every
        all-reduce and the vocabulary gather over IPC): no process-group collective is left in a decode
        step, so it can be captured in a hipGraph even when the TP group itself is gloo (ranks sharing
        one GPU).  Collective on first use (every rank calls it at the same point)."""
        from ..parallel.peer_allreduce import PeerAllReduce

        if self.tp == 1 or not self._check_decode_fusable():
            return False
        ew = self.model.embed_tokens.weight
        if ew.device.type != "cuda":
            return False
        return isinstance(self._decode_tp_state(ew.shape[1], ew.device)["ar"], PeerAllReduce)

    def check_decode_kernels(self) -> None:
        """Raise if a single-launch long-context attention + o_proj (csrc/decode_attn.hip SYNC) timed out
        waiting for a key split's partial (that launch wrote NaN): read once per generate()."""
        if not torch.cuda.is_available() or not ops.ext_available():
            return
        if ops.ext().decode_attn_sync_error(True):
            raise RuntimeError("decode attention: a key-split partial never arrived (bounded spin timed out); "
                               "the step's outputs are NaN")

    def check_collectives(self) -> None:
        """Raise if the TP decode all-reduce lost a peer since it was built (a pinned host word: the
        caller synchronises first so its own step is covered)."""
        st = getattr(self, "_tp_dec", None)
        if st is not None:
            st["ar"].check()

    def _decode_tp_state(self, H: int, device):
        """TP > 1 fused decode: fp32 [8, H] partial / sum buffers and the decode all-reduce (one-shot
        peer all-reduce over IPC when available -- parallel/peer_allreduce.py -- else the process
        group).  Built once; its collective set-up runs on every rank at the same decode step."""
        st = getattr(self, "_tp_dec", None)
        if st is None or st["H"] != H or st["device"] != device:
            from ..parallel.peer_allreduce import make_decode_all_reduce

            vl = self.lm_head.weight.shape[0]   # this rank's vocabulary rows (bf16 logits gathered as bytes)
            ar = make_decode_all_reduce(ps.get_tensor_model_parallel_group(), max(8 * H, 4 * vl), device,
                                        prefer_peer=os.environ.get("NXD_DECODE_PEER_AR", "1") == "1")
            z = lambda: torch.zeros((8, H), dtype=torch.float32, device=device)  # noqa: E731
            st = self._tp_dec = {"H": H, "device": device, "ar": ar, "oacc": z(), "osum": z(), "dacc": z(), "emb": z()}
        return st

    def _forward_decode_fused_tp(self, input_ids, positions, seq_ids, cache_len, last_index, return_hidden):
        """Decode at TP > 1 on the fused GEMV kernels.  Per layer (6 launches):
          RMSNorm+QKV+RoPE+KV-write on this rank's heads; attention + o_proj partial (fp32 atomics
          into oacc); all-reduce oacc -> osum; RMSNorm(res + osum)+gate_up+SwiGLU on this rank's
          intermediate slice; down partial (fp32); all-reduce it and fold res = bf16(bf16(res +
          bf16(osum)) + bf16(down)) -- the TP = 1 kernels' rounding, with the partials summed in fp32
          in rank order (identical bits on every rank).  The embedding is the vocab-parallel gather
          summed the same way; lm_head runs on this rank's vocabulary slice, gathered at the end.
        Reference: examples/inference/modules/gqa.py:641-647 (the TP all-reduces of the fork's
        notebook config, tp_degree = 2), src/neuronx_distributed/trace/spmd.py:82-187."""
        C = ops.ext()
        B, T = input_ids.shape
        M = B * T
        nq, nkv, D = self.nq, self.nkv, self.head_dim
        W = (nq + 2 * nkv) * D
        cos_t, sin_t = self.model.rope_cache.tables(input_ids.device)
        pos = positions.reshape(-1).to(torch.int64).contiguous()
        sid32 = seq_ids.to(torch.int32).contiguous() if seq_ids is not None else None
        emb = self.model.embed_tokens
        ew = emb.weight
        H = ew.shape[1]
        st = self._decode_tp_state(H, ew.device)
        ar, oacc, osum, dacc = st["ar"], st["oacc"], st["osum"], st["dacc"]
        res = torch.empty((M, H), dtype=ew.dtype, device=ew.device)
        ebuf = st["emb"][:M]
        ebuf.copy_(ops.vocab_parallel_embedding(input_ids, ew, emb.start_index).reshape(M, H))
        ar.set_residual_(ebuf, res)                                   # res = the embedding rows
        qkv = torch.empty((M, W), dtype=res.dtype, device=res.device)
        clen32 = cache_len.to(torch.int32)
        fuse_o = _ATTN_OPROJ and B <= _ATTN_OPROJ_MAXB and not getattr(self, "_decode_deterministic", False)
        for i, layer in enumerate(self.model.layers):
            attn = layer.self_attn
            w_qkv = attn.qkv_proj._fused_weight_bias()[0] if hasattr(attn.qkv_proj, "_fused_weight_bias") \
                else attn.qkv_proj.weight
            kc, vc = self.kv_cache[i, 0], self.kv_cache[i, 1]
            C.dgemv(3, res, layer.input_layernorm.weight, self.eps, w_qkv, qkv, nq, nkv, D, cos_t, sin_t, pos, T,
                    kc, vc, sid32)
            q = qkv.view(B, T, nq + 2 * nkv, D)[:, :, :nq]
            ln2, w_gu, w_d = self._fused_ffn_weights(layer)
            if not (fuse_o and C.decode_attn_oproj(q, kc, vc, sid32, clen32, attn.o_proj.weight, oacc, 1.0 / math.sqrt(D))):
                o = ops.decode_attention(q, kc, vc, cache_len, sid32)
                C.dgemv(0, o.reshape(M, nq * D), None, 0.0, attn.o_proj.weight, oacc[:M], 0, 0, 0, None, None, None, 1,
                        None, None, None)                             # fp32 partial (overwrites)
            ar.sum_(oacc[:M], osum[:M], zero_in=True)                 # osum = o_proj; oacc re-zeroed
            a = torch.empty((M, w_d.shape[1]), dtype=res.dtype, device=res.device)
            C.dgemv(2, res, ln2, self.eps, w_gu, a, 0, 0, 0, None, None, None, 1, None, None, None, osum, None)
            C.dgemv(0, a, None, 0.0, w_d, dacc[:M], 0, 0, 0, None, None, None, 1, None, None, None)  # fp32 partial
            ar.fold_residual_(dacc[:M], res, osum[:M])                # res += o_proj + down
        h = res.view(B, T, -1)
        if last_index is not None:
            h = h[torch.arange(B, device=h.device), last_index]
        h2 = h.reshape(-1, h.shape[-1]).contiguous()
        logits = torch.empty((h2.shape[0], self.lm_head.weight.shape[0]), dtype=res.dtype, device=res.device)
        C.dgemv(0, h2, self.model.norm.weight, self.eps, self.lm_head.weight, logits, 0, 0, 0, None, None, None, 1,
                None, None, None)                                       # final norm + this rank's vocab slice
        full = torch.empty((logits.shape[0], self.tp * logits.shape[1]), dtype=logits.dtype, device=logits.device)
        ar.gather_(logits, full)                                        # vocab-parallel slices side by side
        logits = full.view(h.shape[:-1] + (full.shape[-1],))
        if return_hidden:
            return logits, ops.rms_norm(h, self.model.norm.weight, self.eps)[0]
        return logits

    @torch.no_grad()
    def forward_tree(self, tokens: torch.Tensor, positions: torch.Tensor, tree_mask: torch.Tensor, prefix_len: int,
                     seq_id: int = 0):
        """Medusa tree verification for ONE sequence: tokens / positions [N] (tree nodes at
        prefix_len + depth), tree_mask [N, N] bool (node i sees node j iff j is i or an ancestor).
        Every node also sees the cached prefix [0, prefix_len).  Nothing is written to the KV cache;
        returns (logits [N, V], final hidden [N, H], per-layer (k, v) [N, Hkv, D] of the nodes) so
        the caller commits only the accepted path (commit_tree_kv)."""
        N = tokens.shape[0]
        nq, nkv, D = self.nq, self.nkv, self.head_dim
        g = nq // nkv
        W = (nq + 2 * nkv) * D
        cos_t, sin_t = self.model.rope_cache.tables(tokens.device)
        scale = 1.0 / math.sqrt(D)
        emb = self.model.embed_tokens
        x = self._all_reduce(ops.vocab_parallel_embedding(tokens.view(1, N), emb.weight, emb.start_index))
        residual = None
        kvs = []
        tree_bias = torch.zeros((N, N), dtype=torch.float32, device=tokens.device).masked_fill(~tree_mask, float("-inf"))
        for i, layer in enumerate(self.model.layers):
            attn = layer.self_attn
            h, residual = self._norm(x, layer.input_layernorm.weight, residual)
            qkv = self._qkv_hook(self._proj(attn.qkv_proj, h))
            ops.rope_inplace_(qkv.view(N, W), 0, nq + nkv, D, cos_t, sin_t, positions.reshape(-1))
            qkv4 = qkv.view(N, nq + 2 * nkv, D)
            q, k, v = qkv4[:, :nq], qkv4[:, nq:nq + nkv], qkv4[:, nq + nkv:]
            kvs.append((k.clone(), v.clone()))
            kc = self.kv_cache[i, 0, seq_id, :, :prefix_len].float()   # [Hkv, P, D]
            vc = self.kv_cache[i, 1, seq_id, :, :prefix_len].float()
            qf = q.float().permute(1, 0, 2).reshape(nkv, g * N, D)    # heads grouped by kv head
            s_c = torch.matmul(qf, kc.transpose(1, 2)) * scale         # [Hkv, g*N, P]
            s_t = torch.matmul(qf, k.float().permute(1, 2, 0)) * scale  # [Hkv, g*N, N]
            s_t = s_t.view(nkv, g, N, N) + tree_bias
            s = torch.cat([s_c.view(nkv, g, N, prefix_len), s_t], -1)
            p_ = torch.softmax(s, -1)
            o = torch.matmul(p_[..., :prefix_len].reshape(nkv, g * N, prefix_len), vc) + \
                torch.matmul(p_[..., prefix_len:].reshape(nkv, g * N, N), v.float().permute(1, 0, 2))
            o = o.view(nq, N, D).permute(1, 0, 2).reshape(1, N, nq * D).to(x.dtype)
            x = self._row(attn.o_proj, o)
            h, residual = self._norm(x, layer.post_attention_layernorm.weight, residual)
            x = self._ffn(layer, h)
        h, _ = self._norm(x, self.model.norm.weight, residual)
        logits = self._gather_vocab(self._proj(self.lm_head, h))
        return logits.view(N, -1), h.view(N, -1), kvs

    @torch.no_grad()
    def commit_tree_kv(self, kvs, nodes: torch.Tensor, start: int, seq_id: int = 0) -> None:
        """Write the K/V of the accepted tree nodes (in path order) at cache positions start..start+n."""
        sid = torch.tensor([seq_id], dtype=torch.int32, device=nodes.device)
        pos = torch.tensor([start], dtype=torch.int32, device=nodes.device)
        for i, (k, v) in enumerate(kvs):
            ops.kv_cache_write(k.index_select(0, nodes).unsqueeze(0), v.index_select(0, nodes).unsqueeze(0),
                               self.kv_cache[i, 0], self.kv_cache[i, 1], pos, sid)

    def _row(self, mod, x: torch.Tensor) -> torch.Tensor:
        """Row-parallel projection: partial GEMM, TP all-reduce, then the (replicated) bias."""
        y = self._all_reduce(self._proj(mod, x, use_bias=False))
        b = getattr(mod, "bias", None)
        return y + b if b is not None else y

    @staticmethod
    def _proj(mod, x: torch.Tensor, glu: bool = False, use_bias: bool = True) -> torch.Tensor:
        """Local (no-collective) projection of a TP linear: bf16 or int8-quantized weights; decode-sized
        inputs go through the skinny-GEMM kernel (int8 read directly, SwiGLU fused when glu=True)."""
        if hasattr(mod, "_fused_weight_bias"):
            w, b = mod._fused_weight_bias()
        else:
            w, b = mod.weight, getattr(mod, "bias", None)
        if not use_bias:
            b = None
        scale = mod._row_scale() if w.dtype == torch.int8 else None
        M = x.numel() // x.shape[-1]
        if w.dtype == torch.int8 or (M <= 8 and x.is_cuda):
            return skinny_linear(x, w, scale, b, glu=glu)
        from ..trace.weight_layout import packed_linear

        y = packed_linear(mod, x, w, b)   # pre-packed K-major copy when the layout pass chose it
        return ops.swiglu(y) if glu else y

    def _ffn(self, layer, h: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def _qkv_hook(self, qkv: torch.Tensor) -> torch.Tensor:
        return qkv

    def _norm(self, x, w, residual):
        if residual is None:
            y, _ = ops.rms_norm(x, w, self.eps)
            return y, x
        return ops.rms_norm(x, w, self.eps, residual)
