"""Causal-LM inference application: weights, context encoding, graph-captured token generation,
HF-style `generate` (reference: examples/inference/modules/model_base.py:520-1144
`NeuronBaseForCausalLM`, model_wrapper.py:60-368 `ModelWrapper`, llama3/neuron_modeling_llama.py
`NeuronLlamaForCausalLM`).

Lifecycle (same verbs as the reference):
    model = LlamaForCausalLMInference.from_pretrained(hf_dir | None, inference_config, model_config)
    model.compile(out_dir)      # per-rank sharded safetensors + configs (the reference's trace())
    model = LlamaForCausalLMInference.load(out_dir)   # shards -> GPU, KV cache, hipGraph capture
    ids = model.generate(input_ids, attention_mask, max_new_tokens=..., top_k=..., do_sample=...)

Run one process per GPU for TP > 1 (torchrun); every rank executes the same calls (SPMD).
"""

from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..parallel_layers import parallel_state as ps
from ..parallel_layers.sharding import shard_state_dict
from ..utils.logger import get_logger
from ..utils.sampling import Sampler
from .bucketing import pad_to_bucket
from .config import InferenceConfig
from .graphs import DecodeGraph, DecodeState, decode_step
from .modeling_llama import LlamaInferenceModel
from ..utils.graph_capture import graph_capture

logger = get_logger()

CONTEXT_ENCODING_MODEL = "context_encoding_model"
TOKEN_GENERATION_MODEL = "token_generation_model"
SPECULATION_MODEL = "speculation_model"
END_TO_END_MODEL = "e2e_model"


def _device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def load_hf_state_dict(model_dir: str) -> Dict[str, torch.Tensor]:
    """HF checkpoint directory -> state dict (safetensors single/sharded, else torch .bin with
    weights_only=True)."""
    from safetensors.torch import load_file

    idx = os.path.join(model_dir, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            files = sorted(set(json.load(f)["weight_map"].values()))
        sd = {}
        for fn in files:
            sd.update(load_file(os.path.join(model_dir, fn)))
        return sd
    single = os.path.join(model_dir, "model.safetensors")
    if os.path.exists(single):
        return load_file(single)
    binf = os.path.join(model_dir, "pytorch_model.bin")
    if os.path.exists(binf):
        return torch.load(binf, map_location="cpu", weights_only=True)
    raise FileNotFoundError(f"no HF weights found in {model_dir}")


class PrefillGraph:
    """Context encoding of a fixed (batch, bucket) shape captured in one hipGraph: static input
    buffers (token ids, cache rows, last-token index), positions 0..Tb-1 baked in, KV-cache writes
    and all collectives inside the graph.  Graphs of different buckets share one memory pool (they
    replay one at a time)."""

    def __init__(self, model, B: int, Tb: int, device, pool=None):
        self.model = model
        self.ids = torch.zeros((B, Tb), dtype=torch.long, device=device)
        self.seq_ids = torch.arange(B, dtype=torch.int32, device=device)
        self.last = torch.full((B,), Tb - 1, dtype=torch.long, device=device)
        self.positions = torch.arange(Tb, device=device).unsqueeze(0).expand(B, Tb).contiguous()
        # warm-up on a side stream (GEMM autotuning, workspace allocation) before capture; it
        # writes KV-cache rows that the real prefill overwrites
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            self._fwd()
        torch.cuda.current_stream(device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        self.pool = pool if pool is not None else torch.cuda.graph_pool_handle()
        with graph_capture(self.graph, pool=self.pool):
            self.out = self._fwd()

    def _fwd(self):
        return self.model.forward_tokens(self.ids, self.positions, self.seq_ids, last_index=self.last, prefill=True)

    def run(self, ids: torch.Tensor, seq_ids: torch.Tensor, last_index: torch.Tensor) -> torch.Tensor:
        self.ids.copy_(ids)
        self.seq_ids.copy_(seq_ids)
        self.last.copy_(last_index)
        self.graph.replay()
        return self.out


class _SubModel:
    """Callable view used by benchmarks / latency collectors (reference ModelWrapper tags)."""

    def __init__(self, owner: "LlamaForCausalLMInference", tag: str):
        self.owner, self.tag = owner, tag
        self._pre_hooks, self._hooks = [], []

    def register_forward_pre_hook(self, fn):
        self._pre_hooks.append(fn)

    def register_forward_hook(self, fn):
        self._hooks.append(fn)

    def __call__(self, *args, **kwargs):
        for h in self._pre_hooks:
            h(self)
        out = (self.owner._context_encode if self.tag == CONTEXT_ENCODING_MODEL else self.owner._token_generate)(
            *args, **kwargs)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        for h in self._hooks:
            h(self)
        return out


class LlamaForCausalLMInference:
    """Model family hooks (overridden by the MoE applications in inference/moe.py):
    `_model_cls` the device module, `_hf_to_nxd` HF full state dict -> framework names,
    `_config_from_dir` HF config.json -> model config."""

    _model_cls = LlamaInferenceModel

    @staticmethod
    def _hf_to_nxd(hf_sd, model_config):
        from ..models.llama.convert import hf_to_nxd

        return hf_to_nxd(hf_sd, model_config)

    @staticmethod
    def _config_from_dir(path: str):
        from .config import model_config_from_dir

        return model_config_from_dir(path)

    def __init__(self, model_config, config: InferenceConfig, dtype: torch.dtype = torch.bfloat16,
                 device: Optional[torch.device] = None, init_weights: bool = True):
        self.model_config = model_config
        self.config = config
        self.dtype = dtype
        self.device = device or _device()
        if dist.is_initialized() and not ps.model_parallel_is_initialized():
            ps.initialize_model_parallel(tensor_model_parallel_size=config.tp_degree)
        elif not dist.is_initialized():
            assert config.tp_degree == 1, "tp_degree > 1 needs torch.distributed (one process per GPU)"
            if not ps.model_parallel_is_initialized():
                _init_single_process()
                ps.initialize_model_parallel(tensor_model_parallel_size=1)
        self._mha_from = None
        strategy = getattr(config, "gqa_sharding_strategy", None)
        nq = model_config.num_attention_heads
        nkv = getattr(model_config, "num_key_value_heads", None) or nq
        if strategy is not None and nkv < nq:
            from ..modules.gqa import GQA, determine_sharding_strategy

            if determine_sharding_strategy(config.tp_degree, nkv, strategy) == GQA.CONVERT_TO_MHA:
                # reference examples/inference/modules/gqa.py: K/V heads replicated to one per Q head
                import copy as _copy

                self._mha_from = (nq, nkv, getattr(model_config, "head_dim", None) or model_config.hidden_size // nq)
                model_config = _copy.copy(model_config)
                model_config.num_key_value_heads = nq
                self.model_config = model_config
        self.model = self._model_cls(model_config, dtype=dtype,
                                     device=torch.device("meta") if not init_weights else self.device)
        # InferenceConfig(deterministic=True): no fp32-atomic fused decode launches (model_base.py)
        self.model._decode_deterministic = bool(getattr(config, "deterministic", False))
        if config.quantized:
            self._quantize()
        self.max_batch = config.max_batch_size
        self.graph_steps = max(1, int(config.decode_graph_steps))
        # KV-cache slack so a final multi-step replay (decode graph, or speculation rounds of K+1
        # positions each) may overshoot max_length without faulting
        K = int(getattr(config, "speculation_length", 0) or 0)
        spec_slack = (K + 1) * int(getattr(config, "spec_rounds_per_graph", 4)) + 2 if K else 0
        self.cache_len = config.max_length + max(self.graph_steps, spec_slack)
        self._graphs: Dict[tuple, DecodeGraph] = {}
        self._prefill_cache: Dict[tuple, "PrefillGraph"] = {}
        self._prefill_pool = None
        self._states: Dict[int, DecodeState] = {}
        self.kv_cache_populated = False
        self.context_encoding_model = _SubModel(self, CONTEXT_ENCODING_MODEL)
        self.token_generation_model = _SubModel(self, TOKEN_GENERATION_MODEL)
        if init_weights:
            self.model.setup_kv_cache(self.max_batch, self.cache_len, self.device)

    def _quantize(self) -> None:
        """Swap the decoder / lm_head linears for int8 weight-only layers (reference flow:
        run_llama_quantized.py -> quantize_pytorch_model_per_*_symmetric + convert)."""
        from ..quantization import convert, get_default_custom_qconfig_dict, get_default_per_channel_custom_qconfig_dict

        qt = str(self.config.quantization_type)
        q = get_default_per_channel_custom_qconfig_dict() if "channel" in qt else get_default_custom_qconfig_dict()
        convert(self.model, q, inplace=True)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_pretrained(cls, model_path: Optional[str], config: InferenceConfig, model_config=None,
                        dtype: torch.dtype = torch.bfloat16):
        """HF directory -> model on this rank's GPU (random init when model_path is None)."""
        if model_config is None:
            model_config = cls._config_from_dir(model_path)
        if model_path is None:
            return cls(model_config, config, dtype)
        self = cls(model_config, config, dtype, init_weights=False)
        full = cls._hf_to_nxd(load_hf_state_dict(model_path), model_config)
        self._load_full(full)
        return self

    def _load_full(self, full_sd: Dict[str, torch.Tensor]) -> None:
        if self._mha_from is not None:
            from ..modules.gqa import convert_state_dict_to_mha

            full_sd = convert_state_dict_to_mha(full_sd, *self._mha_from)
        tp, rank = ps.get_tensor_model_parallel_size(), ps.get_tensor_model_parallel_rank()
        local = shard_state_dict(self.model, full_sd, tp, rank, strict=False)
        self._load_local(local)

    def _load_local(self, local: Dict[str, torch.Tensor]) -> None:
        if any(p.device.type == "meta" for p in self.model.parameters()):
            self.model.to_empty(device=self.device)
            if getattr(self.model_config, "tie_word_embeddings", False) and self.model.lm_head.weight.is_floating_point():
                self.model.lm_head.weight = self.model.model.embed_tokens.weight
        tied_q = getattr(self.model_config, "tie_word_embeddings", False) and \
            not self.model.lm_head.weight.is_floating_point()
        if tied_q and "lm_head.weight" not in local and "model.embed_tokens.weight" in local:
            local["lm_head.weight"] = local["model.embed_tokens.weight"]   # quantized copy of the tied table
        local = {k: (v.to(self.dtype) if v.is_floating_point() and k.split(".")[-1] != "scale" else v)
                 for k, v in local.items()}
        missing, unexpected = self.model.load_state_dict(local, strict=False)
        missing = [m for m in missing if not (getattr(self.model_config, "tie_word_embeddings", False)
                                              and m == "lm_head.weight" and not tied_q)]
        if missing:
            raise RuntimeError(f"missing weights: {missing[:8]}")
        for p in self.model.parameters():
            p.requires_grad_(False)
        if hasattr(self.model, "post_load"):
            self.model.post_load()
        if getattr(self.config, "weight_layout_optimization", False):
            from ..trace.weight_layout import optimize_weight_layout

            self.weight_layouts = optimize_weight_layout(self.model, int(self.config.max_context_length) * self.max_batch,
                                                         path=getattr(self, "_layout_dir", None))
        self.model.setup_kv_cache(self.max_batch, self.cache_len, self.device)
        # captured graphs hold the previous weight / cache tensors
        self._graphs.clear()
        self._prefill_cache.clear()

    def compile(self, serialize_base_path: str) -> None:
        """Write this rank's weight shard + configs (the reference's trace/compile step; there is
        nothing to compile ahead of time — kernels are prebuilt, graphs are captured on load)."""
        from safetensors.torch import save_file

        os.makedirs(serialize_base_path, exist_ok=True)
        rank = ps.get_tensor_model_parallel_rank()
        sd = {k: v.detach().contiguous().cpu() for k, v in self.model.state_dict().items()}
        if getattr(self.model_config, "tie_word_embeddings", False):
            sd.pop("lm_head.weight", None)
        save_file(sd, os.path.join(serialize_base_path, f"tp{rank}_sharded_checkpoint.safetensors"))
        if rank == 0 and (not dist.is_initialized() or ps.get_data_parallel_rank() == 0):
            self.config.save_pretrained(serialize_base_path)
            self.model_config.save_pretrained(serialize_base_path)
            if getattr(self, "weight_layouts", None) is not None:
                from ..trace.weight_layout import save_layouts

                save_layouts(serialize_base_path, self.weight_layouts)
        if dist.is_initialized():
            dist.barrier()

    @classmethod
    def load(cls, serialize_base_path: str, dtype: torch.dtype = torch.bfloat16):
        from safetensors.torch import load_file

        config = InferenceConfig.from_pretrained(serialize_base_path)
        model_config = cls._config_from_dir(serialize_base_path)
        self = cls(model_config, config, dtype, init_weights=False)
        self._layout_dir = serialize_base_path      # reuse the compiled weight-layout map, if any
        rank = ps.get_tensor_model_parallel_rank()
        local = load_file(os.path.join(serialize_base_path, f"tp{rank}_sharded_checkpoint.safetensors"))
        self._load_local(local)
        return self

    # ------------------------------------------------------------------ model calls
    def reset(self) -> None:
        self.kv_cache_populated = False

    def set_fused_decode(self, enabled: bool) -> None:
        """A/B switch of the fused decode kernels (csrc/decode_fused.hip, decode_attn.hip; at TP > 1 with
        the one-shot peer all-reduce) against the unfused per-op decode; the next decode step re-checks
        whether the model can take the fused path."""
        self.model._decode_fused_ok = None if enabled else False

    def _context_encode(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                        position_ids: Optional[torch.Tensor] = None, seq_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Prefill; returns logits [B, V] of each sequence's last valid token (fp32)."""
        dev = self.device
        input_ids = input_ids.to(dev)
        B, T = input_ids.shape
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        attention_mask = attention_mask.to(dev)
        lengths = attention_mask.sum(1)
        pad = self.model_config.pad_token_id if getattr(self.model_config, "pad_token_id", None) is not None else 0
        ids, mask = pad_to_bucket(input_ids, attention_mask, self.config.buckets + [self.config.max_length], pad)
        Tb = ids.shape[1]
        seq_ids = torch.arange(B, device=dev) if seq_ids is None else seq_ids.to(dev)
        if self._prefill_graphs_on():
            logits = self._prefill_graph(B, Tb).run(ids, seq_ids, lengths - 1)
        else:
            positions = torch.arange(Tb, device=dev).unsqueeze(0).expand(B, Tb)
            logits = self.model.forward_tokens(ids, positions, seq_ids, last_index=lengths - 1, prefill=True)
        self.kv_cache_populated = True
        return logits.float()

    def _graphs_allowed(self) -> bool:
        """hipGraphs capture RCCL kernels, not host-staged gloo collectives: a TP group on gloo
        (several ranks sharing one GPU, the single-GPU rehearsal of a TP server) runs eagerly."""
        if not getattr(self.config, "use_hip_graphs", True) or self.device.type != "cuda":
            return False
        if getattr(self.config, "tp_degree", 1) > 1:
            import torch.distributed as dist

            from ..parallel_layers import parallel_state as ps

            if dist.is_initialized() and ps.model_parallel_is_initialized() and \
                    dist.get_backend(ps.get_tensor_model_parallel_group()) == "gloo":
                return False
        return True

    def _decode_graphs_allowed(self) -> bool:
        """Decode graphs: as `_graphs_allowed`, and also on a gloo TP group when every collective of
        the decode step runs on the one-shot peer kernels (model_base.peer_decode_ready)."""
        if self._graphs_allowed():
            return True
        if not getattr(self.config, "use_hip_graphs", True) or self.device.type != "cuda":
            return False
        return getattr(self.config, "tp_degree", 1) > 1 and self.model.peer_decode_ready()

    def _prefill_graphs_on(self) -> bool:
        return getattr(self.config, "prefill_graphs", True) and self._graphs_allowed()

    def _prefill_graph(self, B: int, Tb: int) -> "PrefillGraph":
        """One captured context-encoding forward per (batch, bucket) -- the reference compiles one
        NEFF per bucket (trace/model_builder.py:380-451, SPMDBucketModel trace/spmd.py:32-61); here a
        hipGraph per bucket removes the per-kernel launch cost of prefill."""
        key = (B, Tb)
        g = self._prefill_cache.get(key)
        if g is None:
            g = self._prefill_cache[key] = PrefillGraph(self.model, B, Tb, self.device, self._prefill_pool)
            self._prefill_pool = g.pool
        return g

    def _token_generate(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                        position_ids: Optional[torch.Tensor] = None, seq_ids: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One eager decode call for T new tokens per sequence at `position_ids[:, 0]`; returns
        logits [B, T, V] (fp32)."""
        dev = self.device
        input_ids = input_ids.to(dev)
        B, T = input_ids.shape
        positions = position_ids.to(dev)
        if positions.shape[1] != T:
            positions = positions[:, :1] + torch.arange(T, device=dev)
        seq_ids = torch.arange(B, device=dev) if seq_ids is None else seq_ids.to(dev)
        cache_len = (positions[:, -1] + 1).to(torch.int32)
        return self.model.forward_tokens(input_ids, positions, seq_ids, cache_len).float()

    def forward(self, input_ids, attention_mask=None, position_ids=None, seq_ids=None):
        if input_ids.shape[-1] > 1 and input_ids.shape[-1] != self.config.speculation_length:
            return self._context_encode(input_ids, attention_mask, position_ids, seq_ids)
        return self._token_generate(input_ids, attention_mask, position_ids, seq_ids)

    __call__ = forward

    # ------------------------------------------------------------------ generation
    def _decode_state(self, batch: int) -> DecodeState:
        st = self._states.get(batch)
        if st is None:
            steps_cap = (math.ceil(self.config.max_length / self.graph_steps) + 1) * self.graph_steps
            st = self._states[batch] = DecodeState(batch, steps_cap, self.device)
        return st

    def _graph(self, batch: int, sampler: Sampler) -> DecodeGraph:
        """Decode graph of (batch, sampler).  Call with the state already loaded: the capture's
        eager warm-up then writes the KV cache only at positions the replay overwrites before it
        reads them (a stale state would overwrite the freshly prefilled prompt positions)."""
        key = (batch, sampler.top_k, sampler.temperature)
        g = self._graphs.get(key)
        if g is None:
            g = self._graphs[key] = DecodeGraph(self.model, sampler, self._decode_state(batch), self.graph_steps,
                                                use_graph=self._decode_graphs_allowed())
        return g

    def _peer_decode(self) -> bool:
        """True once this model's TP decode all-reduces run on the one-shot peer kernels (built at the
        first decode step)."""
        st = getattr(self.model, "_tp_dec", None)
        return st is not None and type(st["ar"]).__name__ == "PeerAllReduce"

    @torch.no_grad()
    def generate(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                 max_new_tokens: Optional[int] = None, do_sample: bool = False, top_k: int = 1,
                 temperature: float = 1.0, eos_token_id=None, pad_token_id: Optional[int] = None,
                 max_length: Optional[int] = None, seed: Optional[int] = None, assistant_model=None,
                 **unused) -> torch.Tensor:
        """HF-style generate: returns [B, T + new] token ids (right-padded prompts keep their pads,
        tokens after EOS are `pad_token_id`).  `assistant_model` (another LlamaForCausalLMInference
        with the same vocabulary) switches to greedy speculative decoding (inference/speculation.py)."""
        if assistant_model is not None:
            if do_sample:
                raise ValueError("Sampling is unsupported as part of speculation. Only greedy speculation is supported.")
            from .speculation import SpeculativeDecoder

            K = int(self.config.speculation_length or 4)
            dec = self._spec.get(id(assistant_model)) if hasattr(self, "_spec") else None
            if dec is None:
                dec = SpeculativeDecoder(self, assistant_model, K, int(getattr(self.config, "spec_rounds_per_graph", 4)))
                if not hasattr(self, "_spec"):
                    self._spec = {}
                self._spec[id(assistant_model)] = dec
            if max_new_tokens is None and max_length is not None:
                max_new_tokens = max_length - input_ids.shape[1]
            return dec.generate(input_ids, attention_mask, max_new_tokens=max_new_tokens, eos_token_id=eos_token_id,
                                pad_token_id=pad_token_id)
        dev = self.device
        B, T = input_ids.shape
        assert B <= self.max_batch, f"batch {B} > max_batch_size {self.max_batch}"
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        if max_new_tokens is None:
            max_new_tokens = (max_length or self.config.max_length) - T
        lengths = attention_mask.to(dev).sum(1)
        max_new_tokens = int(min(max_new_tokens, self.config.max_length - int(lengths.max())))
        if eos_token_id is None:
            eos_token_id = getattr(self.model_config, "eos_token_id", None)
        eos = torch.tensor(eos_token_id if isinstance(eos_token_id, (list, tuple)) else
                           ([eos_token_id] if eos_token_id is not None else []), device=dev, dtype=torch.int64)
        pad_id = pad_token_id if pad_token_id is not None else (int(eos[0]) if eos.numel() else 0)
        sampler = Sampler(None, top_k=top_k if do_sample else 1, temperature=temperature, do_sample=do_sample)
        gen = torch.Generator(device=dev)
        if seed is not None:
            gen.manual_seed(seed)
        elif dist.is_initialized():
            gen.manual_seed(1234)  # identical draws on every TP rank
        else:
            gen.seed()
        logits = self._context_encode(input_ids, attention_mask)
        if hasattr(self.model, "check_collectives"):
            self.model.check_collectives()
        u0 = torch.rand(B, device=dev, generator=gen)
        first = sampler.sample(logits, u0)
        new = [first.view(B, 1)]
        if max_new_tokens > 1:
            Bp = B
            st = self._decode_state(Bp)
            uni = torch.rand((st.max_steps, Bp), device=dev, generator=gen)
            st.load(first, lengths, torch.arange(Bp, device=dev), uni)
            g = self._graph(Bp, sampler)
            todo = max_new_tokens - 1
            done_steps = 0
            while done_steps < todo:
                g.replay()
                done_steps += g.steps
                if self._peer_decode():
                    # a lost TP peer wrote NaN logits / residuals: fail this generate(), never emit them
                    torch.cuda.current_stream().synchronize()
                    self.model.check_collectives()
                if eos.numel():
                    seen = torch.isin(torch.cat([first.view(B, 1), st.out[:, :min(done_steps, todo)]], 1), eos)
                    if bool(seen.any(1).all()):
                        break
            new.append(st.out[:, :min(done_steps, todo)].clone())
            if hasattr(self.model, "check_decode_kernels"):
                self.model.check_decode_kernels()
        out = torch.cat(new, 1)[:, :max_new_tokens]
        if eos.numel():
            hit = torch.isin(out, eos).int()
            after = (hit.cumsum(1) - hit) > 0   # strictly after the first EOS
            out = out.masked_fill(after, pad_id)
        self.kv_cache_populated = False
        return torch.cat([input_ids.to(dev), out], 1)


def _init_single_process():
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        dist.init_process_group("gloo", rank=0, world_size=1)
