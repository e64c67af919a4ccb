"""Per-GPU training memory planner for Llama-family models on MI355X (288 GB HBM3E per GPU).

The reference sizes its configs by trial on 16-32 GB NeuronCores (activation checkpointing,
PP, the long-sequence memory ceilings in test/integration/llama2_7B/test_long_seqlen.py:87-89).
With 288 GB per GPU the question changes to "which recompute / pipeline stages can be dropped",
so this module answers it from measured coefficients of THIS framework's training step:

* resident bytes per parameter (`RESIDENT_BYTES_PER_PARAM`): bf16 weight 2 + K-major dgrad copy 2
  (ops/gemm.py) + fp32 main grad 4 + fp32 master 4 + Adam m, v 8 -- the last 12 sharded over DP
  under ZeRO-1;
* activation bytes per token per decoder layer, in units of the hidden size h
  (`ACT_COEF`): measured at S = 8192 by tools/measure_activation_memory.py
  (profiles/r2_activation_memory.jsonl): Llama-3-8B TP=1 34.0 h without recompute (flash
  attention keeps no S x S matrix, so "selective" recompute saves nothing) and 4.0 h with full
  recompute; Llama-3-70B at TP=8 per-rank shapes 11.2 h, which splits the 34 h into 7.9 h of
  hidden-sized tensors and 26.1 h of tensor-parallel tensors (QKV, attention output, gate/up,
  SwiGLU: divided by TP).  Of the hidden-sized 7.9 h, the two normalised inputs of the
  column-parallel projections (4 h) are kept all-gathered under sequence parallelism when the
  layers save the gathered input for the weight gradient (parallel_layers/layers.py, the default:
  no re-gather in backward), the rest (3.9 h: residuals, norm inputs) is divided by TP;
* fixed activation bytes: logits + loss, 2.5 bytes per (token, local vocab entry) measured.

Calibration check: Llama-3-8B TP=1 mbs 1 plans to 186 GiB against the 189.0 GiB peak bench.py
measures (profiles/r2_bench_1gpu_v4.log).  Llama-3-70B at TP=8 with sequence parallelism plans to
203 GiB at 1 sequence per micro-batch (187 GiB without the saved gathered inputs): it trains on ONE
8-GPU node without pipeline stages and without activation recompute (the reference runs it at
TP=32 x PP=8).
"""

from __future__ import annotations

import math
from dataclasses import asdict, dataclass
from typing import Optional

HBM_BYTES_MI355X = 288 * 10**9

RESIDENT_BYTES_PER_PARAM = {"weight": 2.0, "dgrad_kmajor": 2.0, "main_grad": 4.0, "master": 4.0, "adam_moments": 8.0}
ACT_COEF = {   # x h bytes per token per layer
    "none": {"sp_split": 3.9, "gathered": 4.0, "tp_split": 26.1},
    "selective": {"sp_split": 3.9, "gathered": 4.0, "tp_split": 26.1},
    "full": {"sp_split": 4.0, "gathered": 0.0, "tp_split": 0.0},
}
LOGIT_BYTES = 2.5  # per (token, local vocab entry): bf16 logits + fp32 loss workspace
GIB = 2**30


@dataclass
class MemoryPlan:
    params_per_rank: int
    resident_bytes: float
    activation_bytes: float
    fixed_activation_bytes: float
    total_bytes: float
    hbm_bytes: float
    layers_per_stage: int
    in_flight_microbatches: int

    @property
    def fits(self) -> bool:
        return self.total_bytes <= self.hbm_bytes

    @property
    def headroom_bytes(self) -> float:
        return self.hbm_bytes - self.total_bytes

    def summary(self) -> dict:
        d = asdict(self)
        d.update(total_gib=round(self.total_bytes / GIB, 1), fits=self.fits,
                 headroom_gib=round(self.headroom_bytes / GIB, 1))
        return d


def _cfg(cfg, name, default=None):
    return getattr(cfg, name, default) if not isinstance(cfg, dict) else cfg.get(name, default)


def params_per_rank(cfg, tp: int = 1, pp: int = 1, stage: Optional[int] = None) -> int:
    """Parameters held by one rank: decoder layers of its pipeline stage (the first stage also the
    embedding, the last the final norm + lm_head; default: the larger of the two end stages)."""
    h = _cfg(cfg, "hidden_size")
    nh = _cfg(cfg, "num_attention_heads")
    nkv = _cfg(cfg, "num_key_value_heads", nh)
    hd = _cfg(cfg, "head_dim", None) or h // nh
    inter = _cfg(cfg, "intermediate_size")
    vocab = _cfg(cfg, "vocab_size")
    L = _cfg(cfg, "num_hidden_layers")
    tied = bool(_cfg(cfg, "tie_word_embeddings", False))
    kv_local = max(1, nkv // tp) if nkv < tp else nkv // tp  # KV heads replicated up to the TP degree
    per_layer = (h * (nh // tp + 2 * kv_local) * hd      # fused QKV (column parallel)
                 + nh // tp * hd * h                      # o_proj (row parallel)
                 + 2 * h * (inter // tp) + (inter // tp) * h  # gate_up + down
                 + 2 * h)                                 # two RMSNorm weights (replicated)
    lps = math.ceil(L / pp)
    emb = math.ceil(vocab / tp) * h
    head = h + (0 if tied and pp == 1 else emb)
    if pp == 1:
        return per_layer * L + emb + head
    first, last = per_layer * lps + emb, per_layer * lps + head
    if stage is None:
        return max(first, last)
    return first if stage == 0 else (last if stage == pp - 1 else per_layer * lps)


def plan_training_memory(cfg, tp: int = 1, pp: int = 1, dp: int = 1, mbs: int = 1, seq: int = 8192,
                         sequence_parallel: Optional[bool] = None, activation_checkpoint: Optional[str] = None,
                         zero1: bool = True, num_microbatches: int = 1, save_gathered_input: bool = True,
                         hbm_bytes: float = HBM_BYTES_MI355X) -> MemoryPlan:
    """Peak bytes of one rank of a TP x PP x DP training job (fp32-master AdamW, bf16 compute)."""
    if sequence_parallel is None:
        sequence_parallel = tp > 1
    mode = activation_checkpoint or "none"
    if mode not in ACT_COEF:
        raise ValueError(f"activation_checkpoint must be None | 'selective' | 'full', got {activation_checkpoint!r}")
    h = _cfg(cfg, "hidden_size")
    vocab = _cfg(cfg, "vocab_size")
    L = _cfg(cfg, "num_hidden_layers")
    n = params_per_rank(cfg, tp, pp)
    r = RESIDENT_BYTES_PER_PARAM
    shard = dp if zero1 else 1
    resident = n * (r["weight"] + r["dgrad_kmajor"] + r["main_grad"] + (r["master"] + r["adam_moments"]) / shard)
    coef = ACT_COEF[mode]
    sp_div = tp if sequence_parallel else 1
    gathered_div = 1 if (save_gathered_input or not sequence_parallel) else tp
    per_token_layer = h * (coef["sp_split"] / sp_div + coef["gathered"] / gathered_div + coef["tp_split"] / tp)
    lps = math.ceil(L / pp)
    # 1F1B: the first stage holds the activations of up to `pp` micro-batches at once
    in_flight = min(pp, max(1, num_microbatches)) if pp > 1 else 1
    act = per_token_layer * lps * seq * mbs * in_flight
    fixed = LOGIT_BYTES * seq * mbs * math.ceil(vocab / tp)
    total = resident + act + fixed
    return MemoryPlan(params_per_rank=n, resident_bytes=resident, activation_bytes=act, fixed_activation_bytes=fixed,
                      total_bytes=total, hbm_bytes=hbm_bytes, layers_per_stage=lps, in_flight_microbatches=in_flight)


def largest_micro_batch(cfg, hbm_bytes: float = HBM_BYTES_MI355X, reserve_fraction: float = 0.08, **kw) -> int:
    """Largest micro-batch (sequences) whose plan leaves `reserve_fraction` of HBM for the caching
    allocator, GEMM workspaces and communication buffers (0 if even one sequence does not fit)."""
    best = 0
    for mbs in range(1, 257):
        p = plan_training_memory(cfg, mbs=mbs, hbm_bytes=hbm_bytes, **kw)
        if p.total_bytes > hbm_bytes * (1.0 - reserve_fraction):
            break
        best = mbs
    return best
