"""GQA sharding strategies for tensor parallelism (reference: examples/inference/modules/gqa.py:19-75).

* REPLICATE_TO_TP_DEGREE (default): K/V heads are replicated just enough that every TP rank owns
  whole K/V heads (8 K/V heads at TP=32 -> 32); the Q heads of a group stay with their K/V head.
  Needs (replicated K/V heads) % TP == 0, i.e. TP % num_kv_heads == 0 when TP > num_kv_heads.
* CONVERT_TO_MHA: every Q head gets its own copy of its K/V head (GQA -> MHA).  More K/V memory,
  but it shards at any TP degree that divides the head count.

`kv_size_multiplier` is the factor the framework's GQAQKVColumnParallelLinear replicates the K/V
projection by (modules/qkv_linear.py); the replicated heads are consecutive copies, which keeps
query head i on the rank of its K/V head for both strategies.
"""

from __future__ import annotations

import enum
import math
from typing import Optional, Tuple, Union

import torch


class GQA(enum.Enum):
    CONVERT_TO_MHA = "convert-to-mha"
    REPLICATE_TO_TP_DEGREE = "replicate-to-tp-degree"


def _as_strategy(s: Union[None, str, GQA]) -> Optional[GQA]:
    if s is None or isinstance(s, GQA):
        return s
    return GQA(str(s).lower().replace("_", "-"))


def determine_sharding_strategy(tp_degree: int, source_key_value_heads: int,
                                desired_sharding_strategy: Union[None, str, GQA] = None) -> GQA:
    """Reference rule: REPLICATE_TO_TP_DEGREE unless TP is not a multiple of the K/V head count
    (when TP > K/V heads), which falls back to CONVERT_TO_MHA."""
    strategy = _as_strategy(desired_sharding_strategy) or GQA.REPLICATE_TO_TP_DEGREE
    if strategy == GQA.REPLICATE_TO_TP_DEGREE and tp_degree > source_key_value_heads and \
            tp_degree % source_key_value_heads != 0:
        strategy = GQA.CONVERT_TO_MHA
    return strategy


def get_shardable_head_counts(tp_degree: int, num_attention_heads: int, num_key_value_heads: int,
                              sharding_strategy: Union[str, GQA]) -> Tuple[int, int]:
    """(attention heads, K/V heads) after the strategy's replication (no head padding: the Q
    head count must already divide by TP)."""
    strategy = _as_strategy(sharding_strategy)
    if num_attention_heads % tp_degree:
        raise ValueError(f"num_attention_heads ({num_attention_heads}) must be divisible by tp_degree ({tp_degree})")
    if num_attention_heads == num_key_value_heads:
        return num_attention_heads, num_key_value_heads
    if strategy == GQA.CONVERT_TO_MHA:
        return num_attention_heads, num_attention_heads
    if num_key_value_heads < tp_degree or num_key_value_heads % tp_degree:
        mult = tp_degree // math.gcd(tp_degree, num_key_value_heads)
        return num_attention_heads, num_key_value_heads * mult
    return num_attention_heads, num_key_value_heads


def kv_size_multiplier(tp_degree: int, num_attention_heads: int, num_key_value_heads: int,
                       sharding_strategy: Union[None, str, GQA] = None, minimum: int = 1) -> int:
    """Replication factor of the K/V projection for the chosen strategy."""
    strategy = determine_sharding_strategy(tp_degree, num_key_value_heads, sharding_strategy)
    _, kv = get_shardable_head_counts(tp_degree, num_attention_heads, num_key_value_heads, strategy)
    return max(minimum, kv // num_key_value_heads)


def replicate_kv(tensor, source_heads: int, repeats: int, head_dim: int = 0):
    """Repeat every K/V head `repeats` times in place along `head_dim` (heads are contiguous blocks
    of that dim): [K0, K1] -> [K0, K0, K1, K1] for repeats 2."""
    if tensor is None or repeats == 1:
        return tensor
    shape = tensor.shape[:head_dim] + (source_heads, tensor.shape[head_dim] // source_heads) + tensor.shape[head_dim + 1:]
    t = tensor.reshape(shape).repeat_interleave(repeats, dim=head_dim)
    return t.reshape(tensor.shape[:head_dim] + (-1,) + tensor.shape[head_dim + 1:])


def convert_state_dict_to_mha(full_sd, num_attention_heads: int, num_key_value_heads: int, head_dim: int):
    """CONVERT_TO_MHA on a full (unsharded) framework state dict: the K/V rows of every fused
    `qkv_proj.{weight,bias}_qkv` are replicated so query head i gets its own copy of its K/V head
    (i // group); the model is then built with num_key_value_heads = num_attention_heads."""
    g = num_attention_heads // num_key_value_heads
    if g == 1:
        return dict(full_sd)
    out = {}
    qd, kd = num_attention_heads * head_dim, num_key_value_heads * head_dim
    for k, v in full_sd.items():
        if k.endswith("qkv_proj.weight_qkv") or k.endswith("qkv_proj.bias_qkv"):
            q, kk, vv = v.split([qd, kd, kd], dim=0)
            v = torch.cat([q, replicate_kv(kk, num_key_value_heads, g), replicate_kv(vv, num_key_value_heads, g)], 0)
        out[k] = v
    return out
