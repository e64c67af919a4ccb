"""Sequence-length bucketing (reference: examples/inference/modules/autobucketing.py:6-126).

Buckets are powers of two from the minimum up to (and including) the maximum length.  Prompts are
right-padded to the smallest bucket that holds the longest prompt of the batch so the context
encoder sees a handful of distinct shapes (stable allocator pools, reusable GEMM heuristics); the
decode path needs no length buckets because attention reads the KV cache up to a per-sequence
device-side length.
"""

from __future__ import annotations

from math import log2
from typing import List, Sequence

import torch


def generate_buckets(min_length: int, max_length: int) -> List[int]:
    if min_length >= max_length:
        return [max_length]
    lo = int(log2(min_length))
    hi = round(log2(max_length))
    return [2 ** i for i in range(lo, hi)] + [max_length]


def select_bucket(length: int, buckets: Sequence[int]) -> int:
    for b in sorted(buckets):
        if length <= b:
            return b
    raise ValueError(f"length {length} exceeds the largest bucket {max(buckets)}")


def pad_to_bucket(input_ids: torch.Tensor, attention_mask: torch.Tensor, buckets: Sequence[int], pad_token: int):
    """Right-pad [B, T] ids / mask to the selected bucket length."""
    T = input_ids.shape[1]
    b = select_bucket(T, buckets)
    if b == T:
        return input_ids, attention_mask
    pad = b - T
    ids = torch.nn.functional.pad(input_ids, (0, pad), value=pad_token)
    mask = torch.nn.functional.pad(attention_mask, (0, pad), value=0)
    return ids, mask
