"""Training-loop utilities of the example scripts: LR schedules, weight-decay param groups,
throughput meter, JSON metrics file, dataset packing / loading, PP layer partitioning
(reference: examples/training/llama/training_utils.py:29-359, lr.py:25-190).

Throughput is reported both as the reference's seq/s (moving window over `moving_avg_window_size`
steps, seqs = batch x DP x grad_accum x logging_interval) and as tokens/s (the BASELINE metric).
"""

from __future__ import annotations

import json
import math
import os
import time
from collections import deque
from dataclasses import dataclass, field
from itertools import chain
from typing import Any, Dict, Iterable, List, Optional

import torch
from torch.optim.lr_scheduler import LambdaLR


# ------------------------------------------------------------------------------------------ LR
def warmup_cosine_lambda(warmup_steps: int, max_steps: int, min_ratio: float = 0.0, constant_steps: int = 0,
                         hold_steps: int = 0):
    """Multiplier schedule: linear warmup to 1, optional hold, cosine decay to `min_ratio` at
    max_steps - constant_steps, then constant at min_ratio."""
    decay_end = max(warmup_steps + hold_steps + 1, max_steps - constant_steps)

    def f(step: int) -> float:
        if warmup_steps > 0 and step < warmup_steps:
            return (step + 1) / warmup_steps
        if step < warmup_steps + hold_steps:
            return 1.0
        if step >= decay_end:
            return min_ratio
        t = (step - warmup_steps - hold_steps) / max(1, decay_end - warmup_steps - hold_steps)
        return min_ratio + (1.0 - min_ratio) * 0.5 * (1.0 + math.cos(math.pi * t))

    return f


class CosineAnnealing(LambdaLR):
    """Warmup + cosine annealing to `min_lr` (reference lr.py CosineAnnealing / WarmupAnnealHoldPolicy)."""

    def __init__(self, optimizer, *, max_steps: int, min_lr: float = 0.0, warmup_steps: int = 0,
                 constant_steps: int = 0, hold_steps: int = 0, last_epoch: int = -1):
        base = optimizer.param_groups[0]["lr"]
        ratio = (min_lr / base) if base > 0 else 0.0
        super().__init__(optimizer, warmup_cosine_lambda(warmup_steps, max_steps, ratio, constant_steps, hold_steps),
                         last_epoch=last_epoch)


def get_learning_rate_scheduler(optimizer, args, last_epoch: int = -1):
    """Linear warmup then linear decay to 0 at max_steps (reference training_utils.py:65-74), or
    cosine when `args.lr_schedule == "cosine"`."""
    warm = int(getattr(args, "warmup_steps", 0))
    total = int(getattr(args, "max_steps", 1))
    if getattr(args, "lr_schedule", "linear") == "cosine":
        return CosineAnnealing(optimizer, max_steps=total, min_lr=float(getattr(args, "min_lr", 0.0)),
                               warmup_steps=warm, last_epoch=last_epoch)

    def lin(step):
        if step < warm:
            return float(step + 1) / max(1, warm)
        return max(0.0, float(total - step) / max(1, total - warm))

    return LambdaLR(optimizer, lin, last_epoch=last_epoch)


def get_param_groups_by_weight_decay(model, weight_decay: float = 0.01,
                                     no_decay=("bias", "LayerNorm", "layernorm", "norm")):
    decay, nodecay = [], []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (nodecay if (p.dim() <= 1 or any(k in n for k in no_decay)) else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": nodecay, "weight_decay": 0.0}]


# ------------------------------------------------------------------------------------------ meters
class Throughput:
    def __init__(self, batch_size: int, world_size: int, grad_accum_usteps: int, moving_avg_window_size: int = 10,
                 logging_interval: int = 1, seq_len: Optional[int] = None):
        self.seqs_per_iteration = batch_size * world_size * grad_accum_usteps * logging_interval
        self.seq_len = seq_len
        self.window = deque(maxlen=max(1, math.ceil(moving_avg_window_size / logging_interval)))
        self.start_time = time.time()

    def get_throughput(self) -> float:
        """seq/s over the moving window (call once per logged step)."""
        now = time.time()
        self.window.append(now - self.start_time)
        self.start_time = now
        return len(self.window) * self.seqs_per_iteration / max(1e-9, sum(self.window))

    def tokens_per_second(self, seqs_per_s: float) -> Optional[float]:
        return seqs_per_s * self.seq_len if self.seq_len else None


@dataclass
class Metric:
    name: str
    value: Any
    units: str = ""
    additional_data: Dict[str, Any] = field(default_factory=dict)


class TrainingMetrics:
    """JSON results file {"results": {"parameters": {...}, "metrics": [...]}} (reference schema)."""

    def __init__(self, json_file: str):
        self.json_file = json_file

    def _read(self) -> Dict[str, Any]:
        if os.path.exists(self.json_file):
            with open(self.json_file) as f:
                txt = f.read().strip()
            if txt:
                return json.loads(txt)
        return {}

    def read_modify_write_file(self, data, key: str = "metrics") -> None:
        d = self._read()
        res = d.setdefault("results", {})
        cur = res.get(key)
        if cur is None:
            res[key] = data
        elif isinstance(cur, list):
            cur.extend(data)
        elif isinstance(cur, dict):
            cur.update(data)
        os.makedirs(os.path.dirname(os.path.abspath(self.json_file)), exist_ok=True)
        with open(self.json_file, "w") as f:
            json.dump(d, f, indent=2, default=str)

    def store_metrics(self, metrics: List[Metric]) -> None:
        self.read_modify_write_file([{"MetricName": m.name, "MeasuredValue": m.value, "Units": m.units,
                                      "AdditionalData": m.additional_data} for m in metrics])

    def store_parameters(self, parameters: Dict[str, Any]) -> None:
        self.read_modify_write_file(parameters, "parameters")

    def update(self, **kwargs) -> None:
        self.read_modify_write_file(kwargs, "parameters")


# ------------------------------------------------------------------------------------------ data
def pack_dataset(dataset, chunk_length: int = 2048):
    """Concatenate a tokenized HF dataset and cut it into `chunk_length` windows (+labels);
    the remainder of each map batch is carried into the next batch."""
    carry: Dict[str, list] = {}

    def chunk(sample):
        cat = {k: carry.get(k, []) + list(chain(*sample[k])) for k in sample.keys()}
        n = (len(cat[next(iter(cat))]) // chunk_length) * chunk_length
        out = {k: [t[i:i + chunk_length] for i in range(0, n, chunk_length)] for k, t in cat.items()}
        for k, t in cat.items():
            carry[k] = t[n:]
        out["labels"] = [list(x) for x in out["input_ids"]]
        return out

    return dataset.map(chunk, batched=True, remove_columns=list(dataset.column_names))


class SyntheticTokenDataset(torch.utils.data.Dataset):
    """Deterministic random token sequences (the benchmark's synthetic data)."""

    def __init__(self, vocab_size: int, seq_len: int, num_samples: int = 1 << 20, seed: int = 0):
        self.vocab_size, self.seq_len, self.n, self.seed = vocab_size, seq_len, num_samples, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        ids = torch.randint(0, self.vocab_size, (self.seq_len,), generator=g)
        return {"input_ids": ids, "labels": ids.clone(), "attention_mask": torch.ones_like(ids)}


def create_llama_pretraining_dataset(data_dir: str, mini_batch_size: int, dp_size: int, dp_rank: int, seed: int,
                                     num_workers: int = 0):
    """DataLoader over a tokenized, packed HF dataset saved with `save_to_disk` (no network),
    sharded over DP ranks."""
    import datasets
    from torch.utils.data import DataLoader, DistributedSampler

    ds = datasets.load_from_disk(os.path.expanduser(data_dir))
    ds.set_format("torch", columns=[c for c in ("input_ids", "labels", "attention_mask") if c in ds.column_names])
    sampler = DistributedSampler(ds, num_replicas=dp_size, rank=dp_rank, shuffle=True, seed=seed, drop_last=True)
    return DataLoader(ds, batch_size=mini_batch_size, sampler=sampler, num_workers=num_workers, pin_memory=True,
                      drop_last=True), sampler


def create_partition(num_hidden_layers: int, pipeline_parallel_size: int) -> List[str]:
    """Pipeline cut points: names of the last decoder layer of every stage but the last (layers
    spread evenly, remainder to the later stages)."""
    base, rem = divmod(num_hidden_layers, pipeline_parallel_size)
    sizes = [base + (1 if s >= pipeline_parallel_size - rem else 0) for s in range(pipeline_parallel_size)]
    cuts, acc = [], 0
    for s in sizes[:-1]:
        acc += s
        cuts.append(f"model.layers.{acc - 1}")
    return cuts


def get_dtype(model) -> str:
    p = next(model.parameters())
    return str(p.dtype).replace("torch.", "")


def sample_num_spans(rng, max_num_spans: int = 16) -> int:
    """1 + Poisson(1) spans, capped (reference: examples/training/codegen25/get_dataset_infill.py:35-39)."""
    return int(min(int(rng.poisson(1.0)) + 1, max_num_spans))


def format_to_infill(tokens: List[int], num_spans: int, mask_ids: List[int], eom_id: int, sep_ids: List[int],
                     rng) -> Optional[List[int]]:
    """Causal-infilling ("fill in the middle") rewrite of one token sequence, CodeGen2.5 style:
    `prefix-with-<mask_i>-holes ++ sep_ids ++ (<mask_i> span_i <eom>)...`.  Spans are sampled left to
    right, at least one token apart; returns None when the sequence is too short for `num_spans`.
    Token ids instead of a tokenizer (reference behaviour: get_dataset_infill.py:42-90)."""
    max_len = (len(tokens) - num_spans) // num_spans
    if max_len <= 0 or num_spans > len(mask_ids):
        return None
    start_lo, end_hi = 1, max_len
    prefix: List[int] = []
    suffix: List[int] = []
    for i in range(num_spans):
        n = int(rng.integers(1, max_len + 1))
        start = int(rng.integers(start_lo, end_hi - n + 2))
        span = tokens[start:start + n]
        prefix += tokens[start_lo - 1:start] + [mask_ids[i]]
        suffix += [mask_ids[i]] + span + [eom_id]
        start_lo, end_hi = start + n + 1, start + n + max_len
        if i == num_spans - 1:
            prefix += tokens[start + n:]
    return prefix + list(sep_ids) + suffix


def infill_token_blocks(blocks: Iterable[List[int]], block_size: int, mask_ids: List[int], eom_id: int,
                        sep_ids: List[int], seed: int = 42, fraction: float = 0.5,
                        max_num_spans: int = 16) -> List[List[int]]:
    """Apply `format_to_infill` to `fraction` of the blocks, keeping every block at `block_size`
    tokens: each span adds two masks and one <eom>, so only the first block_size - extra tokens are
    rewritten (reference: get_dataset_infill.py:103-137)."""
    import numpy as np

    rng = np.random.default_rng(seed)
    out = []
    for b in blocks:
        b = list(b)
        if rng.random() < fraction:
            k = sample_num_spans(rng, max_num_spans)
            extra = 3 * k + len(sep_ids)
            filled = format_to_infill(b[:block_size - extra], k, mask_ids, eom_id, sep_ids, rng)
            if filled is not None:
                b = (filled + b[block_size - extra:])[:block_size]
        out.append(b[:block_size])
    return out


# ------------------------------------------------------------------ instruction fine-tuning data
def format_instruction(sample: Dict[str, Any], with_answer: bool = True) -> str:
    """Dolly-style prompt (reference: examples/training/llama/training_utils.py:130-207):
    '### Instruction' / optional '### Context' / '### Answer' sections joined by newlines."""
    parts = [f"### Instruction\n{sample['instruction']}"]
    if sample.get("context"):
        parts.append(f"### Context\n{sample['context']}")
    parts.append(f"### Answer\n{sample['response']}" if with_answer else "### Answer\n")
    return "\n".join(parts)


def build_instruction_datasets(records: List[Dict[str, Any]], tokenizer, chunk_length: int = 2048,
                               test_size: int = 8, seed: int = 0):
    """-> (train windows, test examples).

    Train: every record rendered with its answer + EOS, tokenized, concatenated and cut into
    `chunk_length` windows (labels = inputs; the tail shorter than a window is dropped).
    Test (the last `test_size` records of a seeded shuffle): prompt ids without the answer and the
    answer ids as labels, for response-only loss / generation checks."""
    import random

    recs = list(records)
    random.Random(seed).shuffle(recs)
    test, train = recs[len(recs) - test_size:] if test_size else [], recs[:len(recs) - test_size]
    eos = tokenizer.eos_token or ""
    stream: List[int] = []
    for r in train:
        stream += tokenizer(format_instruction(r) + eos)["input_ids"]
    n = (len(stream) // chunk_length) * chunk_length
    windows = [stream[i:i + chunk_length] for i in range(0, n, chunk_length)]
    tests = [{"input_ids": tokenizer(format_instruction(r, with_answer=False), add_special_tokens=False)["input_ids"],
              "labels": tokenizer(r["response"], add_special_tokens=False)["input_ids"]} for r in test]
    return windows, tests
