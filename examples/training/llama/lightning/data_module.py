"""LightningDataModule for causal-LM pre-training / fine-tuning on MI355X (reference:
examples/training/llama/lightning/data_module.py).

Data: a packed token dataset saved with `datasets.save_to_disk` (columns `input_ids` [+ `labels`],
one `seq_len` window per row -- the reference's get_dataset output), a `.npy` int array
[rows, seq_len] (memory-mapped), or, with no path, synthetic random token windows (benchmarks /
tests).  Each DP rank reads only its share: the sampler gets (num_replicas, rank) from the
strategy's `distributed_sampler_kwargs`, i.e. the NxD data-parallel group, not the world.
"""

from __future__ import annotations

import os
from typing import Dict, Optional

import torch
from torch.utils.data import DataLoader, Dataset, DistributedSampler

from neuronx_distributed_llama3_2_amd.lightning._compat import pl


class _TokenWindows(Dataset):
    def __init__(self, path: Optional[str], seq_len: int, vocab_size: int, num_rows: int = 1024, seed: int = 1234):
        self.seq_len = seq_len
        self.hf = None
        self.arr = None
        if path and os.path.isdir(path):
            from datasets import load_from_disk

            self.hf = load_from_disk(path)
        elif path and path.endswith(".npy"):
            import numpy as np

            self.arr = np.load(path, mmap_mode="r", allow_pickle=False)
        else:
            g = torch.Generator().manual_seed(seed)
            self.synth = torch.randint(0, vocab_size, (num_rows, seq_len), generator=g)

    def __len__(self):
        if self.hf is not None:
            return len(self.hf)
        if self.arr is not None:
            return int(self.arr.shape[0])
        return int(self.synth.shape[0])

    def __getitem__(self, i) -> Dict[str, torch.Tensor]:
        if self.hf is not None:
            row = self.hf[int(i)]
            ids = torch.tensor(row["input_ids"][:self.seq_len], dtype=torch.long)
            labels = torch.tensor(row.get("labels", row["input_ids"])[:self.seq_len], dtype=torch.long)
        elif self.arr is not None:
            ids = torch.as_tensor(self.arr[int(i)][:self.seq_len].astype("int64"))
            labels = ids
        else:
            ids = labels = self.synth[int(i)]
        return {"input_ids": ids, "labels": labels}


class NeuronLlamaDataModule(pl.LightningDataModule):
    def __init__(self, data_path: Optional[str], seq_len: int, vocab_size: int, train_batch_size: int,
                 num_workers: int = 0, seed: int = 1234, num_synthetic_rows: int = 1024):
        super().__init__()
        self.data_path, self.seq_len, self.vocab_size = data_path, seq_len, vocab_size
        self.train_batch_size, self.num_workers, self.seed = train_batch_size, num_workers, seed
        self.num_synthetic_rows = num_synthetic_rows
        self.train_ds = None

    def setup(self, stage: Optional[str] = None) -> None:
        self.train_ds = _TokenWindows(self.data_path, self.seq_len, self.vocab_size, self.num_synthetic_rows, self.seed)

    def train_dataloader(self) -> DataLoader:
        kw = self.trainer.strategy.distributed_sampler_kwargs if self.trainer is not None else {"num_replicas": 1, "rank": 0}
        sampler = DistributedSampler(self.train_ds, shuffle=True, seed=self.seed, drop_last=True, **kw)
        return DataLoader(self.train_ds, batch_size=self.train_batch_size, sampler=sampler,
                          num_workers=self.num_workers, drop_last=True, pin_memory=torch.cuda.is_available())
