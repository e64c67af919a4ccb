"""Llama LightningModule for MI355X (reference: examples/training/llama/lightning/module_llama.py):
NeuronLTModule (model / optimizer through the NxD trainer API, PP schedule when PP > 1) plus the
reference's per-step logging -- loss, lr, global grad norm and throughput in sequences/s and
tokens/s (the BASELINE metric) -- from the rank that owns the loss."""

from __future__ import annotations

import time

from neuronx_distributed_llama3_2_amd.lightning import NeuronLTModule
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps


class NeuronLlamaLTModule(NeuronLTModule):
    def __init__(self, *args, seq_len: int = 4096, **kwargs):
        super().__init__(*args, **kwargs)
        self.seq_len = seq_len
        self._t_last = None
        self.history = []        # (step, loss, seq/s) on the logging rank

    def on_train_batch_start(self, batch, batch_idx):
        if self._t_last is None:
            self._t_last = time.perf_counter()

    def on_train_batch_end(self, outputs, batch, batch_idx):
        now = time.perf_counter()
        dt, self._t_last = now - self._t_last, now
        seqs = self.train_batch_size * ps.get_data_parallel_size()
        if self.loss is not None and self._should_log():
            opt = self.optimizers()
            lr = opt.param_groups[0]["lr"] if hasattr(opt, "param_groups") else None
            self.history.append((int(self.global_step), float(self.loss), seqs / max(dt, 1e-9)))
            self.log("lr", lr, rank_zero_only=False)
            self.log("throughput_seq_per_s", seqs / max(dt, 1e-9), rank_zero_only=False)
            self.log("throughput_tokens_per_s", seqs * self.seq_len / max(dt, 1e-9), rank_zero_only=False)
