"""NxDModel: uniform training wrapper over a plain or pipeline-parallel model
(reference: src/neuronx_distributed/trainer/model.py:8-116)."""

from __future__ import annotations

from typing import Any

import torch


class NxDModel(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, nxd_config):
        super().__init__()
        self.module = module
        self.nxd_config = nxd_config
        self.pp_enabled = nxd_config["pipeline_parallel_size"] > 1
        if not self.pp_enabled:
            self.train()

    def __repr__(self):
        return f"NxDModel({self.module!r})"

    def local_modules(self):
        return self.module.local_stage_modules if self.pp_enabled else [self.module]

    def original_module(self):
        return self.module.original_torch_module if self.pp_enabled else self.module

    def run_train(self, *args, **kwargs):
        if self.pp_enabled:
            return self.module.run_train(*args, **kwargs)
        out = self.forward(*args, **kwargs)
        loss = out.loss if hasattr(out, "loss") else (out[0] if isinstance(out, (tuple, list)) else out)
        loss.backward()
        return loss

    def run_eval(self, *args, **kwargs):
        assert self.pp_enabled, "`run_eval` should be used only when pipeline parallel is enabled."
        return self.module.run_eval(*args, **kwargs)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def named_parameters(self, *args, **kwargs):
        if self.pp_enabled:
            yield from self.module.local_named_parameters(*args, **kwargs)
            return
        yield from self.module.named_parameters(*args, **kwargs)

    def named_buffers(self, *args, **kwargs):
        if self.pp_enabled:
            yield from self.module.local_named_buffers(*args, **kwargs)
            return
        yield from self.module.named_buffers(*args, **kwargs)

    def named_children(self):
        if self.pp_enabled:
            yield from self.module.local_named_children()
            return
        yield from self.module.named_children()

    def named_modules(self, *args, **kwargs):
        if self.pp_enabled:
            yield from self.module.local_named_modules(*args, **kwargs)
            return
        yield from self.module.named_modules(*args, **kwargs)

    def state_dict(self, *args, **kwargs):
        if self.pp_enabled:
            return self.module.local_state_dict(*args, **kwargs)
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True):
        return self.module.load_state_dict(state_dict, strict=strict)

    def __getattr__(self, name: str) -> Any:
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)

    @property
    def dtype(self):
        return next(self.original_module().parameters()).dtype

    @property
    def config(self):
        return self.original_module().config
