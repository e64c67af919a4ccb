"""NxDOptimizer: the optimizer wrapper of the training API
(reference: src/neuronx_distributed/trainer/optimizer.py:10-154).

* flat-buffer optimizers (ZeRO-1 / master weights): `step()` delegates — gradient reduction,
  sequence-parallel all-reduce, clipping and the fused update all happen inside;
* plain torch optimizers: `step()` performs the reference sequence — SP norm-grad all-reduce over
  TP, bucketed DP all-reduce (expert grads over expert-DP), grad clipping — then the inner step.
`grad_norm` exposes the last global gradient norm (a device tensor; no host sync).
`no_sync()` / `set_grad_sync(False)` suppress DP reduction during gradient accumulation.
"""

from __future__ import annotations

import contextlib
from typing import Any, Dict

import torch

from ..parallel import comm
from ..parallel_layers import parallel_state, stream_split
from ..parallel_layers.grads import allreduce_sequence_parallel_gradients, bucket_allreduce_gradients, clip_grad_norm


class NxDOptimizer(torch.optim.Optimizer):
    def __init__(self, optimizer, nxd_config: Dict[str, Any]):
        self.optimizer = optimizer
        self.nxd_config = nxd_config
        self._grad_norm = None
        self._flat = hasattr(optimizer, "buffers")
        self._sync = True

    # torch.optim.Optimizer surface
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @param_groups.setter
    def param_groups(self, v):
        self.optimizer.param_groups = v

    @property
    def state(self):
        return self.optimizer.state

    @property
    def defaults(self):
        return self.optimizer.defaults

    @property
    def grad_norm(self):
        if self._flat:
            return getattr(self.optimizer, "grad_norm", None)
        return self._grad_norm

    def set_grad_sync(self, enabled: bool) -> None:
        self._sync = enabled
        if hasattr(self.optimizer, "set_grad_sync"):
            self.optimizer.set_grad_sync(enabled)

    @contextlib.contextmanager
    def no_sync(self):
        self.set_grad_sync(False)
        try:
            yield
        finally:
            self.set_grad_sync(True)

    def _params(self):
        return [p for g in self.optimizer.param_groups for p in g["params"]]

    @torch.no_grad()
    def step(self, closure=None):
        # the two sequence-parallel halves' streams (parallel_layers/stream_split.py) end the
        # backward and write main_grad: every optimizer kind reads gradients after them
        stream_split.join()
        comm.check_peer_collectives()   # a lost peer (NXD_SP_PEER) raises before its NaN grads are applied
        if self._flat:
            return self.optimizer.step(closure)
        params = self._params()
        allreduce_sequence_parallel_gradients(params)
        grads = [p.grad for p in params if p.grad is not None and not getattr(p, "expert_model_parallel", False)]
        bucket_allreduce_gradients(grads)
        dp = parallel_state.get_data_parallel_size() if parallel_state.model_parallel_is_initialized() else 1
        if dp > 1:
            torch._foreach_div_(grads, float(dp)) if grads else None
        ep_grads = [p.grad for p in params if p.grad is not None and getattr(p, "expert_model_parallel", False)]
        if ep_grads:
            bucket_allreduce_gradients(ep_grads, reduce_over_ep_group=True)
        ocfg = self.nxd_config["optimizer_config"]
        if ocfg.get("grad_clipping", False):
            self._grad_norm = clip_grad_norm(params, ocfg.get("max_grad_norm", 1.0))
        return self.optimizer.step(closure)

    def zero_grad(self, set_to_none: bool = True):
        stream_split.join()
        return self.optimizer.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, state_dict):
        return self.optimizer.load_state_dict(state_dict)

    def add_param_group(self, group):
        return self.optimizer.add_param_group(group)

    def __repr__(self):
        return f"NxDOptimizer({self.optimizer!r})"

    def __getstate__(self):
        return self.__dict__

    def __setstate__(self, d):
        self.__dict__.update(d)
