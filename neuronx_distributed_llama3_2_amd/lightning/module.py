"""LightningModule wrapper that builds the model / optimizer through the NxD trainer API and runs
the pipeline-parallel schedule when PP > 1 (reference: lightning/module.py NeuronLTModule)."""

from typing import Any, Callable, Dict, Optional, Tuple

import torch

from ..parallel_layers import parallel_state as ps
from ..trainer import initialize_parallel_model, initialize_parallel_optimizer
from ..trainer.optimizer import NxDOptimizer
from ..utils.training_utils import get_param_groups_by_weight_decay
from ._compat import pl, require_lightning

require_lightning()


class NeuronLTModule(pl.LightningModule):
    def __init__(self, nxd_config: Dict, opt_cls: Callable, scheduler_cls: Callable, model_args: Tuple = (),
                 model_kwargs: Optional[Dict] = None, opt_args: Tuple = (), opt_kwargs: Optional[Dict] = None,
                 scheduler_args: Tuple = (), scheduler_kwargs: Optional[Dict] = None,
                 model_fn: Optional[Callable[..., Any]] = None, grad_accum_steps: int = 1,
                 train_batch_size: int = 16, logging_interval: int = 1, log_rank0: bool = False,
                 manual_opt: bool = True, weight_decay: float = 0.01):
        super().__init__()
        self.nxd_config, self.model_fn = nxd_config, model_fn
        self.opt_cls, self.scheduler_cls = opt_cls, scheduler_cls
        self.model_args, self.model_kwargs = model_args, dict(model_kwargs or {})
        self.opt_args, self.opt_kwargs = opt_args, dict(opt_kwargs or {})
        self.scheduler_args, self.scheduler_kwargs = scheduler_args, dict(scheduler_kwargs or {})
        self.grad_accum_steps, self.train_batch_size = grad_accum_steps, train_batch_size
        self.logging_interval, self.log_rank0, self.weight_decay = logging_interval, log_rank0, weight_decay
        self.automatic_optimization = not manual_opt
        self.model = None
        self.loss = self.lr = self.global_norm = None

    def setup(self, stage=None):
        if self.model is None:
            self.model = initialize_parallel_model(self.nxd_config, self.model_fn, *self.model_args,
                                                   **self.model_kwargs)

    def forward(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def configure_optimizers(self):
        groups = get_param_groups_by_weight_decay(self.model, self.weight_decay)
        opt = initialize_parallel_optimizer(self.nxd_config, self.opt_cls, groups, *self.opt_args, **self.opt_kwargs)
        sch = self.scheduler_cls(opt, *self.scheduler_args, **self.scheduler_kwargs)
        return [opt], [{"scheduler": sch, "interval": "step"}]

    def configure_gradient_clipping(self, *args, **kwargs):   # the NxD optimizer clips (TP/PP aware)
        pass

    def training_step(self, batch, batch_idx):
        opt = self.optimizers()
        while not isinstance(opt, NxDOptimizer) and hasattr(opt, "optimizer"):   # LightningOptimizer wrapper
            opt = opt.optimizer
        pp = ps.get_pipeline_model_parallel_size() > 1
        if pp:
            loss = self.model.run_train(**batch)
        else:
            loss = None
            for i in range(self.grad_accum_steps):
                opt.set_grad_sync(i == self.grad_accum_steps - 1)
                mb = {k: v.chunk(self.grad_accum_steps)[i] for k, v in batch.items()}
                out = self.model(**mb)
                (out.loss / self.grad_accum_steps).backward()
                loss = out.loss.detach() if loss is None else loss + out.loss.detach()
            loss = loss / self.grad_accum_steps
        opt.step()
        opt.zero_grad()
        sch = self.lr_schedulers()
        if sch is not None:
            sch.step()
        self.loss, self.global_norm = loss, getattr(opt, "grad_norm", None)
        if self.global_step % self.logging_interval == 0 and loss is not None and self._should_log():
            self.log("loss", float(loss), prog_bar=True, rank_zero_only=False)
            if self.global_norm is not None:
                self.log("global_norm", float(self.global_norm), rank_zero_only=False)
        return loss

    def _should_log(self) -> bool:
        # the loss lives on the last pipeline stage; log from its (tp 0, dp 0) rank
        return (ps.get_pipeline_model_parallel_rank() == ps.get_pipeline_model_parallel_size() - 1
                and ps.get_tensor_model_parallel_rank() == 0 and ps.get_data_parallel_rank() == 0)

    def state_dict(self, *args, **kwargs):
        return self.model.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True):
        return self.model.load_state_dict(state_dict, strict=strict)
