"""A small stand-in for the part of the `lightning.pytorch` 2.x public API that the Lightning
integration touches (Lightning is not installed in this image and cannot be).  `install()` puts it
in sys.modules as `lightning.pytorch`; only the Lightning tests call it, in their own rank processes.

Trainer.fit follows Lightning's order for manual optimisation: strategy launcher -> strategy
setup_distributed -> module.setup / datamodule.setup -> callbacks' setup -> configure_optimizers
(optimizers wrapped like LightningOptimizer) -> _setup_model -> on_train_start -> per batch
(on_train_batch_start, training_step, global_step += 1, on_train_batch_end, callbacks, logger) ->
on_train_end.  Checkpoints are the Lightning dict (state_dict / optimizer_states / lr_schedulers /
global_step) handed to strategy.save_checkpoint.  This pins our code to that call protocol, not
to Lightning's behaviour in general (parity with real Lightning unpinned)."""

from __future__ import annotations

import json
import os
import sys
import types

import torch
import torch.distributed as dist


class LightningModule(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.trainer = None
        self.automatic_optimization = True

    @property
    def global_step(self) -> int:
        return self.trainer.global_step if self.trainer is not None else 0

    def optimizers(self):
        opts = self.trainer.optimizers
        return opts[0] if len(opts) == 1 else opts

    def lr_schedulers(self):
        cfgs = self.trainer.lr_scheduler_configs
        return cfgs[0]["scheduler"] if cfgs else None

    def log(self, name, value, prog_bar=False, rank_zero_only=False, **kw):
        self.trainer.callback_metrics[name] = value

    def setup(self, stage=None):
        pass

    def on_train_start(self):
        pass

    def on_train_end(self):
        pass

    def on_train_batch_start(self, batch, batch_idx):
        pass

    def on_train_batch_end(self, outputs, batch, batch_idx):
        pass


class LightningDataModule:
    def __init__(self):
        self.trainer = None

    def setup(self, stage=None):
        pass


class _LightningOptimizer:
    def __init__(self, optimizer):
        self.optimizer = optimizer

    def __getattr__(self, name):
        return getattr(self.optimizer, name)


class Callback:
    def setup(self, trainer, pl_module, stage):
        pass

    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx):
        pass


class TQDMProgressBar(Callback):
    def __init__(self):
        self.enabled, self.updates = True, 0

    def disable(self):
        self.enabled = False

    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx):
        if self.enabled:
            self.updates += 1


class ModelCheckpoint(Callback):
    def __init__(self, dirpath=None, every_n_train_steps=None, save_top_k=1, **kw):
        self.dirpath, self.every = dirpath, every_n_train_steps

    def on_train_batch_end(self, trainer, pl_module, outputs, batch, batch_idx):
        if self.every and trainer.global_step % self.every == 0:
            trainer.save_checkpoint(os.path.join(self.dirpath, f"step={trainer.global_step}.ckpt"))


class TensorBoardLogger:
    def __init__(self, save_dir=".", name="lightning_logs", **kw):
        self.save_dir = save_dir

    def log_metrics(self, metrics, step=None):
        os.makedirs(self.save_dir, exist_ok=True)
        with open(os.path.join(self.save_dir, f"metrics.{dist.get_rank() if dist.is_initialized() else 0}.jsonl"),
                  "a") as f:
            f.write(json.dumps({"step": step, **metrics}) + "\n")

    def log_hyperparams(self, params, metrics=None):
        pass


class CheckpointIO:
    def __init__(self, *a, **kw):
        pass


class Precision:
    def __init__(self, *a, **kw):
        pass

    def optimizer_step(self, optimizer, model, closure, **kwargs):
        closure()
        return optimizer.step(**kwargs)


class CUDAAccelerator:
    pass


class _Launcher:
    pass


class DDPStrategy:
    def __init__(self, process_group_backend=None, checkpoint_io=None, **kw):
        self._process_group_backend = process_group_backend
        self.checkpoint_io = checkpoint_io
        self._launcher = None
        self.num_processes = 1

    def _configure_launcher(self):
        self._launcher = None

    def setup_distributed(self):
        if not dist.is_initialized():
            dist.init_process_group(self._process_group_backend, rank=int(os.environ["RANK"]),
                                    world_size=int(os.environ["WORLD_SIZE"]))

    def _setup_model(self, model):
        return model

    def barrier(self, name=None):
        if dist.is_initialized():
            dist.barrier()

    @property
    def distributed_sampler_kwargs(self):
        return {"num_replicas": dist.get_world_size(), "rank": dist.get_rank()}


class Trainer:
    def __init__(self, strategy=None, plugins=None, max_steps=-1, accelerator="auto", devices=1, num_nodes=1,
                 enable_checkpointing=True, callbacks=None, logger=None, log_every_n_steps=50, **kw):
        self.strategy = strategy
        self.strategy.num_processes = int(devices) * int(num_nodes)
        self.precision_plugin = next((p for p in plugins or [] if isinstance(p, Precision)), Precision())
        self.max_steps, self.callbacks = max_steps, list(callbacks or [])
        self.logger = logger or None
        self.log_every_n_steps = log_every_n_steps
        self.global_step = 0
        self.callback_metrics = {}
        self.optimizers, self.lr_scheduler_configs = [], []
        self.lightning_module = None

    def fit(self, model, datamodule=None):
        self.strategy._configure_launcher()
        if self.strategy._launcher is not None:
            return self.strategy._launcher.launch(self._fit, model, datamodule, trainer=self)
        return self._fit(model, datamodule)

    def _fit(self, model, dm):
        self.strategy.setup_distributed()
        self.lightning_module = model
        model.trainer = dm.trainer = self
        model.setup("fit")
        dm.setup("fit")
        for cb in self.callbacks:
            cb.setup(self, model, "fit")
        opts, scheds = model.configure_optimizers()
        self.optimizers = [_LightningOptimizer(o) for o in opts]
        self.lr_scheduler_configs = list(scheds)
        self.strategy._setup_model(model)
        loader = dm.train_dataloader()
        model.on_train_start()
        epoch = 0
        while self.global_step < self.max_steps:
            if hasattr(loader.sampler, "set_epoch"):
                loader.sampler.set_epoch(epoch)
            for i, batch in enumerate(loader):
                model.on_train_batch_start(batch, i)
                out = model.training_step(batch, i)
                self.global_step += 1
                model.on_train_batch_end(out, batch, i)
                for cb in self.callbacks:
                    cb.on_train_batch_end(self, model, out, batch, i)
                if self.logger and self.global_step % self.log_every_n_steps == 0:
                    self.logger.log_metrics({k: float(v) for k, v in self.callback_metrics.items() if v is not None},
                                            self.global_step)
                if self.global_step >= self.max_steps:
                    break
            epoch += 1
        model.on_train_end()

    def _checkpoint(self):
        return {"state_dict": self.lightning_module.state_dict(), "global_step": self.global_step,
                "optimizer_states": [o.optimizer.state_dict() for o in self.optimizers],
                "lr_schedulers": [c["scheduler"].state_dict() for c in self.lr_scheduler_configs]}

    def save_checkpoint(self, path):
        self.strategy.save_checkpoint(self._checkpoint(), path)


def install() -> None:
    root = types.ModuleType("lightning")
    pl = types.ModuleType("lightning.pytorch")
    mods = {
        "accelerators": {"CUDAAccelerator": CUDAAccelerator},
        "callbacks": {"TQDMProgressBar": TQDMProgressBar, "ModelCheckpoint": ModelCheckpoint, "Callback": Callback},
        "loggers": {"TensorBoardLogger": TensorBoardLogger},
        "plugins": {}, "plugins.io": {"CheckpointIO": CheckpointIO}, "plugins.precision": {"Precision": Precision},
        "strategies": {"DDPStrategy": DDPStrategy}, "strategies.launchers": {},
        "strategies.launchers.launcher": {"_Launcher": _Launcher},
    }
    sys.modules["lightning"], sys.modules["lightning.pytorch"] = root, pl
    root.pytorch = pl
    for name, attrs in mods.items():
        m = types.ModuleType(f"lightning.pytorch.{name}")
        m.__dict__.update(attrs)
        sys.modules[m.__name__] = m
        parent = pl
        for part in name.split(".")[:-1]:
            parent = getattr(parent, part)
        setattr(parent, name.split(".")[-1], m)
    pl.LightningModule, pl.LightningDataModule, pl.Trainer = LightningModule, LightningDataModule, Trainer
