"""Instruction fine-tuning of a Hugging Face Llama checkpoint with TP (+SP, ZeRO-1) under PyTorch
Lightning on MI355X (reference: examples/training/llama/lightning/tp_llama_hf_finetune_ptl.py).
Same data / weights / evaluation flow as ../tp_llama_hf_finetune.py (the plain-loop version); here
Lightning drives the loop through NeuronXLAStrategy + NeuronLTModule.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tp_llama_hf_finetune_ptl.py \
        --hf_model_dir /models/Llama-3-8B --data_file dolly.jsonl --tensor_parallel_size 8 --use_zero_1
"""

from __future__ import annotations

import json
import os
import sys
from types import SimpleNamespace

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(_HERE, "..", "..", "..", "..")))
sys.path.insert(0, os.path.abspath(os.path.join(_HERE, "..")))

from tp_llama_hf_finetune import load_hf_state, parse, response_loss  # noqa: E402


def _build(a, cpu: bool):
    import transformers
    from torch.utils.data import DataLoader, DistributedSampler

    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.lightning import NeuronLTModule, NeuronXLAPrecisionPlugin, NeuronXLAStrategy
    from neuronx_distributed_llama3_2_amd.lightning._compat import pl
    from neuronx_distributed_llama3_2_amd.models.llama.convert import hf_to_nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import shard_state_dict
    from neuronx_distributed_llama3_2_amd.utils.training_utils import (build_instruction_datasets,
                                                                        get_learning_rate_scheduler)

    cfg = transformers.LlamaConfig.from_pretrained(a.hf_model_dir)
    cfg.sequence_parallel_enabled = a.sequence_parallel_enabled and a.tensor_parallel_size > 1
    tok = transformers.AutoTokenizer.from_pretrained(a.tokenizer_dir or a.hf_model_dir)
    with open(a.data_file) as f:
        records = [json.loads(line) for line in f if line.strip()]
    windows, tests = build_instruction_datasets(records, tok, a.seq_len, a.test_size, a.seed)
    pad_id = tok.eos_token_id if tok.eos_token_id is not None else 0
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=a.tensor_parallel_size, sequence_parallel=cfg.sequence_parallel_enabled,
        optimizer_config={"zero_one_enabled": a.use_zero_1, "grad_clipping": True, "max_grad_norm": 1.0},
        mixed_precision_config={"use_master_weights": True, "use_fp32_grad_acc": True,
                                "use_master_weights_in_ckpt": False})
    dtype = torch.float32 if cpu else torch.bfloat16

    class FinetuneModule(NeuronLTModule):
        """Loads this rank's TP shard of the HF weights after the model is built and scores the
        held-out answers (response-only loss) before and after training."""

        eval_before = eval_after = None

        def setup(self, stage=None):
            fresh = self.model is None
            super().setup(stage)
            if fresh:
                inner = getattr(self.model, "module", self.model)
                full = hf_to_nxd(load_hf_state(a.hf_model_dir), cfg)
                local = shard_state_dict(inner, full, ps.get_tensor_model_parallel_size(),
                                         ps.get_tensor_model_parallel_rank())
                inner.load_state_dict({k: v.to(dtype) for k, v in local.items()}, strict=False)

        def _score(self):
            inner = getattr(self.model, "module", self.model)
            dev = next(inner.parameters()).device
            return response_loss(inner, tests, dev, pad_id) if tests else float("nan")

        def on_train_start(self):
            self.eval_before = self._score()

        def on_train_end(self):
            self.eval_after = self._score()

    class Windows(pl.LightningDataModule):
        def train_dataloader(self):
            kw = self.trainer.strategy.distributed_sampler_kwargs
            ds = [{"input_ids": torch.tensor(w), "labels": torch.tensor(w)} for w in windows]
            return DataLoader(ds, batch_size=a.batch_size, drop_last=True,
                              sampler=DistributedSampler(ds, shuffle=True, seed=a.seed, drop_last=True, **kw))

    module = FinetuneModule(
        nxd_config, torch.optim.AdamW, get_learning_rate_scheduler, model_fn=LlamaForCausalLM,
        model_args=(cfg,), model_kwargs={"dtype": dtype},
        opt_kwargs={"lr": a.lr, "betas": (0.9, 0.999), "eps": 1e-8},
        scheduler_args=(SimpleNamespace(lr_schedule=a.lr_schedule, warmup_steps=a.warmup_steps,
                                        max_steps=a.max_steps, min_lr=a.min_lr),),
        train_batch_size=a.batch_size, weight_decay=a.weight_decay)
    strategy = NeuronXLAStrategy(nxd_config=nxd_config, save_load_xser=True,
                                 process_group_backend="gloo" if cpu else "nccl")
    devices = int(os.environ.get("WORLD_SIZE", "0")) or max(1, torch.cuda.device_count())
    trainer = pl.Trainer(strategy=strategy, plugins=[NeuronXLAPrecisionPlugin()], max_steps=a.max_steps,
                         accelerator="cpu" if cpu else "gpu", devices=devices,
                         enable_checkpointing=False, logger=False)
    return trainer, module, Windows()


def main(argv=None, cpu: bool = False):
    a = parse(argv)
    trainer, module, data = _build(a, cpu)
    trainer.fit(module, datamodule=data)
    if a.checkpoint_dir:
        trainer.save_checkpoint(os.path.join(a.checkpoint_dir, f"step_{a.max_steps}"))
    return module.eval_before, module.eval_after


if __name__ == "__main__":
    main()
