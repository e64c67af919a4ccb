"""Llama pre-training (TP [+PP, ZeRO-1]) with PyTorch Lightning on MI355X (reference:
examples/training/llama/lightning/run_llama_nxd_ptl.py).  One process per GPU: launch under
torchrun, or let the strategy's launcher spawn the ranks.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 run_llama_nxd_ptl.py \
        --model llama3-8b --tensor_parallel_size 8 --use_zero1_optimizer 1 --seq_len 8192 \
        --train_batch_size 1 --max_steps 100 --data_path /data/llama3_packed_8k
"""

from __future__ import annotations

import argparse
import os
import sys
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..", "..")))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def build_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama3-8b", help="llama_config preset (random init) or an HF config dir")
    p.add_argument("--data_path", default=None, help="save_to_disk dataset / .npy token windows; none: synthetic")
    p.add_argument("--train_batch_size", type=int, default=1, help="sequences per DP rank per step")
    p.add_argument("--grad_accum_usteps", type=int, default=1)
    p.add_argument("--max_steps", type=int, default=100)
    p.add_argument("--warmup_steps", type=int, default=10)
    p.add_argument("--lr", type=float, default=3e-4)
    p.add_argument("--min_lr", type=float, default=3e-5)
    p.add_argument("--weight_decay", type=float, default=0.01)
    p.add_argument("--beta1", type=float, default=0.9)
    p.add_argument("--beta2", type=float, default=0.95)
    p.add_argument("--seq_len", type=int, default=4096)
    p.add_argument("--tensor_parallel_size", type=int, default=8)
    p.add_argument("--pipeline_parallel_size", type=int, default=1)
    p.add_argument("--num_microbatches", type=int, default=8)
    p.add_argument("--use_zero1_optimizer", type=int, default=1)
    p.add_argument("--use_fp32_optimizer", type=int, default=1, help="fp32 master weights in the optimizer")
    p.add_argument("--use_sequence_parallel", type=int, default=1)
    p.add_argument("--activation_checkpoint", default=None, choices=[None, "full", "selective"])
    p.add_argument("--num_layers", type=int, default=None)
    p.add_argument("--checkpoint_dir", default=None)
    p.add_argument("--checkpoint_freq", type=int, default=0)
    p.add_argument("--save_load_xser", type=int, default=1)
    p.add_argument("--tb_dir", default="")
    p.add_argument("--logging_interval", type=int, default=1)
    p.add_argument("--log_rank0", type=int, default=0)
    p.add_argument("--num_nodes", type=int, default=1)
    p.add_argument("--devices", type=int, default=None, help="GPUs per node (default: WORLD_SIZE or all visible)")
    p.add_argument("--cpu", action="store_true", help="gloo / CPU ranks (plumbing tests)")
    p.add_argument("--seed", type=int, default=1234)
    return p.parse_args(argv)


def _model_config(a):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import llama_config

    over = dict(sequence_parallel_enabled=bool(a.use_sequence_parallel) and a.tensor_parallel_size > 1,
                max_position_embeddings=max(a.seq_len, 128))
    if a.num_layers:
        over["num_hidden_layers"] = a.num_layers
    if a.activation_checkpoint == "selective":
        over["selective_checkpoint_enabled"] = True
    if os.path.isdir(a.model):
        from transformers import LlamaConfig

        cfg = LlamaConfig.from_pretrained(a.model)
        for k, v in over.items():
            setattr(cfg, k, v)
        return cfg
    return llama_config(a.model, **over)


def train_llama(a):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.lightning import (NeuronTensorBoardLogger, NeuronTQDMProgressBar,
                                                             NeuronXLAPrecisionPlugin, NeuronXLAStrategy)
    from neuronx_distributed_llama3_2_amd.lightning._compat import pl
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaDecoderLayer, LlamaForCausalLM
    from neuronx_distributed_llama3_2_amd.utils.training_utils import get_learning_rate_scheduler

    from data_module import NeuronLlamaDataModule
    from module_llama import NeuronLlamaLTModule

    cfg = _model_config(a)
    pipeline_config = None
    if a.pipeline_parallel_size > 1:
        pipeline_config = {"transformer_layer_cls": LlamaDecoderLayer, "num_microbatches": a.num_microbatches,
                           "input_names": ["input_ids", "labels"], "auto_partition": True,
                           "output_loss_value_spec": (True, False)}
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=a.tensor_parallel_size, pipeline_parallel_size=a.pipeline_parallel_size,
        pipeline_config=pipeline_config, sequence_parallel=cfg.sequence_parallel_enabled,
        optimizer_config={"zero_one_enabled": bool(a.use_zero1_optimizer), "grad_clipping": True, "max_grad_norm": 1.0},
        activation_checkpoint_config="full" if a.activation_checkpoint == "full" else None,
        mixed_precision_config={"use_master_weights": bool(a.use_fp32_optimizer),
                                "use_fp32_grad_acc": bool(a.use_fp32_optimizer),
                                "use_master_weights_in_ckpt": False})
    dtype = torch.float32 if a.cpu else torch.bfloat16
    module = NeuronLlamaLTModule(
        nxd_config, torch.optim.AdamW, get_learning_rate_scheduler, model_fn=LlamaForCausalLM,
        model_args=(cfg,), model_kwargs={"dtype": dtype},
        opt_kwargs={"lr": a.lr, "betas": (a.beta1, a.beta2), "weight_decay": a.weight_decay},
        scheduler_args=(SimpleNamespace(lr_schedule="cosine", warmup_steps=a.warmup_steps, max_steps=a.max_steps,
                                        min_lr=a.min_lr),),
        grad_accum_steps=a.grad_accum_usteps, train_batch_size=a.train_batch_size,
        logging_interval=a.logging_interval, log_rank0=bool(a.log_rank0), seq_len=a.seq_len)
    data = NeuronLlamaDataModule(a.data_path, a.seq_len, cfg.vocab_size, a.train_batch_size * a.grad_accum_usteps,
                                 seed=a.seed)
    strategy = NeuronXLAStrategy(nxd_config=nxd_config, save_load_xser=bool(a.save_load_xser),
                                 process_group_backend="gloo" if a.cpu else "nccl")
    callbacks = [NeuronTQDMProgressBar()]
    if a.checkpoint_dir and a.checkpoint_freq:
        callbacks.append(pl.callbacks.ModelCheckpoint(dirpath=a.checkpoint_dir, every_n_train_steps=a.checkpoint_freq,
                                                      save_top_k=-1))
    devices = a.devices or int(os.environ.get("WORLD_SIZE", "0")) or max(1, torch.cuda.device_count())
    trainer = pl.Trainer(strategy=strategy, plugins=[NeuronXLAPrecisionPlugin()], max_steps=a.max_steps,
                         accelerator="cpu" if a.cpu else "gpu", devices=devices, num_nodes=a.num_nodes,
                         enable_checkpointing=bool(a.checkpoint_dir), callbacks=callbacks,
                         logger=NeuronTensorBoardLogger(save_dir=a.tb_dir or "tb", log_rank0=bool(a.log_rank0)),
                         log_every_n_steps=a.logging_interval)
    trainer.fit(module, datamodule=data)
    return module.history


if __name__ == "__main__":
    train_llama(build_args())
