"""Llama-2/3 pre-training with tensor + pipeline parallelism (NxDPPModel 1F1B / interleaved) and
ZeRO-1 — the MI355X counterpart of the reference's tp_pp_llama_hf_pretrain/run_llama_nxd.py
(examples/training/llama/tp_pp_llama_hf_pretrain/run_llama_nxd.py:1-479; launchers
run_llama{2_13B,2_70B,3_70B}_tp_pp.sh).

One process per GPU over RCCL.  The pipeline runtime sends activations between stages with
`batch_isend_irecv` on xGMI; micro-batches flow through a 1F1B (or interleaved, with
--virtual_pipeline_size > 1) schedule and the optimizer steps once per global batch.  Resume
semantics follow the reference (latest checkpoint with a `done` marker, step + data position in
user content); `--watchdog_timeout` arms the host step watchdog (utils/resilience.py).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tp_pp_llama_hf_pretrain.py \
        --model_path llama3-70b --tensor_parallel_size 4 --pipeline_parallel_size 2 --num_microbatches 8 ...
"""

from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

import neuronx_distributed_llama3_2_amd as nxd  # noqa: E402
from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaDecoderLayer  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.resilience import StepWatchdog, configure_collective_watchdog  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.training_utils import (  # noqa: E402
    Metric,
    Throughput,
    TrainingMetrics,
    create_partition,
    get_learning_rate_scheduler,
    get_param_groups_by_weight_decay,
)

import tp_zero1_llama_hf_pretrain as base  # noqa: E402  (config / data helpers shared with the TP example)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model_path", default="llama3-8b")
    p.add_argument("--data_dir", default=None)
    p.add_argument("--output_dir", default="output")
    p.add_argument("--metrics_file", default="results.json")
    p.add_argument("--train_batch_size", type=int, default=8, help="global batch per DP rank (sequences)")
    p.add_argument("--num_microbatches", type=int, default=4)
    p.add_argument("--max_steps", type=int, default=100)
    p.add_argument("--steps_this_run", type=int, default=-1)
    p.add_argument("--seed", type=int, default=12349)
    p.add_argument("--lr", type=float, default=1.5e-4)
    p.add_argument("--min_lr", type=float, default=1e-5)
    p.add_argument("--lr_schedule", default="cosine", choices=["cosine", "linear"])
    p.add_argument("--warmup_steps", type=int, default=10)
    p.add_argument("--tensor_parallel_size", type=int, default=1)
    p.add_argument("--pipeline_parallel_size", type=int, default=2)
    p.add_argument("--virtual_pipeline_size", type=int, default=1)
    p.add_argument("--seq_len", type=int, default=4096)
    p.add_argument("--use_zero_1", action="store_true")
    p.add_argument("--num_layers", type=int, default=-1)
    p.add_argument("--hidden_size", type=int, default=-1)
    p.add_argument("--sequence_parallel_enabled", action="store_true")
    p.add_argument("--selective_checkpoint_enabled", action="store_true")
    p.add_argument("--activation_checkpoint", default=None, choices=[None, "full"])
    p.add_argument("--kv_replicator", type=int, default=1)
    p.add_argument("--auto_partition", action="store_true", help="even layer split instead of --pipeline_cuts")
    p.add_argument("--pipeline_cuts", default=None, help="comma-separated layer names ending each stage")
    p.add_argument("--weight_decay", type=float, default=0.1)
    p.add_argument("--beta1", type=float, default=0.9)
    p.add_argument("--beta2", type=float, default=0.95)
    p.add_argument("--max_grad_norm", type=float, default=1.0)
    p.add_argument("--checkpoint_freq", type=int, default=-1)
    p.add_argument("--checkpoint_dir", default=None)
    p.add_argument("--loading_step", default="latest_if_exists")
    p.add_argument("--num_kept_checkpoint", type=int, default=-1)
    p.add_argument("--async_checkpoint_saving", action="store_true")
    p.add_argument("--watchdog_timeout", type=float, default=0.0, help="seconds; 0 disables the step watchdog")
    p.add_argument("--logging_interval", type=int, default=1)
    a = p.parse_args(argv)
    # fields the shared helpers of the TP example read
    a.model_family, a.expert_parallel_size, a.capacity_factor, a.moe_router = "llama", 1, None, "topk"
    a.batch_size = a.train_batch_size
    return a


def main(argv=None):
    a = parse(argv)
    use_cuda = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_cuda:
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if not dist.is_initialized():
        timeout = configure_collective_watchdog()
        dist.init_process_group("nccl" if use_cuda else "gloo", rank=int(os.environ.get("RANK", "0")),
                                world_size=int(os.environ.get("WORLD_SIZE", "1")), timeout=timeout)
    dev = torch.device("cuda", local_rank) if use_cuda else torch.device("cpu")
    cfg = base.model_config(a)
    cuts = a.pipeline_cuts.split(",") if a.pipeline_cuts else None
    if cuts is None and not a.auto_partition and a.pipeline_parallel_size > 1:
        cuts = create_partition(cfg.num_hidden_layers, a.pipeline_parallel_size * a.virtual_pipeline_size)
    pcfg = {"transformer_layer_cls": LlamaDecoderLayer, "num_microbatches": a.num_microbatches,
            "virtual_pipeline_size": a.virtual_pipeline_size, "input_names": ["input_ids", "labels"],
            "broadcast_and_average_loss": True,
            "auto_partition": cuts is None, "pipeline_cuts": cuts}
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=a.tensor_parallel_size, pipeline_parallel_size=a.pipeline_parallel_size,
        pipeline_config=pcfg, sequence_parallel=cfg.sequence_parallel_enabled,
        optimizer_config={"zero_one_enabled": a.use_zero_1, "grad_clipping": True, "max_grad_norm": a.max_grad_norm},
        activation_checkpoint_config=a.activation_checkpoint,
        mixed_precision_config={"use_master_weights": True, "use_fp32_grad_acc": True,
                                "use_master_weights_in_ckpt": False})
    model_parallel_manual_seed(a.seed)
    dtype = torch.bfloat16 if use_cuda else torch.float32
    model = nxd.initialize_parallel_model(nxd_config, base.LlamaForCausalLM, cfg, dtype=dtype, device=dev)
    groups = get_param_groups_by_weight_decay(model, a.weight_decay)
    optimizer = nxd.initialize_parallel_optimizer(nxd_config, torch.optim.AdamW, groups, lr=a.lr,
                                                  betas=(a.beta1, a.beta2), eps=1e-8)
    scheduler = get_learning_rate_scheduler(optimizer, a)
    dp_rank, dp_size = ps.get_data_parallel_rank(), ps.get_data_parallel_size()
    data, loader = base.batches(a, cfg, dp_rank, dp_size, dev)
    step = 0
    if a.checkpoint_dir and a.loading_step != "-1" and nxd.has_checkpoint(a.checkpoint_dir):
        tag = None if a.loading_step == "latest_if_exists" else a.loading_step
        uc = nxd.load_checkpoint(a.checkpoint_dir, tag=tag, model=model, optimizer=optimizer, scheduler=scheduler)
        if uc:
            step = int(uc.get("step", 0))
            if loader is not None and "data" in uc:
                loader.load_state_dict(uc["data"])
    rank0 = dist.get_rank() == 0
    metrics = TrainingMetrics(os.path.join(a.output_dir, a.metrics_file)) if rank0 else None
    if rank0:
        os.makedirs(a.output_dir, exist_ok=True)
        metrics.store_parameters({k: v for k, v in vars(a).items()})
    meter = Throughput(a.train_batch_size, dp_size, 1, 10, a.logging_interval, a.seq_len)
    end = a.max_steps if a.steps_this_run < 0 else min(a.max_steps, step + a.steps_this_run)
    wd = StepWatchdog(a.watchdog_timeout) if a.watchdog_timeout > 0 else None
    tput, loss = [], float("nan")
    t_start = time.time()
    while step < end:
        b = next(data)
        loss_t = model.run_train(input_ids=b["input_ids"], labels=b["labels"])
        optimizer.step()
        optimizer.zero_grad()
        scheduler.step()
        step += 1
        if wd is not None:
            wd.kick()
        if step % a.logging_interval == 0:
            loss = float(loss_t)   # broadcast from the last stage and averaged over DP by the runtime
            seqs = meter.get_throughput()
            tput.append(seqs)
            if rank0:
                print(f"step {step} loss {loss:.4f} lr {scheduler.get_last_lr()[0]:.3e} "
                      f"throughput {seqs:.2f} seq/s ({seqs * a.seq_len:.0f} tokens/s)", flush=True)
        if a.checkpoint_dir and a.checkpoint_freq > 0 and (step % a.checkpoint_freq == 0 or step == end):
            uc = {"step": step}
            if loader is not None:
                uc["data"] = loader.state_dict()
            nxd.save_checkpoint(a.checkpoint_dir, tag=f"step_{step}", model=model, optimizer=optimizer,
                                scheduler=scheduler, user_content=uc, zero1_optimizer=a.use_zero_1,
                                num_kept_ckpts=a.num_kept_checkpoint if a.num_kept_checkpoint > 0 else None,
                                async_save=a.async_checkpoint_saving)
    if wd is not None:
        wd.stop()
    nxd.finalize_checkpoint()
    if rank0 and tput:
        metrics.store_metrics([
            Metric("Final loss", loss, ""),
            Metric("Average throughput", round(sum(tput) / len(tput), 3), "seq/s"),
            Metric("Peak throughput", round(max(tput), 3), "seq/s"),
            Metric("Run time", round(time.time() - t_start, 2), "s")])
    return loss


if __name__ == "__main__":
    main()
