"""Llama-2/3/3.1 pre-training with tensor parallel (+sequence parallel) and ZeRO-1 on MI355X
(reference: examples/training/llama/tp_zero1_llama_hf_pretrain/tp_zero1_llama_hf_pretrain.py,
same command-line flags where they still mean something).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/training/llama/tp_zero1_llama_hf_pretrain.py \\
        --model_path llama3-8b --tensor_parallel_size 8 --seq_len 8192 --batch_size 1 --grad_accum_usteps 8 \\
        --max_steps 1000 --use_zero_1 --sequence_parallel_enabled --checkpoint_dir ckpt --checkpoint_freq 100

Data: `--data_dir` = a tokenized+packed HF dataset saved with save_to_disk, or a flat token file
(`*.bin`, uint32 ids; read by the native loader), or omitted for synthetic tokens.
`--model_path`: an HF config.json / directory, or a preset name (llama3-8b, llama3.1-8b, llama2-7b, ...).
`--model_family`: llama (default; also CodeGen2.5, a Llama architecture), mixtral (sparse MoE, with
`--expert_parallel_size` / `--capacity_factor`; reference examples/training/mixtral) or gpt_neox
(reference examples/training/tp_dp_gpt_neox_hf_pretrain) — same loop, optimizer and checkpointing.
"""

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))

import neuronx_distributed_llama3_2_amd as nxd  # noqa: E402
from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.training_utils import (  # noqa: E402
    Metric, SyntheticTokenDataset, Throughput, TrainingMetrics, create_llama_pretraining_dataset,
    get_learning_rate_scheduler, get_param_groups_by_weight_decay)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model_path", default="llama3-8b")
    p.add_argument("--data_dir", default=None)
    p.add_argument("--output_dir", default="output")
    p.add_argument("--metrics_file", default="results.json")
    p.add_argument("--batch_size", type=int, default=1, help="micro-batch per DP rank")
    p.add_argument("--max_steps", type=int, default=100)
    p.add_argument("--steps_this_run", type=int, default=-1)
    p.add_argument("--seed", type=int, default=12349)
    p.add_argument("--lr", type=float, default=3e-4)
    p.add_argument("--min_lr", type=float, default=3e-5)
    p.add_argument("--lr_schedule", default="cosine", choices=["cosine", "linear"])
    p.add_argument("--warmup_steps", type=int, default=10)
    p.add_argument("--grad_accum_usteps", type=int, default=1)
    p.add_argument("--print_grad_norm", action="store_true")
    p.add_argument("--tensor_parallel_size", type=int, default=1)
    p.add_argument("--seq_len", type=int, default=2048)
    p.add_argument("--use_zero_1", action="store_true")
    p.add_argument("--num_layers", type=int, default=-1)
    p.add_argument("--sequence_parallel_enabled", action="store_true")
    p.add_argument("--selective_checkpoint_enabled", action="store_true")
    p.add_argument("--activation_checkpoint", default=None, choices=[None, "full"])
    p.add_argument("--kv_replicator", type=int, default=1)
    p.add_argument("--weight_decay", type=float, default=0.01)
    p.add_argument("--beta1", type=float, default=0.9)
    p.add_argument("--beta2", type=float, default=0.95)
    p.add_argument("--max_grad_norm", type=float, default=1.0)
    p.add_argument("--checkpoint_freq", type=int, default=-1)
    p.add_argument("--checkpoint_dir", default=None)
    p.add_argument("--loading_step", default="latest_if_exists", help="-1 | latest_if_exists | <step>")
    p.add_argument("--num_kept_checkpoint", type=int, default=-1)
    p.add_argument("--async_checkpoint_saving", action="store_true")
    p.add_argument("--logging_interval", type=int, default=1)
    p.add_argument("--hidden_size", type=int, default=-1)
    p.add_argument("--model_family", default="llama", choices=["llama", "mixtral", "gpt_neox"])
    p.add_argument("--expert_parallel_size", type=int, default=1)
    p.add_argument("--capacity_factor", type=float, default=None, help="MoE: None = dropless (full capacity)")
    p.add_argument("--moe_router", default="topk", choices=["topk", "sinkhorn"])
    return p.parse_args(argv)


def model_family(a):
    """(model class, config preset function, HF config class name) of --model_family."""
    if a.model_family == "mixtral":
        from neuronx_distributed_llama3_2_amd.models.mixtral.modeling_mixtral import MixtralForCausalLM, mixtral_config

        return MixtralForCausalLM, mixtral_config, "MixtralConfig"
    if a.model_family == "gpt_neox":
        from neuronx_distributed_llama3_2_amd.models.gpt_neox.modeling_gpt_neox import (GPTNeoXForCausalLM,
                                                                                        gpt_neox_config)

        return GPTNeoXForCausalLM, gpt_neox_config, "GPTNeoXConfig"
    return LlamaForCausalLM, llama_config, "LlamaConfig"


def model_config(a):
    _, preset, hf_cls = model_family(a)
    if os.path.exists(a.model_path):
        import transformers

        path = a.model_path if a.model_path.endswith(".json") else os.path.join(a.model_path, "config.json")
        with open(path) as f:
            d = json.load(f)
        cfg = getattr(transformers, hf_cls)(**{k: v for k, v in d.items()
                                               if k not in ("architectures", "transformers_version", "model_type")})
    else:
        cfg = preset(a.model_path)
    if a.num_layers > 0:
        cfg.num_hidden_layers = a.num_layers
    if a.hidden_size > 0:
        cfg.hidden_size = a.hidden_size
    cfg.sequence_parallel_enabled = a.sequence_parallel_enabled and a.tensor_parallel_size > 1
    cfg.selective_checkpoint_enabled = a.selective_checkpoint_enabled
    cfg.kv_shared_group_size = a.kv_replicator
    cfg.max_position_embeddings = max(cfg.max_position_embeddings, a.seq_len)
    if a.model_family == "mixtral":
        cfg.capacity_factor = a.capacity_factor
        cfg.moe_router = a.moe_router
    return cfg


def batches(a, cfg, dp_rank, dp_size, dev):
    if a.data_dir and a.data_dir.endswith(".bin"):
        from neuronx_distributed_llama3_2_amd.utils.data_loader import DevicePrefetcher, TokenDataLoader

        ld = TokenDataLoader(a.data_dir, a.seq_len, a.batch_size, dp_rank, dp_size, seed=a.seed)
        return DevicePrefetcher(ld, dev), ld
    if a.data_dir:
        dl, sampler = create_llama_pretraining_dataset(a.data_dir, a.batch_size, dp_size, dp_rank, a.seed)

        def gen():
            epoch = 0
            while True:
                sampler.set_epoch(epoch)
                for b in dl:
                    yield {k: v.to(dev, non_blocking=True) for k, v in b.items()}
                epoch += 1
        return gen(), None
    ds = SyntheticTokenDataset(cfg.vocab_size, a.seq_len, seed=a.seed + dp_rank)

    def syn():
        i = 0
        while True:
            ids = torch.stack([ds[i * a.batch_size + j]["input_ids"] for j in range(a.batch_size)]).to(dev)
            yield {"input_ids": ids, "labels": ids}
            i += 1
    return syn(), None


def main(argv=None):
    a = parse(argv)
    use_cuda = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_cuda:
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    if not dist.is_initialized():
        dist.init_process_group("nccl" if use_cuda else "gloo", rank=int(os.environ.get("RANK", "0")),
                                world_size=int(os.environ.get("WORLD_SIZE", "1")))
    dev = torch.device("cuda", local_rank) if use_cuda else torch.device("cpu")
    cfg = model_config(a)
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=a.tensor_parallel_size, expert_parallel_size=a.expert_parallel_size,
        optimizer_config={"zero_one_enabled": a.use_zero_1, "grad_clipping": True, "max_grad_norm": a.max_grad_norm},
        sequence_parallel=cfg.sequence_parallel_enabled, activation_checkpoint_config=a.activation_checkpoint,
        mixed_precision_config={"use_master_weights": True, "use_fp32_grad_acc": True,
                                "use_master_weights_in_ckpt": False})
    model_parallel_manual_seed(a.seed)
    dtype = torch.bfloat16 if use_cuda else torch.float32
    model = nxd.initialize_parallel_model(nxd_config, model_family(a)[0], cfg, dtype=dtype, device=dev)
    groups = get_param_groups_by_weight_decay(model, a.weight_decay)
    optimizer = nxd.initialize_parallel_optimizer(nxd_config, torch.optim.AdamW, groups, lr=a.lr,
                                                  betas=(a.beta1, a.beta2), eps=1e-8)
    scheduler = get_learning_rate_scheduler(optimizer, a)
    dp_rank, dp_size = ps.get_data_parallel_rank(), ps.get_data_parallel_size()
    data, loader = batches(a, cfg, dp_rank, dp_size, dev)
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
    meter = Throughput(a.batch_size, dp_size, a.grad_accum_usteps, 10, a.logging_interval, a.seq_len)
    end = a.max_steps if a.steps_this_run < 0 else min(a.max_steps, step + a.steps_this_run)
    tput = []
    t_start = time.time()
    while step < end:
        model.train()
        for i in range(a.grad_accum_usteps):
            optimizer.set_grad_sync(i == a.grad_accum_usteps - 1)
            b = next(data)
            out = model(b["input_ids"], labels=b["labels"])
            (out.loss / a.grad_accum_usteps).backward()
        optimizer.step()
        optimizer.zero_grad()
        scheduler.step()
        step += 1
        if step % a.logging_interval == 0:
            loss = out.loss.detach()
            dist.all_reduce(loss, group=ps.get_data_parallel_group())
            loss = float(loss) / dp_size
            seqs = meter.get_throughput()
            tput.append(seqs)
            if rank0:
                gn = optimizer.grad_norm
                print(f"step {step} loss {loss:.4f} lr {scheduler.get_last_lr()[0]:.3e} "
                      f"{'grad_norm ' + format(float(gn), '.3f') + ' ' if (a.print_grad_norm and gn is not None) else ''}"
                      f"throughput {seqs:.2f} seq/s ({seqs * a.seq_len:.0f} tokens/s)", flush=True)
        if a.checkpoint_dir and a.checkpoint_freq > 0 and (step % a.checkpoint_freq == 0 or step == end):
            uc = {"step": step}
            if loader is not None:
                uc["data"] = loader.state_dict()
            nxd.save_checkpoint(a.checkpoint_dir, tag=f"step_{step}", model=model, optimizer=optimizer,
                                scheduler=scheduler, user_content=uc, zero1_optimizer=a.use_zero_1,
                                num_kept_ckpts=a.num_kept_checkpoint if a.num_kept_checkpoint > 0 else None,
                                async_save=a.async_checkpoint_saving)
    nxd.finalize_checkpoint()
    if rank0 and tput:
        metrics.store_metrics([
            Metric("Final loss", loss, ""),
            Metric("Average throughput", round(sum(tput) / len(tput), 3), "seq/s"),
            Metric("Peak throughput", round(max(tput), 3), "seq/s"),
            Metric("Average throughput", round(sum(tput) / len(tput) * a.seq_len, 1), "tokens/s"),
            Metric("Run time", round(time.time() - t_start, 2), "s")])
    return loss


if __name__ == "__main__":
    main()
