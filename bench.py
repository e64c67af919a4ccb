"""Headline benchmark: Llama-3-8B bf16 pre-training throughput (tokens/s, whole job) on N MI355X.

Config (BASELINE.json): Llama-3-8B architecture (random init, synthetic token data), sequence
length 8192, micro-batch 1, tensor parallel TP = N (<= 8) with sequence parallelism, flash
attention, fp32 master weights + fused AdamW (ZeRO-1 when DP > 1), gradient accumulation up to the
global batch.  `--parallelism dp` instead runs TP=1 x DP=N (weak scaling).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Times exactly K optimizer steps between barrier + device synchronisation on both sides, takes
the max over ranks, rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.profiling import llama_num_params, mfu, model_flops_per_token  # noqa: E402

BASELINE_TOKENS_PER_S = None  # the reference publishes no Llama-3-8B throughput


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1, help="micro-batch size (sequences)")
    ap.add_argument("--gbs", type=int, default=8, help="global batch (sequences per optimizer step)")
    ap.add_argument("--parallelism", choices=["tp", "dp"], default="tp")
    ap.add_argument("--layers", type=int, default=None, help="override #layers (NOT the headline config)")
    ap.add_argument("--no-sp", action="store_true")
    ap.add_argument("--ckpt", default=None, help="activation checkpointing: None | full | selective")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == a.gpus, f"--gpus {a.gpus} but WORLD_SIZE={world}"
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    dist.init_process_group("nccl" if use_cuda else "gloo", rank=rank, world_size=world,
                            device_id=torch.device("cuda", local_rank) if use_cuda else None)
    tp = min(world, 8) if a.parallelism == "tp" else 1
    ps.initialize_model_parallel(tensor_model_parallel_size=tp)
    dp = ps.get_data_parallel_size()
    model_parallel_manual_seed(1234)
    dev = torch.device("cuda", local_rank) if use_cuda else torch.device("cpu")

    over = dict(sequence_parallel_enabled=(tp > 1 and not a.no_sp), max_position_embeddings=max(8192, a.seq))
    if a.layers is not None:
        over["num_hidden_layers"] = a.layers
    if a.ckpt == "full":
        over["activation_checkpoint"] = "full"
    elif a.ckpt == "selective":
        over["selective_checkpoint_enabled"] = True
    cfg = llama_config(a.model, **over)
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=dev)
    model.train()
    nparams_local = sum(p.numel() for p in model.parameters())
    decay = [p for n, p in model.named_parameters() if p.dim() > 1]
    no_decay = [p for n, p in model.named_parameters() if p.dim() <= 1]
    opt = FlatMixedPrecisionAdamW([{"params": decay, "weight_decay": 0.01}, {"params": no_decay, "weight_decay": 0.0}],
                                  lr=1e-5, betas=(0.9, 0.95), eps=1e-8, zero1=dp > 1, grad_clipping=True,
                                  max_grad_norm=1.0, shared_param_ids=find_shared_params(model))
    assert a.gbs % (a.mbs * dp) == 0, "global batch must be divisible by micro-batch x DP"
    accum = a.gbs // (a.mbs * dp)
    g = torch.Generator(device="cpu").manual_seed(4321 + ps.get_data_parallel_rank())
    batches = [torch.randint(0, cfg.vocab_size, (a.mbs, a.seq), generator=g).to(dev) for _ in range(min(accum, 4))]

    def train_step():
        for i in range(accum):
            opt.set_grad_sync(i == accum - 1)
            ids = batches[i % len(batches)]
            out = model(ids, labels=ids)
            (out.loss / accum).backward()
        opt.step()
        opt.zero_grad()
        return out.loss

    for _ in range(a.warmup):
        loss = train_step()
    if use_cuda:
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = train_step()
    if use_cuda:
        torch.cuda.synchronize()
    dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    el = float(elapsed.item())
    tokens = a.gbs * a.seq * a.steps
    value = tokens / el
    if rank == 0:
        mem = torch.cuda.max_memory_allocated(dev) / 2**30 if use_cuda else 0.0
        nparams = llama_num_params(cfg)
        fpt = model_flops_per_token(nparams, cfg.num_hidden_layers, cfg.hidden_size, a.seq)
        par = f"tp{tp}" + ("_sp" if over["sequence_parallel_enabled"] else "") + (f"_dp{dp}_zero1" if dp > 1 else "")
        rec = {
            "metric": "tokens/sec (whole node) Llama-3-8B TP=8 bf16 training at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * el / a.steps, 2),
            "higher_is_better": True,
            "scaling": "strong" if a.parallelism == "tp" else "weak",
            "vs_baseline": (value / BASELINE_TOKENS_PER_S) if BASELINE_TOKENS_PER_S else None,
            "dtype": "bf16",
            "data": "synthetic (random token ids, random-init weights)",
            "config": {"model": a.model if a.layers is None else f"{a.model}-{a.layers}L", "global_batch": a.gbs,
                       "micro_batch": a.mbs, "seq_len": a.seq, "parallelism": par, "grad_accum": accum,
                       "optimizer": "AdamW fp32-master" + (" ZeRO-1" if dp > 1 else ""),
                       "activation_checkpoint": a.ckpt or "none"},
            "loss": round(float(loss.item()), 4),
            "params_per_rank": nparams_local,
            "model_params": nparams,
            "mfu": round(mfu(value, fpt, world), 4),   # vs 2.5 PFLOP/s dense bf16 per GPU
            "peak_mem_gib": round(mem, 1),
        }
        print(json.dumps(rec), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
