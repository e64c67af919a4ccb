"""Instruction fine-tuning of a Hugging Face Llama checkpoint with TP (+SP, ZeRO-1) — the MI355X
counterpart of the reference's Lightning fine-tune (examples/training/llama/lightning/
tp_llama_hf_finetune_ptl.py, data prep training_utils.py:130-207).  PyTorch Lightning is not a
dependency here: the loop is the framework's own trainer API.

Flow: HF config + weights (safetensors or pytorch_model.bin, loaded weights_only) -> NxD names
(fused qkv / gate_up) -> TP shard of this rank -> Dolly-style instruction records (JSONL with
instruction / context / response) rendered, tokenized, packed into seq_len windows -> train ->
response-only loss on held-out prompts before and after -> NxD checkpoint.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tp_llama_hf_finetune.py \
        --hf_model_dir /models/Llama-3-8B --data_file dolly.jsonl --tensor_parallel_size 8 --use_zero_1
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

import neuronx_distributed_llama3_2_amd as nxd  # noqa: E402
from neuronx_distributed_llama3_2_amd.models.llama.convert import hf_to_nxd  # noqa: E402
from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import shard_state_dict  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.training_utils import (  # noqa: E402
    Metric,
    TrainingMetrics,
    build_instruction_datasets,
    get_learning_rate_scheduler,
    get_param_groups_by_weight_decay,
)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--hf_model_dir", required=True)
    p.add_argument("--tokenizer_dir", default=None)
    p.add_argument("--data_file", required=True, help="JSONL records with instruction / context / response")
    p.add_argument("--output_dir", default="output_finetune")
    p.add_argument("--checkpoint_dir", default=None)
    p.add_argument("--tensor_parallel_size", type=int, default=1)
    p.add_argument("--use_zero_1", action="store_true")
    p.add_argument("--sequence_parallel_enabled", action="store_true")
    p.add_argument("--seq_len", type=int, default=2048)
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--max_steps", type=int, default=100)
    p.add_argument("--warmup_steps", type=int, default=5)
    p.add_argument("--lr", type=float, default=5e-6)
    p.add_argument("--min_lr", type=float, default=0.0)
    p.add_argument("--lr_schedule", default="linear", choices=["cosine", "linear"])
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--test_size", type=int, default=8)
    p.add_argument("--seed", type=int, default=42)
    return p.parse_args(argv)


def load_hf_state(d):
    files = sorted(glob.glob(os.path.join(d, "*.safetensors")))
    sd = {}
    if files:
        from safetensors.torch import load_file

        for f in files:
            sd.update(load_file(f))
    else:
        for f in sorted(glob.glob(os.path.join(d, "pytorch_model*.bin"))):
            sd.update(torch.load(f, map_location="cpu", weights_only=True))
    return sd


@torch.no_grad()
def response_loss(model, tests, dev, pad_id=0, multiple=8):
    """Mean NLL of the reference answers given the prompts (prompt and padding positions labelled
    -100, so the vocab-parallel cross entropy only scores the answer tokens).  Sequences are
    right-padded to a multiple of 8 (sequence parallelism splits the sequence over TP ranks)."""
    model.eval()
    tot, n = 0.0, 0
    for t in tests:
        seq = t["input_ids"] + t["labels"]
        pad = (-len(seq)) % multiple
        ids = torch.tensor([seq + [pad_id] * pad], device=dev)
        labels = torch.tensor([[-100] * len(t["input_ids"]) + t["labels"] + [-100] * pad], device=dev)
        out = model(ids, labels=labels)
        k = len(t["labels"])
        tot += float(out.loss) * k
        n += k
    model.train()
    return tot / max(1, n)


def main(argv=None):
    a = parse(argv)
    use_cuda = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_cuda:
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29537")
    if not dist.is_initialized():
        dist.init_process_group("nccl" if use_cuda else "gloo", rank=int(os.environ.get("RANK", "0")),
                                world_size=int(os.environ.get("WORLD_SIZE", "1")))
    dev = torch.device("cuda", local_rank) if use_cuda else torch.device("cpu")
    import transformers

    cfg = transformers.LlamaConfig.from_pretrained(a.hf_model_dir)
    cfg.sequence_parallel_enabled = a.sequence_parallel_enabled and a.tensor_parallel_size > 1
    tok = transformers.AutoTokenizer.from_pretrained(a.tokenizer_dir or a.hf_model_dir)
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=a.tensor_parallel_size, sequence_parallel=cfg.sequence_parallel_enabled,
        optimizer_config={"zero_one_enabled": a.use_zero_1, "grad_clipping": True, "max_grad_norm": 1.0},
        mixed_precision_config={"use_master_weights": True, "use_fp32_grad_acc": True,
                                "use_master_weights_in_ckpt": False})
    model_parallel_manual_seed(a.seed)
    dtype = torch.bfloat16 if use_cuda else torch.float32
    model = nxd.initialize_parallel_model(nxd_config, LlamaForCausalLM, cfg, dtype=dtype, device=dev)
    inner = getattr(model, "module", model)
    full = hf_to_nxd(load_hf_state(a.hf_model_dir), cfg)
    local = shard_state_dict(inner, full, ps.get_tensor_model_parallel_size(), ps.get_tensor_model_parallel_rank())
    inner.load_state_dict({k: v.to(dtype) for k, v in local.items()}, strict=False)
    del full, local
    optimizer = nxd.initialize_parallel_optimizer(nxd_config, torch.optim.AdamW,
                                                  get_param_groups_by_weight_decay(model, a.weight_decay),
                                                  lr=a.lr, betas=(0.9, 0.999), eps=1e-8)
    scheduler = get_learning_rate_scheduler(optimizer, a)
    with open(a.data_file) as f:
        records = [json.loads(line) for line in f if line.strip()]
    windows, tests = build_instruction_datasets(records, tok, a.seq_len, a.test_size, a.seed)
    dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
    per_step = a.batch_size * dp
    assert len(windows) >= per_step, f"only {len(windows)} packed windows for a global batch of {per_step}"
    rank0 = dist.get_rank() == 0
    pad_id = tok.eos_token_id if tok.eos_token_id is not None else 0
    before = response_loss(inner, tests, dev, pad_id) if tests else float("nan")
    g = torch.Generator().manual_seed(a.seed)
    order, pos, loss = torch.randperm(len(windows), generator=g).tolist(), 0, float("nan")
    for step in range(a.max_steps):
        if pos + per_step > len(order):
            order, pos = torch.randperm(len(windows), generator=g).tolist(), 0
        mine = order[pos + dpr * a.batch_size: pos + (dpr + 1) * a.batch_size]
        pos += per_step
        ids = torch.tensor([windows[i] for i in mine], device=dev)
        out = model(ids, labels=ids)
        out.loss.backward()
        optimizer.step()
        optimizer.zero_grad()
        scheduler.step()
        lt = out.loss.detach().float().reshape(1)
        dist.all_reduce(lt, group=ps.get_data_parallel_group())
        loss = float(lt) / dp
        if rank0:
            print(f"step {step + 1} loss {loss:.4f} lr {scheduler.get_last_lr()[0]:.2e}", flush=True)
    after = response_loss(inner, tests, dev, pad_id) if tests else float("nan")
    if a.checkpoint_dir:
        nxd.save_checkpoint(a.checkpoint_dir, tag=f"step_{a.max_steps}", model=model, optimizer=optimizer,
                            user_content={"step": a.max_steps}, zero1_optimizer=a.use_zero_1)
        nxd.finalize_checkpoint()
    if rank0:
        os.makedirs(a.output_dir, exist_ok=True)
        m = TrainingMetrics(os.path.join(a.output_dir, "results.json"))
        m.store_parameters(vars(a))
        m.store_metrics([Metric("Final loss", loss, ""), Metric("Eval response loss before", before, ""),
                         Metric("Eval response loss after", after, "")])
        print(f"response loss before {before:.4f} after {after:.4f}", flush=True)
    return before, after


if __name__ == "__main__":
    main()
