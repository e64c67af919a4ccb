"""BERT-large pre-training (MLM + NSP) with tensor + data parallelism — the MI355X counterpart of
the reference's tp_dp_bert_hf_pretrain (examples/training/tp_dp_bert_hf_pretrain/
tp_dp_bert_large_hf_pretrain_hdf5.py:402-521): raw `parallel_state` + parallel layers, the DP
gradient all-reduce done explicitly with `bucket_allreduce_gradients` (the reference calls
`xm.reduce_gradients`), `clip_grad_norm`, plain torch AdamW, linear warmup/decay, optional
gradient accumulation.  Data: synthetic masked-LM batches (15 % masking, 80/10/10 replacement,
random sentence-order labels) of the phase-1 shape.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tp_dp_bert_hf_pretrain.py --tensor_parallel_size 2
"""

from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from neuronx_distributed_llama3_2_amd.models.bert.modeling_bert import BertForPreTraining, bert_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.grads import (  # noqa: E402
    bucket_allreduce_gradients,
    clip_grad_norm,
)
from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.training_utils import Metric, Throughput, TrainingMetrics  # noqa: E402


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="bert-large-uncased")
    p.add_argument("--tensor_parallel_size", type=int, default=1)
    p.add_argument("--batch_size", type=int, default=16, help="micro-batch per DP rank")
    p.add_argument("--grad_accum_usteps", type=int, default=1)
    p.add_argument("--seq_len", type=int, default=128)
    p.add_argument("--max_steps", type=int, default=100)
    p.add_argument("--warmup_steps", type=int, default=10)
    p.add_argument("--lr", type=float, default=4e-4)
    p.add_argument("--max_grad_norm", type=float, default=1.0)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--output_dir", default="output_bert")
    p.add_argument("--num_layers", type=int, default=-1)
    return p.parse_args(argv)


def mlm_batch(g, bs, seq, vocab, dev, mask_id=103):
    lo = min(1000, vocab // 2)   # skip the special / unused ids of the BERT vocab
    ids = torch.randint(lo, vocab, (bs, seq), generator=g)
    labels = torch.full_like(ids, -100)
    sel = torch.rand(bs, seq, generator=g) < 0.15
    labels[sel] = ids[sel]
    r = torch.rand(bs, seq, generator=g)
    ids[sel & (r < 0.8)] = mask_id
    rnd = sel & (r >= 0.8) & (r < 0.9)
    ids[rnd] = torch.randint(lo, vocab, (int(rnd.sum()),), generator=g)
    tt = torch.zeros_like(ids)
    tt[:, seq // 2:] = 1
    nsp = torch.randint(0, 2, (bs,), generator=g)
    return {k: v.to(dev) for k, v in dict(input_ids=ids, token_type_ids=tt, labels=labels,
                                          next_sentence_label=nsp, attention_mask=torch.ones_like(ids)).items()}


def main(argv=None):
    a = parse(argv)
    use_cuda = torch.cuda.is_available()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_cuda:
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29535")
    if not dist.is_initialized():
        dist.init_process_group("nccl" if use_cuda else "gloo", rank=int(os.environ.get("RANK", "0")),
                                world_size=int(os.environ.get("WORLD_SIZE", "1")))
    ps.initialize_model_parallel(tensor_model_parallel_size=a.tensor_parallel_size)
    dev = torch.device("cuda", local_rank) if use_cuda else torch.device("cpu")
    over = {"num_hidden_layers": a.num_layers} if a.num_layers > 0 else {}
    cfg = bert_config(a.model, **over)
    model_parallel_manual_seed(a.seed)
    model = BertForPreTraining(cfg, dtype=torch.bfloat16 if use_cuda else torch.float32, device=dev)
    params = [p for p in model.parameters() if p.requires_grad]
    decay = [p for n, p in model.named_parameters() if p.dim() > 1]
    no_decay = [p for n, p in model.named_parameters() if p.dim() <= 1]
    opt = torch.optim.AdamW([{"params": decay, "weight_decay": 0.01}, {"params": no_decay, "weight_decay": 0.0}],
                            lr=a.lr, betas=(0.9, 0.999), eps=1e-6)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda s: min((s + 1) / max(1, a.warmup_steps), max(0.0, (a.max_steps - s) / max(1, a.max_steps - a.warmup_steps))))
    dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
    g = torch.Generator().manual_seed(a.seed + dpr)   # TP ranks of one DP replica see the same batch
    rank0 = dist.get_rank() == 0
    meter = Throughput(a.batch_size, dp, a.grad_accum_usteps, 10, 1, a.seq_len)
    metrics = TrainingMetrics(os.path.join(a.output_dir, "results.json")) if rank0 else None
    if rank0:
        os.makedirs(a.output_dir, exist_ok=True)
        metrics.store_parameters(vars(a))
    tput, loss_v, t0 = [], float("nan"), time.time()
    for step in range(a.max_steps):
        tot = 0.0
        for _ in range(a.grad_accum_usteps):
            out = model(**mlm_batch(g, a.batch_size, a.seq_len, cfg.vocab_size, dev))
            (out.loss / a.grad_accum_usteps).backward()
            tot += float(out.loss.detach()) / a.grad_accum_usteps
        grads = [p.grad for p in params if p.grad is not None]
        bucket_allreduce_gradients(grads)            # DP sum (the reference's xm.reduce_gradients)
        if dp > 1:
            torch._foreach_div_(grads, float(dp))
        gnorm = clip_grad_norm(params, a.max_grad_norm)
        opt.step()
        opt.zero_grad(set_to_none=True)
        sched.step()
        lt = torch.tensor([tot], device=dev)
        dist.all_reduce(lt, group=ps.get_data_parallel_group())
        loss_v = float(lt) / dp
        seqs = meter.get_throughput()
        tput.append(seqs)
        if rank0:
            print(f"step {step + 1} loss {loss_v:.4f} grad_norm {float(gnorm):.3f} throughput {seqs:.1f} seq/s",
                  flush=True)
    if rank0:
        metrics.store_metrics([Metric("Final loss", loss_v, ""),
                               Metric("Average throughput", round(sum(tput) / len(tput), 3), "seq/s"),
                               Metric("Run time", round(time.time() - t0, 2), "s")])
    return loss_v


if __name__ == "__main__":
    main()
