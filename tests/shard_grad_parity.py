"""Per-shard gradient parity of the TP / SP layers (helpers shared by the CPU and GPU tests).

Every rank saves its fp32 `main_grad` of every parameter after two accumulated micro-batches
(before the optimizer step); each shard is compared with the same slice of the TP=1 gradient,
sliced by the checkpoint converter's partition rules (parallel_layers/sharding.py
`shard_tensor`: fused QKV with replicated KV heads and the q-group order, gate_up stride 2,
o_proj regrouped, vocab-parallel embedding / lm_head).  Norm weights under sequence parallelism hold
per-rank partial sums until the optimizer's TP all-reduce, so their shards are summed over ranks.
Reference: test/integration/parallel_layers/test_layers.py:79-82,316-321,410-415 (each parallel
layer's weight-gradient chunk against the unsharded layer's)."""

import os
import tempfile

import torch

from dist_utils import run_distributed

MICRO = 2


def _w_grads(rank, world, preset, sp, streams, dev_kind, out):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.parallel_layers import stream_split

    if dev_kind == "cuda":
        torch.cuda.set_device(0)
    dev = torch.device(dev_kind)
    dtype = torch.bfloat16 if dev_kind == "cuda" else torch.float32
    stream_split.set_enabled(streams >= 2, streams)
    ps.initialize_model_parallel(world)
    seq = 512 if dev_kind == "cuda" else 128
    cfg = llama_config(preset, sequence_parallel_enabled=sp, max_position_embeddings=seq)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=dtype, device=dev)
    model.train()
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=1e-3, grad_clipping=True, max_grad_norm=1.0,
                                  shared_param_ids=find_shared_params(model))
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (MICRO, 2, seq), device=dev)
    for i in range(MICRO):
        opt.set_grad_sync(i == MICRO - 1)
        (model(ids[i], labels=ids[i]).loss / MICRO).backward()
    stream_split.join()
    if dev_kind == "cuda":
        torch.cuda.synchronize()
    grads = {n: p.main_grad.detach().float().cpu().clone() for n, p in model.named_parameters()}
    torch.save({"grads": grads, "kv_mult": model.model.layers[0].self_attn.kv_mult,
                "cfg": cfg.to_dict()}, f"{out}.{rank}")


def collect(world, preset, sp, streams=1, dev_kind="cpu"):
    d = tempfile.mkdtemp()
    out = os.path.join(d, "g")
    run_distributed(_w_grads, world, preset, sp, streams, dev_kind, out)
    return [torch.load(f"{out}.{r}", weights_only=False) for r in range(world)]


def compare(ref, shards, sp: bool):
    """{param name: relative max error} of every TP shard against the TP=1 gradient slice."""
    from neuronx_distributed_llama3_2_amd.parallel_layers.sharding import shard_tensor
    from neuronx_distributed_llama3_2_amd.scripts.checkpoint_converter import CheckpointConverterBase, _Cfg

    conv = CheckpointConverterBase()
    cfg = _Cfg(shards[0]["cfg"])
    tp = len(shards)
    full = ref[0]["grads"]
    errs = {}
    for name, g_full in full.items():
        attrs = conv.get_partition_attrs(name, cfg, shards[0]["kv_mult"])
        if not attrs["tp"]:
            got = [s["grads"][name] for s in shards]
            # replicated weights: SP norms hold per-rank partial sums, otherwise every rank the full one
            cands = [sum(got)] if sp and "norm" in name else got
            errs[name] = max(float((c - g_full).abs().max() / g_full.abs().max().clamp(min=1e-30)) for c in cands)
            continue
        e = 0.0
        for r, s in enumerate(shards):
            want = shard_tensor(g_full, attrs, tp, r)
            got = s["grads"][name]
            assert got.shape == want.shape, (name, r, got.shape, want.shape)
            e = max(e, float((got - want).abs().max() / want.abs().max().clamp(min=1e-30)))
        errs[name] = e
    return errs
