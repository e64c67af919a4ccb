"""Measure the training memory of one micro-batch on ONE GPU, split into the resident part (bf16
weights, fp32 master + Adam moments, fp32 main grads, K-major dgrad weight copies) and the
activation peak of a forward + backward, per layer (difference of two layer counts), for a model
preset at TP=N per-rank *shapes* (no communication; without sequence parallelism every
elementwise activation is held for all S rows).  Calibrates utils/memory_planner.py.

    python tools/measure_activation_memory.py --model llama3-8b --tp 1 --layers 2 4 --ckpt none selective full
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402


def one(a, layers, ckpt, dev):
    base = llama_config(a.model)
    tp = a.tp
    over = dict(num_attention_heads=base.num_attention_heads // tp,
                num_key_value_heads=max(1, base.num_key_value_heads // tp),
                intermediate_size=base.intermediate_size // tp, head_dim=base.hidden_size // base.num_attention_heads,
                vocab_size=base.vocab_size // tp, num_hidden_layers=layers,
                max_position_embeddings=max(8192, a.seq))
    if ckpt == "full":
        over["activation_checkpoint"] = "full"
    elif ckpt == "selective":
        over["selective_checkpoint_enabled"] = True
    cfg = llama_config(a.model, **over)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=dev)
    model.train()
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=1e-6)
    ids = torch.randint(0, cfg.vocab_size, (a.mbs, a.seq), device=dev)

    def step():
        out = model(ids, labels=ids)
        out.loss.backward()
        opt.step()
        opt.zero_grad()

    step()  # creates the optimizer state, the K-major dgrad copies and the GEMM workspaces
    torch.cuda.synchronize()
    resident = torch.cuda.memory_allocated(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    step()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(dev)
    nparams = sum(p.numel() for p in model.parameters())
    del model, opt, ids
    torch.cuda.empty_cache()
    return {"params": nparams, "resident_bytes": resident, "peak_bytes": peak, "activation_peak_bytes": peak - resident}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--layers", type=int, nargs=2, default=[2, 4])
    ap.add_argument("--ckpt", nargs="+", default=["none", "selective", "full"])
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ps.initialize_model_parallel(tensor_model_parallel_size=1)
    dev = torch.device("cuda", 0)
    torch.empty(1, device=dev)  # (allocator initialised before the first peak-stat reset)
    l1, l2 = a.layers
    for ckpt in a.ckpt:
        r1 = one(a, l1, ckpt, dev)
        r2 = one(a, l2, ckpt, dev)
        per_layer_act = (r2["activation_peak_bytes"] - r1["activation_peak_bytes"]) / (l2 - l1)
        per_layer_params = (r2["params"] - r1["params"]) / (l2 - l1)
        per_layer_res = (r2["resident_bytes"] - r1["resident_bytes"]) / (l2 - l1)
        print(json.dumps({"model": a.model, "tp_shapes": a.tp, "seq": a.seq, "mbs": a.mbs, "ckpt": ckpt,
                          "layers": [l1, l2], "act_bytes_per_layer": per_layer_act,
                          "act_bytes_per_layer_per_token": per_layer_act / (a.seq * a.mbs),
                          "resident_bytes_per_layer": per_layer_res,
                          "resident_bytes_per_param": per_layer_res / per_layer_params,
                          "act_fixed_bytes": r1["activation_peak_bytes"] - l1 * per_layer_act,
                          "peak_gib": [round(r1["peak_bytes"] / 2**30, 2), round(r2["peak_bytes"] / 2**30, 2)]}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
