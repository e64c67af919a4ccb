"""Mixtral-8x7B training throughput on ONE GPU with a reduced layer count (the full 47B-parameter
model needs ~750 GB of weights + fp32 optimizer state: 8 GPUs with TP/EP).  Full-width layers
(H 4096, I 14336, 8 experts, top-2, 32 q / 8 kv heads), synthetic tokens, random init, bf16
compute, fp32-master AdamW, dropless MoE.  One JSON line per expert-GEMM backend with tokens/s
and model TFLOP/s (active parameters: attention + router + top-2 of 8 experts, plus causal
attention FLOPs).

    python tools/bench_mixtral_train.py --layers 4 --seq 4096 --mbs 2 --accum 4 --steps 3
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402
from neuronx_distributed_llama3_2_amd.models.mixtral import MixtralForCausalLM, mixtral_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--accum", type=int, default=4, help="micro-batches per optimizer step")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--backends", default="grouped,loop")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ps.initialize_model_parallel(tensor_model_parallel_size=1)
    dev = torch.device("cuda", 0)
    cfg = mixtral_config("mixtral-8x7b", num_hidden_layers=a.layers, max_position_embeddings=max(4096, a.seq))
    torch.manual_seed(0)
    model = MixtralForCausalLM(cfg, dtype=torch.bfloat16, device=dev)
    model.train()
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=1e-5)
    H, I, E, k, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_local_experts, cfg.num_experts_per_tok, a.layers
    hd = H // cfg.num_attention_heads
    attn_params = H * (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * hd + cfg.num_attention_heads * hd * H
    active = L * (attn_params + E * H + k * 3 * H * I) + cfg.vocab_size * H      # + lm_head
    flops_per_token = 6 * active + 6 * L * H * a.seq                            # causal attention: half of 12 L H S
    g = torch.Generator(device="cpu").manual_seed(1)

    def step():
        for _ in range(a.accum):
            ids = torch.randint(0, cfg.vocab_size, (a.mbs, a.seq), generator=g).to(dev, non_blocking=True)
            loss = model(ids, labels=ids).loss / a.accum
            loss.backward()
        opt.step()
        opt.zero_grad()
        return loss.detach() * a.accum

    for backend in a.backends.split(","):
        ops.grouped_gemm.MOE_GEMM = backend
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            loss = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        tok = a.accum * a.mbs * a.seq / dt
        print(json.dumps({"model": f"mixtral-8x7b-{L}L", "backend": backend, "seq": a.seq, "mbs": a.mbs, "accum": a.accum,
                          "ms_per_step": round(dt * 1e3, 2), "tokens_per_s": round(tok, 1),
                          "model_tflops": round(tok * flops_per_token / 1e12, 1),
                          "mfu_vs_2.5PF": round(tok * flops_per_token / 2.5e15, 3), "loss": round(float(loss), 4),
                          "peak_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
