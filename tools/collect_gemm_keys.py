"""Record the hipBLASLt GEMM problem keys one Llama training step issues at TP=N (input of
tools/tune_gemm.py).  All ranks share cuda:0 and talk over gloo, so TP=2/4/8 key sets can be
collected on a one-GPU box; GEMM shapes do not depend on the layer count, so 2 layers suffice.

    NXD_GEMM_LOG_KEYS=keys.txt python -m torch.distributed.run --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port 29601 tools/collect_gemm_keys.py --tp N
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--layers", type=int, default=2)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29601")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ps.initialize_model_parallel(tensor_model_parallel_size=a.tp)
    model_parallel_manual_seed(1)
    cfg = llama_config(a.model, num_hidden_layers=a.layers, sequence_parallel_enabled=a.tp > 1,
                       max_position_embeddings=max(8192, a.seq))
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device("cuda", 0))
    for p in model.parameters():  # wgrad accumulates into fp32 main_grad, as under the flat buffers
        p.main_grad = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
    ids = torch.randint(0, cfg.vocab_size, (1, a.seq), device="cuda")
    out = model(ids, labels=ids)
    out.loss.backward()
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        print(f"collected keys for tp={a.tp}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
