"""One dropless MoE layer forward + backward (router, permutation, expert MLPs, un-permute) on
Mixtral-8x7B expert shapes at TP=1 (E = 8, top-2, H = 4096, I = 14336), comparing the two expert
GEMM backends of ops/grouped_gemm.py: the device-side grouped kernel (no host sync) and the
per-expert hipBLASLt loop (NXD_MOE_GEMM=loop, one host read of the group sizes per layer).
Prints one JSON line per (backend, tokens) with ms per fwd+bwd and expert-GEMM TFLOP/s."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402
from neuronx_distributed_llama3_2_amd.modules.moe import MoE, ExpertMLPs, RouterTopK  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29651")
    dist.init_process_group("gloo", rank=0, world_size=1)
    ps.initialize_model_parallel(1)
    E, k, H, I = 8, 2, 4096, 14336
    torch.manual_seed(0)
    layer = MoE(RouterTopK(E, k, H), ExpertMLPs(E, k, H, I, "silu", True, None, normalize_top_k_affinities=True,
                                               dtype=torch.bfloat16), return_router_logits=False).cuda()
    layer.train()
    tokens = [int(a) for a in os.environ.get("MOE_TOKENS", "4096,16384").split(",")]
    backends = os.environ.get("MOE_BACKENDS", "grouped,loop,grouped,loop").split(",")
    for T in tokens:
        x = (torch.randn(T, 1, H, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_(True)
        dy = torch.randn(T, 1, H, device="cuda", dtype=torch.bfloat16)
        flops = 3 * 2.0 * T * k * H * 3 * I          # (gate_up 2I + down I) x (fwd + dgrad + wgrad)
        for backend in backends:   # alternated by default: the second pass of each is the one to read
            ops.grouped_gemm.MOE_GEMM = backend

            def step():
                out = layer(x)
                out = out[0] if isinstance(out, tuple) else out
                out.backward(dy)
                layer.zero_grad(set_to_none=True)
                x.grad = None

            for _ in range(2):
                step()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            s.record()
            for _ in range(reps):
                step()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / reps
            print(json.dumps({"backend": backend, "tokens": T, "E": E, "top_k": k, "H": H, "I": I,
                              "ms_fwd_bwd": round(ms, 3), "expert_gemm_tflops": round(flops / ms / 1e9, 1)}),
                  flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
