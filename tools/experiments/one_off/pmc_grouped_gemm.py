"""Run the three grouped-GEMM kernels (Mixtral gate_up, TP=1, 16384 sorted rows) twice each, for
rocprofv3 --pmc passes (tools/gpu_gg_pmc.sh)."""
import sys

import torch

sys.path.insert(0, ".")
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402

C = ops.ext()
E, T, k, H, I = 8, 8192, 2, 4096, 14336
g = torch.Generator(device="cpu").manual_seed(0)
idx = torch.topk(torch.randn(T, E, generator=g), k).indices.to("cuda")
_, _, offs = ops.moe_permutation(idx, E)
M, K, N = T * k, H, 2 * I
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(E, K, N, device="cuda", dtype=torch.bfloat16) * 0.02
dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
dw = torch.zeros(E, K, N, device="cuda", dtype=torch.float32)
for _ in range(2):
    C.grouped_gemm(0, x, w, offs, y, False)
    C.grouped_gemm(1, dy, w, offs, dx, False)
    C.grouped_gemm(2, x, dy, offs, dw, True)
torch.cuda.synchronize()
print("ok")
