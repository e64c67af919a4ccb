"""Workload for PMC counter passes: the framework's hand-written kernels at the Llama-3-8B shapes
(flash attention fwd+bwd at TP=1 and TP=8 head counts, RMSNorm, SwiGLU, cross-entropy, AdamW)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bench_kernels as bk  # noqa: E402

torch.manual_seed(0)
bk.bench_fa(sdpa=False)
bk.bench_fa(Hq=4, Hkv=1, sdpa=False)
bk.bench_mem()

# MoE grouped GEMM (Mixtral TP=8 expert shapes) and the fused decode kernels (Llama-3.2-1B)
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402

C = ops.ext()
E, T, k, H, I = 8, 8192, 2, 4096, 1792
idx = torch.topk(torch.randn(T, E), k).indices.cuda()
_, _, offs = ops.moe_permutation(idx, E)
M = T * k
x = torch.randn(M, H, device="cuda", dtype=torch.bfloat16)
w = torch.randn(E, H, 2 * I, device="cuda", dtype=torch.bfloat16) * 0.02
dy = torch.randn(M, 2 * I, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, 2 * I, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(M, H, device="cuda", dtype=torch.bfloat16)
dw = torch.zeros(E, H, 2 * I, device="cuda")
for _ in range(2):
    C.grouped_gemm(0, x, w, offs, y, False)
    C.grouped_gemm(1, dy, w, offs, dx, False)
    C.grouped_gemm(2, x, dy, offs, dw, True)
xd = torch.randn(1, 2048, device="cuda", dtype=torch.bfloat16)
nw = torch.randn(2048, device="cuda", dtype=torch.bfloat16)
wgu = torch.randn(16384, 2048, device="cuda", dtype=torch.bfloat16) * 0.02
a = torch.empty(1, 8192, device="cuda", dtype=torch.bfloat16)
wd = torch.randn(2048, 8192, device="cuda", dtype=torch.bfloat16) * 0.02
res = torch.zeros(1, 2048, device="cuda", dtype=torch.bfloat16)
kc = torch.randn(1, 8, 1024, 64, device="cuda", dtype=torch.bfloat16)
vc = torch.randn_like(kc)
q = torch.randn(1, 1, 32, 64, device="cuda", dtype=torch.bfloat16)
seq = torch.tensor([1000], device="cuda", dtype=torch.int32)
for _ in range(3):
    C.dgemv(2, xd, nw, 1e-5, wgu, a, 0, 0, 0, None, None, None, 1, None, None, None)
    C.dgemv(1, a, None, 0.0, wd, res, 0, 0, 0, None, None, None, 1, None, None, None)
    ops.decode_attention(q, kc, vc, seq)
torch.cuda.synchronize()
