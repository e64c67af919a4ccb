"""PMC workload: the hand-written dense GEMM (csrc/dense_gemm.hip) and hipBLASLt on one shape, a few
launches each (rocprofv3 --pmc passes aggregate per kernel name).
Usage: python tools/pmc_dense_gemm.py [T N K] [--tn]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.ops import ext  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops import gemm as G  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
T, N, K = (int(v) for v in args) if args else (8192, 4096, 4096)
x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
y = torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
if "--tn" in sys.argv:
    dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
    mg = torch.zeros(N, K, device="cuda")
    for _ in range(5):
        ext().dense_gemm(1, 1, dy, x, mg)
        G.ext().gemm(G.transpose(dy), G.transpose(x).t(), mg, None, 1.0, 1.0)
else:
    for _ in range(5):
        ext().dense_gemm(0, 0, x, w, y)
        G.linear(x, w, out=y)
torch.cuda.synchronize()
