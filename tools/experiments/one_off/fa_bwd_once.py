"""Run the flash-attention backward a few times at one shape (profiling target)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--hq", type=int, default=32)
ap.add_argument("--hkv", type=int, default=8)
ap.add_argument("--s", type=int, default=8192)
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
D = 128
q = torch.randn(1, a.s, a.hq, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(1, a.s, a.hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(1, a.s, a.hkv, D, device="cuda", dtype=torch.bfloat16)
o, lse = ops.flash_attn_fwd_lse(q, k, v, causal=True)
do = torch.randn_like(o)
dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
for _ in range(a.iters):
    ops.ext().flash_attn_bwd(q, k, v, o, do, lse, dq, dk, dv, D ** -0.5, True, 0)
torch.cuda.synchronize()
print("ok")
