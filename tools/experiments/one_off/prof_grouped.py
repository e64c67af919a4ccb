"""One grouped MoE GEMM (csrc/grouped_rowgemm.hip fwd / dgrad, csrc/wgrad_gemm.hip grouped wgrad) in a
loop, Mixtral-8x7B gate_up shapes (E = 8, 16384 sorted rows), for rocprofv3 --pmc passes:
    python tools/prof_grouped.py MODE [reps]      MODE = 0 fwd | 1 dgrad | 2 wgrad"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402

mode = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
E, T, k, H, I = 8, 8192, 2, 4096, 14336
g = torch.Generator(device="cpu").manual_seed(0)
idx = torch.topk(torch.randn(T, E, generator=g), k).indices.to("cuda")
_, _, offs = ops.moe_permutation(idx, E)
M, K, N = T * k, H, 2 * I
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(E, K, N, device="cuda", dtype=torch.bfloat16) * 0.02
dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
C = ops.ext()
if mode == 0:
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fn = lambda: C.grouped_gemm(0, x, w, offs, out, False)  # noqa: E731
elif mode == 1:
    out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    fn = lambda: C.grouped_gemm(1, dy, w, offs, out, False)  # noqa: E731
else:
    out = torch.zeros(E, K, N, device="cuda", dtype=torch.float32)
    fn = lambda: C.grouped_gemm(2, x, dy, offs, out, True)  # noqa: E731
fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    fn()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(json.dumps({"mode": mode, "M": M, "K": K, "N": N, "E": E, "ms": round(ms, 4),
                  "tf": round(2.0 * M * K * N / ms / 1e9, 1)}), flush=True)
