"""RMSNorm backward (csrc/rmsnorm.hip bwd + colsum) at the TP=1 bench shape: one half micro-batch of
8192 tokens x 4096, with the residual gradient.  Prints one JSON line (mean of 50 timed calls).
NXD_RMS_BWD_PIPE=0|1 selects the unpipelined / pipelined row loop (read once per process)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402

T, H = int(os.environ.get("T", "8192")), 4096
x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
r = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
w = torch.ones(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
y, h = ops.rms_norm(x, w, 1e-5, residual=r)
dy, dh = torch.randn_like(y), torch.randn_like(h)


def step():
    torch.autograd.backward([y, h], [dy, dh], retain_graph=True)


for _ in range(5):
    step()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(50):
    step()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 50
print(json.dumps({"pipe": os.environ.get("NXD_RMS_BWD_PIPE", "1"), "T": T, "H": H, "ms": round(ms, 4),
                  "tbps_min_bytes": round(4 * T * H * 2 / ms / 1e9, 2)}), flush=True)
