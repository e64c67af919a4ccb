"""One weight-gradient GEMM shape in a loop (for rocprofv3 --pmc passes and ablations):
    python tools/prof_wgrad.py T M N [reps] [ablate] [splits]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.ops._ext import ext  # noqa: E402

T, M, N = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
ablate = int(sys.argv[5]) if len(sys.argv) > 5 else 0
splits = int(sys.argv[6]) if len(sys.argv) > 6 else 0
dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
mg = torch.zeros(M, N, device="cuda", dtype=torch.float32)
ext().wgrad_gemm_set_ablate(ablate)
ext().wgrad_gemm(mg, dy, x, splits)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    ext().wgrad_gemm(mg, dy, x, splits)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(json.dumps({"T": T, "M": M, "N": N, "ablate": ablate, "splits": splits or ext().wgrad_gemm_splits(T, M, N),
                  "ms": round(ms, 4), "tf": round(2.0 * T * M * N / ms / 1e9, 1)}), flush=True)
