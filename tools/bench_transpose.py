"""bf16 transpose kernels (csrc/transpose.hip) at the wgrad-operand and weight-copy shapes of
Llama-3-8B TP=1: the ds_read_b64_tr_b16 tile kernel vs the 16-bit LDS one, interleaved rounds in one
process.  One JSON line per (shape, variant): median ms and TB/s (read + write bytes)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import _C  # noqa: E402

SHAPES = [(8192, 4096), (8192, 6144), (8192, 14336), (8192, 28672), (4096, 128256)]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for R, C in SHAPES:
    x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    y = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
    res = {True: [], False: []}
    for _ in range(5):
        for v in (True, False):
            _C.transpose_set_variant(v)
            res[v].append(timed(lambda: _C.transpose_bf16(x, y)))
    _C.transpose_set_variant(True)
    for v, ms in res.items():
        med = statistics.median(ms)
        print(json.dumps({"R": R, "C": C, "kernel": "tr_b16" if v else "lds16", "ms": round(med, 4),
                          "tbps": round(4 * R * C / med / 1e9, 2)}), flush=True)
