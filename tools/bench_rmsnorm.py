"""RMSNorm fwd (+ residual) / bwd (+ residual gradient, dw accumulated into an fp32 main_grad) on
the HIP kernels, row-per-wave path vs the one-row-per-workgroup path (`_C.rmsnorm_set_rows_path`),
interleaved rounds in ONE process (cdna_hip_programming.md rule 24).  Minimum bytes: fwd reads x, res
and writes y, h (4 T H x 2 B); bwd reads dy, h, dres and writes dx (4 T H x 2 B).  One JSON line per
(T, path, direction): median / min ms over the rounds and TB/s on the minimum bytes."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import _C  # noqa: E402

H = int(os.environ.get("H", "4096"))
ROUNDS, REPS = 7, 20


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / REPS


for T in (8192, 16384, 32768):
    x, r = (torch.randn(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    w = (1 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16)
    y, h = torch.empty_like(x), torch.empty_like(x)
    rstd = torch.empty(T, device="cuda", dtype=torch.float32)
    dy, dres = torch.randn_like(x), torch.randn_like(x)
    dx = torch.empty_like(x)
    dw = torch.zeros(H, device="cuda", dtype=torch.float32)
    fwd = lambda: _C.rmsnorm_fwd(x, r, w, y, h, rstd, 1e-5)  # noqa: E731
    bwd = lambda: _C.rmsnorm_bwd(dy, h, w, rstd, dres, dx, dw, True)  # noqa: E731
    res = {}
    for _ in range(ROUNDS):
        for path in (1, 0):
            _C.rmsnorm_set_rows_path(bool(path))
            for name, fn in (("fwd", fwd), ("bwd", bwd)):
                fn()
                res.setdefault((path, name), []).append(timed(fn))
    for (path, name), ms in sorted(res.items()):
        med = statistics.median(ms)
        print(json.dumps({"T": T, "H": H, "op": name, "path": "rows" if path else "row_per_wg", "ms_median": round(med, 4),
                          "ms_min": round(min(ms), 4), "tbps_min_bytes": round(4 * T * H * 2 / med / 1e9, 2)}), flush=True)
    del x, r, y, h, dy, dres, dx
