"""Dense forward GEMM y = x W^T (x [T, H], W [N, H]) at the Llama-3-8B TP=1 shapes: hipBLASLt through
ops.gemm.linear (the framework's tuned path) against this tree's hand-written 256 x 256 ping-pong kernel
(csrc/grouped_rowgemm.hip in its NT mode with one group, NXD_GG_BIG=1).  Interleaved rounds in one
process; random data.  One JSON line per shape: TF/s of each, and what an epilogue-fused replacement
would have to beat (hipBLASLt + the separate elementwise pass it would remove)."""
import json
import os
import statistics
import sys

os.environ.setdefault("NXD_GG_BIG", "1")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import ops  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops import ext  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops.gemm import linear  # noqa: E402

T, H = 8192, 4096
SHAPES = {"qkv": (6144, H), "o_proj": (H, H), "gate_up": (28672, H), "down": (H, 14336)}


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for name, (N, K) in SHAPES.items():
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    offs = torch.tensor([0, T], dtype=torch.int32, device="cuda")
    y1, y2 = torch.empty(T, N, dtype=torch.bfloat16, device="cuda"), torch.empty(T, N, dtype=torch.bfloat16, device="cuda")
    hb = lambda: linear(x, w, out=y1)  # noqa: E731
    hw = lambda: ext().grouped_gemm(1, x, w.unsqueeze(0), offs, y2, False)  # noqa: E731
    res = {"hipblaslt": [], "handwritten": []}
    for _ in range(5):
        res["hipblaslt"].append(timed(hb))
        res["handwritten"].append(timed(hw))
    err = ((y1.float() - y2.float()).abs().max() / y1.float().abs().max()).item()
    fl = 2.0 * T * N * K
    rec = {"shape": name, "T": T, "N": N, "K": K, "max_rel_diff": round(err, 5)}
    for k, v in res.items():
        ms = statistics.median(v)
        rec[k + "_ms"] = round(ms, 4)
        rec[k + "_tflops"] = round(fl / ms / 1e9, 1)
    if name == "gate_up":
        gu = y1
        sw = lambda: ops.swiglu(gu, token_major=True)  # noqa: E731
        rec["swiglu_dual_ms"] = round(statistics.median([timed(sw) for _ in range(3)]), 4)
    print(json.dumps(rec), flush=True)
