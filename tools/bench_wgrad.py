"""Weight-gradient GEMM: hand-written kernel (csrc/wgrad_gemm.hip) vs the hipBLASLt path of
ops/gemm.wgrad_accumulate_ (TN with transposes where it pays) on the Llama-3-8B TP=1 / TP=8 shapes.
One JSON line per shape; TF/s on random data, interleaved rounds in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.ops import gemm as G  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops._ext import ext  # noqa: E402

SHAPES = [  # (name, tp, tokens, M = out features, N = in features)
    ("qkv", 1, 8192, 6144, 4096), ("o", 1, 8192, 4096, 4096), ("gate_up", 1, 8192, 28672, 4096),
    ("down", 1, 8192, 4096, 14336), ("lm_head", 1, 8192, 128256, 4096),
    ("qkv", 8, 32768, 768, 4096), ("o", 8, 32768, 4096, 512), ("gate_up", 8, 32768, 3584, 4096),
    ("down", 8, 32768, 4096, 1792), ("lm_head", 8, 32768, 16032, 4096),
]


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    only = sys.argv[1:]
    G._WG_KERNEL = "0"   # the comparison arm is the hipBLASLt path (the framework default routes skinny shards to the kernel)
    for name, tp, T, M, N in SHAPES:
        if only and f"{name}{tp}" not in only:
            continue
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        mg = torch.zeros(M, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * T * M * N
        reps = max(3, min(50, int(2e13 / fl)))
        k_fn = lambda: ext().wgrad_gemm(mg, dy, x, 0)  # noqa: E731
        b_fn = lambda: G.wgrad_accumulate_(mg, dy, x)  # noqa: E731
        k_fn(); b_fn(); torch.cuda.synchronize()
        tk, tb = [], []
        for _ in range(3):
            tk.append(timed(k_fn, reps))
            tb.append(timed(b_fn, reps))
        # numerics: one call of each on zeroed accumulators
        mg.zero_(); k_fn(); a = mg.clone(); mg.zero_(); b_fn(); b = mg.clone()
        rel = float((a - b).abs().max() / b.abs().max())
        print(json.dumps({"name": name, "tp": tp, "T": T, "M": M, "N": N,
                          "splits": ext().wgrad_gemm_splits(T, M, N),
                          "kernel_ms": round(min(tk), 4), "kernel_tf": round(fl / min(tk) / 1e9, 1),
                          "hipblaslt_ms": round(min(tb), 4), "hipblaslt_tf": round(fl / min(tb) / 1e9, 1),
                          "max_rel_diff": rel}), flush=True)
        del dy, x, mg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
