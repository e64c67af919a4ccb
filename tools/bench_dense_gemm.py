"""The hand-written dense GEMM (csrc/dense_gemm.hip) against the framework's hipBLASLt paths at the
Llama-3-8B shapes of the bench: TP=1 (8,192-token halves) and the TP=8 per-rank shards (65,536 tokens,
micro-batch 8).  Per shape and pass:

  fwd    y[T, N]  = x[T, K] W[N, K]^T           hipBLASLt (ops.gemm.linear)  vs  NT, bf16 out
  dgrad  dx[T, K] = dy[T, N] W[N, K]            hipBLASLt on the K-major copy (ops.gemm.dgrad)  vs  NT on it
  wgrad  mg[N, K] += dy[T, N]^T x[T, K]         the framework's route (hipBLASLt TN + the two operand
                                                transposes, or the older wgrad kernel)  vs  TN fp32 += acc
                                                (one RMW per element) and TN split-K atomics

Interleaved rounds in one process, random data, median ms; max |err| / max |ref| against an fp32
torch reference.  One JSON line per (shape, pass).
Usage: python tools/bench_dense_gemm.py [--set tp1|tp8|all] [--reps 10] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.ops import ext  # noqa: E402
from neuronx_distributed_llama3_2_amd.ops import gemm as G  # noqa: E402

TP1 = {"qkv": (8192, 6144, 4096), "o_proj": (8192, 4096, 4096), "gate_up": (8192, 28672, 4096),
       "down": (8192, 4096, 14336), "lm_head": (8192, 128256, 4096)}
TP8 = {"qkv": (65536, 768, 4096), "o_proj": (65536, 4096, 512), "gate_up": (65536, 3584, 4096),
       "down": (65536, 4096, 1792), "lm_head": (65536, 16032, 4096)}


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def rel_err(got, ref):
    return ((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()


def run(name, T, N, K, passes, reps, rounds, tag):
    dev = "cuda"
    x = torch.randn(T, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
    dy = torch.randn(T, N, device=dev).to(torch.bfloat16)
    out = []
    for ps in passes:
        if ps == "fwd":
            flops = 2.0 * T * N * K
            y1 = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
            y2 = torch.empty_like(y1)
            arms = {"hipblaslt": lambda: G.linear(x, w, out=y1),
                    "handwritten": lambda: ext().dense_gemm(0, 0, x, w, y2)}
            check = lambda: ([f() for f in arms.values()], rel_err(y2, x.float() @ w.float().t()),  # noqa: E731
                             rel_err(y1, x.float() @ w.float().t()))[1:]
        elif ps == "dgrad":
            flops = 2.0 * T * N * K
            wt = w.t().contiguous()
            d1 = torch.empty(T, K, dtype=torch.bfloat16, device=dev)
            d2 = torch.empty_like(d1)
            arms = {"hipblaslt": lambda: G.matmul(dy, wt.t(), out=d1),
                    "handwritten": lambda: ext().dense_gemm(0, 0, dy, wt, d2)}
            check = lambda: ([f() for f in arms.values()], rel_err(d2, dy.float() @ w.float()),  # noqa: E731
                             rel_err(d1, dy.float() @ w.float()))[1:]
        else:
            flops = 2.0 * T * N * K
            mg = [torch.zeros(N, K, dtype=torch.float32, device=dev) for _ in range(4)]
            splits = ext().dense_gemm_splits(N, K, T)
            arms = {"framework": lambda: G.wgrad_accumulate_(mg[0], dy, x),
                    "hipblaslt_tn": lambda: G.ext().gemm(G.transpose(dy), G.transpose(x).t(), mg[1], None, 1.0, 1.0),
                    "handwritten": lambda: ext().dense_gemm(1, 1, dy, x, mg[2]),
                    "handwritten_atomic": lambda: ext().dense_gemm(1, 2, dy, x, mg[3], 0)}

            def check():
                ref = dy.float().t() @ x.float()
                res = []
                for i, fn in ((2, arms["handwritten"]), (3, arms["handwritten_atomic"]), (0, arms["framework"])):
                    mg[i].zero_()
                    fn()
                    res.append(rel_err(mg[i], ref))
                return tuple(res)
        errs = check()
        if PIPES:
            for k in [k for k in arms if k.startswith("handwritten")]:
                fn = arms.pop(k)
                for pv in PIPES:
                    arms[f"{k}_p{pv}"] = (lambda f, v: (lambda: (ext().dense_gemm_set_pipe(v), f())))(fn, pv)
        res = {k: [] for k in arms}
        for _ in range(rounds):
            for k, fn in arms.items():
                res[k].append(timed(fn, reps))
        rec = {"set": tag, "shape": name, "pass": ps, "T": T, "N": N, "K": K, "rel_err": [round(e, 6) for e in errs]}
        if ps == "wgrad":
            rec["atomic_splits"] = splits
        for k, v in res.items():
            ms = statistics.median(v)
            rec[k + "_ms"] = round(ms, 4)
            rec[k + "_tflops"] = round(flops / ms / 1e9, 1)
        print(json.dumps(rec), flush=True)
        out.append(rec)
    return out


PIPES = []


def main():
    global PIPES
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="all")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--pipes", default="", help="A/B the main-loop variants (dense_gemm_set_pipe), e.g. 0,1")
    a = ap.parse_args()
    PIPES = [int(v) for v in a.pipes.split(",") if v]
    sets = {"tp1": TP1, "tp8": TP8}
    for tag in (["tp1", "tp8"] if a.set == "all" else [a.set]):
        for name, (T, N, K) in sets[tag].items():
            if a.shapes and name not in a.shapes.split(","):
                continue
            passes = a.passes.split(",")
            if name == "lm_head" and tag == "tp1":
                passes = [p for p in passes if p != "dgrad"]
            run(name, T, N, K, passes, a.reps, a.rounds, tag)


if __name__ == "__main__":
    main()
