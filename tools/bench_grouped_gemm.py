"""MoE grouped GEMM (csrc/grouped_gemm.hip) vs a per-expert hipBLASLt loop (host-known group sizes)
on Mixtral-8x7B expert shapes: E = 8, top-2, 8192 tokens (M = 16384 sorted rows), H = 4096,
I = 14336 / TP.  Prints one JSON line per (TP, projection) with TFLOP/s of fwd / dgrad / wgrad."""
import json
import sys

import torch

sys.path.insert(0, ".")
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402


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


def main():
    C = ops.ext()
    E, T, k, H = 8, 8192, 2, 4096
    g = torch.Generator(device="cpu").manual_seed(0)
    logits = torch.randn(T, E, generator=g)
    idx = torch.topk(logits, k).indices.to("cuda")
    _, _, offs = ops.moe_permutation(idx, E)
    counts = (offs[1:] - offs[:-1]).tolist()
    M = T * k
    for tp in (1, 8):
        I = 14336 // tp
        for name, (K, N) in {"gate_up": (H, 2 * I), "down": (I, H)}.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(E, K, N, device="cuda", dtype=torch.bfloat16) * 0.02
            dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
            dw = torch.zeros(E, K, N, device="cuda", dtype=torch.float32)
            fl = 2.0 * M * K * N
            r = {"tp": tp, "proj": name, "M": M, "K": K, "N": N, "E": E}
            r["fwd_grouped_tf"] = fl / timed(lambda: C.grouped_gemm(0, x, w, offs, y, False)) / 1e9
            r["dgrad_grouped_tf"] = fl / timed(lambda: C.grouped_gemm(1, dy, w, offs, dx, False)) / 1e9
            r["wgrad_grouped_tf"] = fl / timed(lambda: C.grouped_gemm(2, x, dy, offs, dw, True)) / 1e9

            from neuronx_distributed_llama3_2_amd.ops.grouped_gemm import _loop_dgrad, _loop_fwd, _loop_wgrad

            bounds = offs.tolist()   # the framework's loop backend (NXD_MOE_GEMM=loop): fp32-output addmm wgrad
            loop_fwd = lambda: _loop_fwd(x, w, bounds, y)  # noqa: E731
            loop_dgrad = lambda: _loop_dgrad(dy, w, bounds, dx)  # noqa: E731
            loop_wgrad = lambda: _loop_wgrad(x, dy, bounds, dw, True)  # noqa: E731

            r["fwd_loop_tf"] = fl / timed(loop_fwd) / 1e9
            r["dgrad_loop_tf"] = fl / timed(loop_dgrad) / 1e9
            r["wgrad_loop_tf"] = fl / timed(loop_wgrad) / 1e9
            print(json.dumps({a: (round(b, 1) if isinstance(b, float) else b) for a, b in r.items()}), flush=True)
            del x, w, dy, y, dx, dw


if __name__ == "__main__":
    main()
