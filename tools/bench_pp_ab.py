"""A/B of the ping-pong main loop (staggered wave groups, two 16-MFMA phases per stage) against the
one-barrier-per-stage loop of the two hand-written GEMMs: the grouped MoE row GEMM
(csrc/grouped_rowgemm.hip, Mixtral-8x7B shapes) and the token-major weight-gradient kernel
(csrc/wgrad_gemm.hip, dense Llama-3-8B TP=1 / TP=8 shards and grouped MoE).  Interleaved rounds in
one process; each line also reports the max relative difference of each PP output to the old one.
v0 = one barrier per stage, v1 = ping-pong with the LDS-DMA issued in the load phase."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402


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


VARIANTS = (0, 1)   # one barrier per stage | ping-pong (a third, DMA inside the MFMA burst, was measured and
                    # dropped: profiles/r3_pp_dma_in_mfma_rejected.jsonl)


def ab(kname, fl, fn, out, setter, reps=10, rounds=3, zero=False, **info):
    outs = {}
    for v in VARIANTS:
        setter(v)
        if zero:
            out.zero_()
        fn()
        torch.cuda.synchronize()
        outs[v] = out.float().clone()
    t = {v: [] for v in VARIANTS}
    for _ in range(rounds):
        for v in VARIANTS:
            setter(v)
            t[v].append(timed(fn, reps))
    setter(1)
    ref = outs[0]
    res = {"kernel": kname, **info}
    for v in VARIANTS:
        res[f"v{v}_tf"] = round(fl / min(t[v]) / 1e9, 1)
    for v in VARIANTS[1:]:
        res[f"v{v}_max_rel_diff"] = float((outs[v] - ref).abs().max() / ref.abs().max().clamp(min=1e-30))
    print(json.dumps(res), flush=True)
    return res


def main():
    C = ops.ext()
    E, T, k, H = 8, 8192, 2, 4096
    g = torch.Generator(device="cpu").manual_seed(0)
    idx = torch.topk(torch.randn(T, E, generator=g), k).indices.to("cuda")
    _, _, offs = ops.moe_permutation(idx, E)
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
            info = {"tp": tp, "proj": name, "M": M, "K": K, "N": N}
            ab("moe_fwd", fl, lambda: C.grouped_gemm(0, x, w, offs, y, False), y, C.grouped_rowgemm_set_pp, **info)
            ab("moe_dgrad", fl, lambda: C.grouped_gemm(1, dy, w, offs, dx, False), dx, C.grouped_rowgemm_set_pp, **info)
            ab("moe_wgrad", fl, lambda: C.grouped_gemm(2, x, dy, offs, dw, True), dw, C.wgrad_gemm_set_pp, zero=True,
               **info)
            del x, w, dy, y, dx, dw
            torch.cuda.empty_cache()
    for name, tp, Tt, Mo, Ni in [("qkv", 8, 32768, 768, 4096), ("o", 8, 32768, 4096, 512), ("qkv", 1, 8192, 6144, 4096),
                                 ("gate_up", 1, 8192, 28672, 4096)]:
        dy = torch.randn(Tt, Mo, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(Tt, Ni, device="cuda", dtype=torch.bfloat16)
        mg = torch.zeros(Mo, Ni, device="cuda", dtype=torch.float32)
        ab("dense_wgrad", 2.0 * Tt * Mo * Ni, lambda: C.wgrad_gemm(mg, dy, x, 0), mg, C.wgrad_gemm_set_pp, zero=True,
           name=name, tp=tp, T=Tt, M=Mo, N=Ni)
        del dy, x, mg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
