"""A/B of the flash-attention backward's dK/dV reduction: f32 atomics (knob 5 = 0) vs per-item
slabs + convert pass (knob 5 = 1), interleaved in one process; outputs compared bitwise / max diff.

    python tools/bench_fab_slab.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    ext = ops.ext()
    for (B, Hq, Hkv, D) in ((1, 32, 8, 128), (4, 4, 1, 128), (1, 4, 1, 128), (2, 16, 4, 64)):
        S = 8192
        torch.manual_seed(0)
        q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
        o, lse = ops.flash_attn_fwd_lse(q, k, v, causal=True)
        do = torch.randn_like(o)
        scale = D ** -0.5
        outs = {}

        def run(dq, dk, dv):
            ext.flash_attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True, 0, 0.0, 0, 0)

        times = {0: [], 1: []}
        for rep in range(5):
            for mode in (0, 1):
                ext.flash_attn_set_knob(5, mode)
                bufs = outs.setdefault(mode, (torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)))
                run(*bufs)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run(*bufs)
                e1.record()
                torch.cuda.synchronize()
                times[mode].append(e0.elapsed_time(e1) / 10)
        ext.flash_attn_set_knob(5, -1)
        flops = 2.5 * 4 * B * Hq * S * S * D / 2
        med = {m: sorted(t)[len(t) // 2] for m, t in times.items()}
        diff = {n: (outs[0][i].float() - outs[1][i].float()).abs().max().item() for i, n in enumerate(("dq", "dk", "dv"))}
        print(json.dumps({"B": B, "Hq": Hq, "Hkv": Hkv, "D": D, "S": S,
                          "atomics_ms": round(med[0], 4), "slab_ms": round(med[1], 4),
                          "atomics_tf": round(flops / med[0] / 1e9, 1), "slab_tf": round(flops / med[1] / 1e9, 1),
                          "rounds": {m: [round(x, 4) for x in t] for m, t in times.items()},
                          "max_abs_diff": diff}), flush=True)


if __name__ == "__main__":
    main()
