"""Timing-only ablation of the flash-attention backward kernel (outputs are wrong when a phase
is switched off; only the time matters).  Interleaves variants in one process.

    python tools/bench_fa_ablate.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd import ops  # noqa: E402

VARIANTS = {"full": 0, "no_dq_atomics": 1, "no_dkdv_atomics": 2, "no_atomics": 3, "no_tile_loads": 16,
            "no_barriers": 32, "no_loads_no_bar": 48, "no_atomics_loads_bar": 51}


def main():
    dev = "cuda"
    for (Hq, Hkv) in ((32, 8), (4, 1)):
        S, D, B = 8192, 128, 1
        q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
        o, lse = ops.flash_attn_fwd_lse(q, k, v, causal=True)
        do = torch.randn_like(o)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        ext = ops.ext()
        scale = D ** -0.5

        def run():
            ext.flash_attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True, 0)

        times = {n: [] for n in VARIANTS}
        for rep in range(5):
            for n, f in VARIANTS.items():
                ext.flash_attn_set_knob(0, f)
                run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / 5)
        ext.flash_attn_set_knob(0, 0)
        flops = 2.5 * 4 * B * Hq * S * S * D / 2
        for n, t in times.items():
            m = sorted(t)[len(t) // 2]
            print(json.dumps({"Hq": Hq, "Hkv": Hkv, "variant": n, "ms": round(m, 4), "tflops_equiv": round(flops / m / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
