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


def price_dq_slabs():
    """Price of an atomic-free dQ (round-4 review item): every (query row, 256-key block) pair's
    partial stored plainly into a per-key-block slab, then one pass summing the slabs per row.
    Measured pieces at S=8192 causal, 32 q heads, D=128, B=1 (2.21 GB of dQ partials):
      store: a kernel writing that many fp32 bytes (torch fill of a fresh buffer) -- the bytes the
             main kernel would add to its HBM traffic (overlappable with its compute);
      reduce: reading them back and summing per row (torch sum over the slab axis), which replaces
             the current memset + fp32->bf16 convert of the 0.14 GB dQ accumulator.
    Compare: full kernel (atomics) vs no_dq_atomics body + reduce (the store is at best hidden)."""
    n_pairs = sum(8192 - kb * 256 for kb in range(32))          # 135,168 (query row, key block) pairs
    nbytes = n_pairs * 128 * 4 * 32
    buf = torch.empty(nbytes // 4, device="cuda", dtype=torch.float32)
    rows = 32 * 8192
    slabs = buf[: (nbytes // 4) // (rows * 128) * rows * 128].view(-1, rows, 128)   # ~16.5 slabs of all rows
    out = torch.empty(rows, 128, device="cuda", dtype=torch.bfloat16)

    def t(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    store = t(lambda: buf.fill_(1.0))
    reduce = t(lambda: out.copy_(slabs.sum(0)))
    print(json.dumps({"dq_slab_bytes_GB": round(nbytes / 1e9, 3), "store_ms": round(store, 4),
                      "store_TBps": round(nbytes / store / 1e9, 2), "reduce_ms": round(reduce, 4),
                      "reduce_read_TBps": round(slabs.numel() * 4 / reduce / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
    price_dq_slabs()
