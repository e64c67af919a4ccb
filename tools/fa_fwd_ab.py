"""A/B of flash-attention forward variants (NXD_FA_FWD_VARIANT) at the Llama-3-8B TP=1 and TP=8
head shapes; checks each variant against the default output.  One JSON line per (variant, shape)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402
from bench_kernels import timeit  # noqa: E402

for (Hq, Hkv) in ((32, 8), (4, 1)):
    S, D = 8192, 128
    q = torch.randn(1, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    ops.ext().flash_attn_set_knob(2, 0)
    ref, _ = ops.flash_attn_fwd_lse(q, k, v, causal=True)
    fl = 4 * Hq * S * S * D / 2
    for var in sys.argv[1:] or ["0", "1", "2", "3"]:
        ops.ext().flash_attn_set_knob(2, int(var))
        o, _ = ops.flash_attn_fwd_lse(q, k, v, causal=True)
        err = float((o.float() - ref.float()).abs().max())
        t = timeit(lambda: ops.flash_attn_fwd_lse(q, k, v, causal=True), iters=30)
        print(json.dumps({"variant": var, "Hq": Hq, "Hkv": Hkv, "ms": round(t, 4), "tflops": round(fl / t / 1e9, 1),
                          "max_abs_diff_vs_default": err}), flush=True)
