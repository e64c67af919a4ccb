"""A/B of the FA forward block->XCD map (variant bits 64 / 128 on top of the default 13), interleaved
rounds in one process, causal shapes of the bench (TP=1 and TP=8 per-rank) plus the guide shape.
Outputs are compared bit-for-bit against the default map."""
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


C = ops.ext()
variants = {"contiguous": 13, "balanced": 13 | 64, "interleaved": 13 | 128}
for (B, S, H, Hkv) in [(1, 8192, 32, 8), (4, 8192, 4, 1), (2, 8192, 4, 1), (2, 4096, 32, 8), (16, 2048, 64, 8),
                       (1, 16384, 32, 8)]:
    q = torch.randn(B, S, H, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * B * H * S * S * 128
    C.flash_attn_set_knob(2, 13)
    ref, _ = ops.flash_attn_fwd_lse(q, k, v, causal=True)
    ref = ref.clone()
    res = {k_: [] for k_ in variants}
    for _ in range(3):
        for name, var in variants.items():
            C.flash_attn_set_knob(2, var)
            res[name].append(fl / timed(lambda: ops.flash_attn_fwd_lse(q, k, v, causal=True)) / 1e9)
    same = {}
    for name, var in variants.items():
        C.flash_attn_set_knob(2, var)
        o, _ = ops.flash_attn_fwd_lse(q, k, v, causal=True)
        same[name] = bool(torch.equal(o, ref))
    C.flash_attn_set_knob(2, 13)
    print(json.dumps({"B": B, "S": S, "H": H, "Hkv": Hkv, **{f"{n}_tf": round(max(t), 1) for n, t in res.items()},
                      "bitwise_equal": same}), flush=True)
