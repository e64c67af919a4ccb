"""FA forward / backward TFLOP/s on several shapes (guide comparison point: H=64, Hkv=8, N=2048,
D=128, B=16, random data)."""
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


for (B, S, H, Hkv, causal) in [(16, 2048, 64, 8, False), (16, 2048, 64, 8, True), (1, 8192, 32, 8, True),
                               (1, 8192, 32, 8, False), (4, 8192, 4, 1, True), (2, 4096, 32, 8, True)]:
    q = torch.randn(B, S, H, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * B * H * S * S * 128 * (0.5 if causal else 1.0)
    tf = fl / timed(lambda: ops.flash_attn_fwd_lse(q, k, v, causal=causal)) / 1e9
    qg, kg, vg = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = ops.flash_attn_func(qg, kg, vg, causal=causal)
    do = torch.randn_like(o)
    tb = 2.5 * fl / timed(lambda: torch.autograd.grad(o, (qg, kg, vg), do, retain_graph=True)) / 1e9
    print(json.dumps({"B": B, "S": S, "H": H, "Hkv": Hkv, "causal": causal, "fwd_tf": round(tf, 1),
                      "bwd_tf": round(tb, 1)}), flush=True)
