"""Flash attention fwd / bwd TFLOP/s with in-kernel dropout (p = 0.1) vs without, Llama-3-8B
attention shapes (S = 8192, D = 128, causal)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from neuronx_distributed_llama3_2_amd.ops.flash_attn import FlashAttnFunc, _fwd  # noqa: E402


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


for (B, S, H, Hkv) in [(1, 8192, 32, 8), (1, 8192, 4, 1)]:
    q = torch.randn(B, S, H, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16)
    fl = 4.0 * B * H * S * S * 128 * 0.5
    for p in (0.0, 0.1):
        drop = (p, 1234, 0)
        tf = fl / timed(lambda: _fwd(q, k, v, True, 128 ** -0.5, 0, dropout=drop)) / 1e9
        qg, kg, vg = (t.clone().requires_grad_(True) for t in (q, k, v))
        o = FlashAttnFunc.apply(qg, kg, vg, True, 128 ** -0.5, 0, drop)
        do = torch.randn_like(o)
        tb = 2.5 * fl / timed(lambda: torch.autograd.grad(o, (qg, kg, vg), do, retain_graph=True)) / 1e9
        print(json.dumps({"B": B, "S": S, "H": H, "Hkv": Hkv, "dropout_p": p, "fwd_tf": round(tf, 1),
                          "bwd_tf": round(tb, 1)}), flush=True)
