"""A/B of the FA backward work-item -> XCD map (knob 3: 0 contiguous per XCD, 2 interleaved) and
the work-item chunk (knob 1, 0 = model), interleaved rounds in one process; gradients compared
against the round-1 configuration."""
import json
import sys

import torch

sys.path.insert(0, ".")
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402


def timed(fn, reps=6):
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
variants = {"contig_auto": (0, 0), "inter_auto": (2, 0), "inter_c32": (2, 32), "inter_c64": (2, 64),
            "inter_c128": (2, 128)}
for (B, S, H, Hkv) in [(1, 8192, 32, 8), (4, 8192, 4, 1), (2, 4096, 32, 8), (1, 16384, 32, 8)]:
    q = torch.randn(B, S, H, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attn_func(q, k, v, causal=True)
    do = torch.randn_like(o)
    fl = 2.5 * 2.0 * B * H * S * S * 128
    res = {n: [] for n in variants}
    grads = {}
    for rnd in range(3):
        for name, (xm, ch) in variants.items():
            C.flash_attn_set_knob(3, xm)
            C.flash_attn_set_knob(1, ch)
            res[name].append(fl / timed(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)) / 1e9)
            if rnd == 0:
                grads[name] = [g.float() for g in torch.autograd.grad(o, (q, k, v), do, retain_graph=True)]
    C.flash_attn_set_knob(3, 2)
    C.flash_attn_set_knob(1, 0)
    ref = grads["contig_auto"]
    err = {n: max(((a - b).abs().max() / (b.abs().max() + 1e-6)).item() for a, b in zip(g, ref)) for n, g in grads.items()}
    print(json.dumps({"B": B, "S": S, "H": H, "Hkv": Hkv, **{f"{n}_tf": round(max(t), 1) for n, t in res.items()},
                      "max_rel_diff": {n: round(e, 5) for n, e in err.items()}}), flush=True)
