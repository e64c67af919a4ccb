"""A/B of the FA backward software-pipeline depth variants (knob 4: 12 = S/dP reads 1 step ahead +
dV/dK reads 2 steps ahead (default), 11, 21, 0 = no prefetch), interleaved rounds in one process;
gradients compared against a chunked fp32 reference."""
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


def ref_grads(q, k, v, do):
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    g = q.shape[2] // k.shape[2]
    ke, ve = kf.repeat_interleave(g, 2), vf.repeat_interleave(g, 2)
    o = torch.nn.functional.scaled_dot_product_attention(qf.transpose(1, 2), ke.transpose(1, 2), ve.transpose(1, 2),
                                                         is_causal=True).transpose(1, 2)
    return torch.autograd.grad(o, (qf, kf, vf), do.float())


C = ops.ext()
variants = {"p12": 12, "p11": 11, "p21": 21, "p0": 0}
for (B, S, H, Hkv) in [(1, 8192, 32, 8), (4, 8192, 4, 1), (2, 4096, 32, 8)]:
    torch.manual_seed(0)
    q = torch.randn(B, S, H, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attn_func(q, k, v, causal=True)
    do = torch.randn_like(o)
    fl = 2.5 * 2.0 * B * H * S * S * 128
    res = {n: [] for n in variants}
    grads = {}
    for rnd in range(3):
        for name, pv in variants.items():
            C.flash_attn_set_knob(4, pv)
            res[name].append(fl / timed(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)) / 1e9)
            if rnd == 0:
                grads[name] = [gr.float() for gr in torch.autograd.grad(o, (q, k, v), do, retain_graph=True)]
    C.flash_attn_set_knob(4, 12)
    err = {}
    if S * B <= 8192:
        ref = ref_grads(q, k, v, do)
        err = {n: max(((a - b).abs().max() / (b.abs().max() + 1e-6)).item() for a, b in zip(g, ref)) for n, g in grads.items()}
        del ref
    same = {n: max((a - b).abs().max().item() for a, b in zip(g, grads["p0"])) for n, g in grads.items()}
    print(json.dumps({"B": B, "S": S, "H": H, "Hkv": Hkv, **{f"{n}_tf": round(max(t), 1) for n, t in res.items()},
                      "max_rel_err_vs_fp32": {n: round(e, 5) for n, e in err.items()},
                      "max_abs_diff_vs_p0": {n: round(e, 5) for n, e in same.items()}}), flush=True)
