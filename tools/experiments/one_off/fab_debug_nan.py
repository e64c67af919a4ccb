"""FA backward numerics probe: per-tensor relative error / NaN count vs fp32 for small shapes."""
import sys

import torch

sys.path.insert(0, ".")
import neuronx_distributed_llama3_2_amd.ops as ops  # noqa: E402

C = ops.ext()
for pv in (12, 0):
    C.flash_attn_set_knob(4, pv)
    for D in (64, 128):
        for S in (128, 1024):
            for causal in (True, False):
                torch.manual_seed(0)
                B, Hq, Hkv = 2, 8, 2
                q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
                k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
                v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
                o = ops.flash_attn_func(q, k, v, causal=causal)
                do = torch.randn_like(o)
                g = torch.autograd.grad(o, (q, k, v), do)
                qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
                ro, _ = ops.attention_reference(qf, kf, vf, causal=causal)
                rg = torch.autograd.grad(ro, (qf, kf, vf), do.float())
                out = []
                for name, a, b in zip("qkv", g, rg):
                    a = a.float()
                    nan = int(torch.isnan(a).sum())
                    err = ((a - b).abs().max() / b.abs().max()).item() if nan == 0 else float("nan")
                    bad_rows = ""
                    if nan:
                        idx = torch.isnan(a).nonzero()[:3].tolist()
                        bad_rows = f" first_nan={idx}"
                    out.append(f"d{name}: nan={nan} rel={err:.4f}{bad_rows}")
                print(f"pipe={pv} D={D} S={S} causal={causal} | " + " | ".join(out), flush=True)
C.flash_attn_set_knob(4, 12)
