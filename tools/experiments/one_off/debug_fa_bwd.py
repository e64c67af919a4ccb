import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import neuronx_distributed_llama3_2_amd.ops as ops


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-9)).item()


torch.manual_seed(0)
for (B, S, Hq, Hkv, D, causal) in [(1, 32, 1, 1, 128, False), (1, 128, 1, 1, 128, False), (1, 128, 1, 1, 64, False),
                                   (1, 256, 2, 1, 128, True), (2, 257, 8, 2, 128, True)]:
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attn_func(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ro, _ = ops.attention_reference(qf, kf, vf, causal=causal)
    ro.backward(do.float())
    print(B, S, Hq, Hkv, D, causal, "dq", rel(q.grad, qf.grad), "dk", rel(k.grad, kf.grad), "dv", rel(v.grad, vf.grad))
    if S == 32:
        print("dq ratio sample", (q.grad.float() / qf.grad)[0, :4, 0, :6])
        print("dq ours", q.grad[0, :3, 0, :6])
        print("dq ref ", qf.grad[0, :3, 0, :6])
