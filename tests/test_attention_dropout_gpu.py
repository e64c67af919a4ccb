"""In-kernel attention dropout of the CDNA4 flash kernels (csrc/flash_attn_{fwd,bwd}.hip DROP
variants; reference: NKI flash_fwd / flash_attn_bwd dropout_p + seed, kernels/flash_attn.py:85-148)
against the fp32 host path of ops/attention_dropout.py with the same hashed keep mask: output and
dQ / dK / dV, GQA, causal with Sq != Sk, D = 64 / 128, TP head offsets."""

import pytest
import torch

from neuronx_distributed_llama3_2_amd.ops import attention_dropout as AD
from neuronx_distributed_llama3_2_amd.ops._ext import ext

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.detach().float() - b.detach().float()).norm() / b.detach().float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("B,Hq,Hkv,Sq,Sk,D,causal,hoff", [
    (2, 8, 2, 300, 300, 128, True, 0),
    (1, 4, 4, 256, 384, 128, True, 4),      # bottom-right causal alignment, head offset
    (2, 4, 1, 200, 200, 64, False, 0),
    (1, 16, 2, 1024, 1024, 128, True, 0),   # 8-wave forward variant
])
def test_kernel_dropout_matches_host_path(B, Hq, Hkv, Sq, Sk, D, causal, hoff):
    assert ext() is not None
    torch.manual_seed(0)
    p, seed = 0.2, 987654
    q = torch.randn(B, Hq, Sq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, Sk, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, Sk, D, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(B, Hq, Sq, D, device="cuda", dtype=torch.bfloat16)
    qk, kk, vk = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = AD.attention_with_dropout(qk, kk, vk, p, causal=causal, seed=seed, head_offset=hoff)   # HIP kernels
    o.backward(g)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    orf = AD.DropoutAttentionFunc.apply(qr, kr, vr, causal, D ** -0.5, p, seed, hoff)        # fp32 host path
    orf.backward(g.float())
    assert _rel(o, orf) < 1.5e-2, _rel(o, orf)
    for a, b, n in ((qk.grad, qr.grad, "dq"), (kk.grad, kr.grad, "dk"), (vk.grad, vr.grad, "dv")):
        assert _rel(a, b) < 2.5e-2, (n, _rel(a, b))
    # the mask is really applied: the undropped kernel output differs by ~sqrt(p/(1-p))
    qn, kn, vn = (t.transpose(1, 2) for t in (q, k, v))
    from neuronx_distributed_llama3_2_amd.ops.flash_attn import flash_attn_func

    o0 = flash_attn_func(qn, kn, vn, causal=causal).transpose(1, 2)
    assert _rel(o, o0) > 0.1


def test_dropout_zero_is_the_plain_kernel_and_masks_are_seeded():
    torch.manual_seed(1)
    q = torch.randn(1, 512, 8, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, 512, 2, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, 512, 2, 128, device="cuda", dtype=torch.bfloat16)
    from neuronx_distributed_llama3_2_amd.ops.flash_attn import flash_attn_func

    a = flash_attn_func(q, k, v, dropout_p=0.1, seed=3)
    b = flash_attn_func(q, k, v, dropout_p=0.1, seed=3)
    c = flash_attn_func(q, k, v, dropout_p=0.1, seed=4)
    assert torch.equal(a, b) and not torch.equal(a, c)
