"""Attention with dropout (reference NKI flash kernels' dropout_p + seed): chunked flash path vs a
naive softmax with the same hashed keep mask, forward and gradients, GQA, causal offset."""

import torch

from neuronx_distributed_llama3_2_amd.kernels.flash_attn import flash_attn_func
from neuronx_distributed_llama3_2_amd.ops import attention_dropout as AD


def _naive(q, k, v, p, seed, causal, scale):
    B, H, Sq, D = q.shape
    ke = k.repeat_interleave(H // k.shape[1], 1)
    ve = v.repeat_interleave(H // v.shape[1], 1)
    s = q @ ke.transpose(-1, -2) * scale
    Sk = ke.shape[2]
    if causal:
        m = torch.arange(Sk)[None, :] > (torch.arange(Sq)[:, None] + Sk - Sq)
        s = s.masked_fill(m, float("-inf"))
    pr = torch.softmax(s, -1)
    keep = AD.dropout_keep_mask(seed, B, H, torch.arange(Sq), Sk, p)
    return (pr * keep / (1 - p)) @ ve


def test_dropout_attention_matches_naive_fwd_bwd(monkeypatch):
    monkeypatch.setattr(AD, "Q_CHUNK", 16)        # several query chunks
    torch.manual_seed(0)
    B, Hq, Hkv, S, D = 2, 4, 2, 40, 16
    q = torch.randn(B, Hq, S, D, dtype=torch.float64, requires_grad=True)
    k = torch.randn(B, Hkv, S, D, dtype=torch.float64, requires_grad=True)
    v = torch.randn(B, Hkv, S, D, dtype=torch.float64, requires_grad=True)
    for causal in (True, False):
        o = AD.attention_with_dropout(q, k, v, 0.3, causal=causal, seed=1234)
        r = _naive(q, k, v, 0.3, 1234, causal, D ** -0.5)
        torch.testing.assert_close(o, r.to(o.dtype), atol=1e-5, rtol=1e-5)
        g = torch.randn_like(o)
        gq, gk, gv = torch.autograd.grad(o, (q, k, v), g)
        rq, rk, rv = torch.autograd.grad(r, (q, k, v), g)
        torch.testing.assert_close(gq, rq, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(gk, rk, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(gv, rv, atol=1e-5, rtol=1e-5)


def test_dropout_rate_and_api_layouts():
    keep = AD.dropout_keep_mask(7, 1, 2, torch.arange(256), 256, 0.25)
    assert abs(keep.float().mean().item() - 0.75) < 0.01
    # head_offset: a TP rank's local heads draw the global heads' masks
    full = AD.dropout_keep_mask(7, 1, 4, torch.arange(8), 8, 0.25)
    part = AD.dropout_keep_mask(7, 1, 2, torch.arange(8), 8, 0.25, head_offset=2)
    assert torch.equal(full[:, 2:], part)
    torch.manual_seed(1)
    q = torch.randn(1, 8, 2, 16)
    k = torch.randn(1, 8, 2, 16)
    v = torch.randn(1, 8, 2, 16)
    a = flash_attn_func(q, k, v, layout="bshd", dropout_p=0.1, seed=5)
    b = flash_attn_func(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), layout="bhsd", dropout_p=0.1, seed=5)
    torch.testing.assert_close(a, b.transpose(1, 2))
    z = flash_attn_func(q, k, v, layout="bshd", dropout_p=0.0)
    assert not torch.allclose(a, z)
