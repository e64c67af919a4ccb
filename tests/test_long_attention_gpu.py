"""Flash attention at the bench's shapes and beyond, against a chunked fp32 reference.

S = 8192 at the TP=1 head counts (Hq 32 / Hkv 8: the grid is >= 512 workgroups, so the default
8-wave forward runs) and the TP=8 per-rank head counts (Hq 4 / Hkv 1, B = 2 as the TP=8 bench
micro-batch), plus S = 16384 and 32768 (long-context configurations of the reference's only
published numbers, test/integration/llama2_7B/test_long_seqlen.py).  The reference is exact
fp32 attention evaluated one query block at a time (memory O(block x S) per head).
"""

import math

import pytest
import torch

import neuronx_distributed_llama3_2_amd.ops as ops
from neuronx_distributed_llama3_2_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _chunked_reference(q, k, v, do, blk=1024):
    """fp32 causal attention fwd + bwd, q block by q block.  q/do: [B, S, Hq, D], k/v: [B, S, Hkv, D]."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    g = Hq // Hkv
    scale = 1.0 / math.sqrt(D)
    qf = q.float().permute(0, 2, 1, 3)                                   # [B, Hq, S, D]
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)     # [B, Hq, S, D]
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(g, dim=1)
    dof = do.float().permute(0, 2, 1, 3)
    o = torch.empty_like(qf)
    lse = torch.empty(B, Hq, S, device=q.device)
    dq = torch.empty_like(qf)
    dk = torch.zeros_like(kf)
    dv = torch.zeros_like(vf)
    kpos = torch.arange(S, device=q.device)
    for s0 in range(0, S, blk):
        s1 = min(S, s0 + blk)
        qb = qf[:, :, s0:s1]
        sc = torch.matmul(qb, kf.transpose(-1, -2)) * scale            # [B, Hq, blk, S]
        mask = kpos[None, :] > torch.arange(s0, s1, device=q.device)[:, None]
        sc.masked_fill_(mask, float("-inf"))
        l = torch.logsumexp(sc, dim=-1)
        p = torch.exp(sc - l[..., None])
        ob = torch.matmul(p, vf)
        o[:, :, s0:s1] = ob
        lse[:, :, s0:s1] = l
        dob = dof[:, :, s0:s1]
        dv += torch.matmul(p.transpose(-1, -2), dob)
        dp = torch.matmul(dob, vf.transpose(-1, -2))
        delta = (dob * ob).sum(-1, keepdim=True)
        ds = p * (dp - delta) * scale
        dq[:, :, s0:s1] = torch.matmul(ds, kf)
        dk += torch.matmul(ds.transpose(-1, -2), qb)
        del sc, p, dp, ds
    dk = dk.view(B, Hkv, g, S, D).sum(2)
    dv = dv.view(B, Hkv, g, S, D).sum(2)
    back = lambda t: t.permute(0, 2, 1, 3)
    return back(o), lse, back(dq), back(dk), back(dv)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.mark.parametrize("B,S,Hq,Hkv", [(1, 8192, 32, 8), (2, 8192, 4, 1), (1, 16384, 4, 1), (1, 32768, 4, 1)])
def test_flash_attention_long_vs_fp32(B, S, Hq, Hkv):
    assert _ext.ext_available()
    torch.manual_seed(0)
    D = 128
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    for t in (q, k, v):
        t.requires_grad_(True)
    o = ops.flash_attn_func(q, k, v, causal=True)
    o.backward(do)
    _, lse = ops.flash_attn_fwd_lse(q.detach(), k.detach(), v.detach(), causal=True)
    ro, rlse, rdq, rdk, rdv = _chunked_reference(q.detach(), k.detach(), v.detach(), do)
    assert (o.float() - ro).abs().max().item() < 2e-2
    assert (lse - rlse).abs().max().item() < 1e-2
    assert _rel(q.grad, rdq) < 2e-2
    assert _rel(k.grad, rdk) < 2e-2
    assert _rel(v.grad, rdv) < 2e-2
