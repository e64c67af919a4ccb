"""Numerics of every hand-written HIP kernel against a plain PyTorch fp32 reference of the same op.

Runs only on an MI355X (marker `gpu`).  Each test also asserts that the native extension is the
code path in use (no silent fallback).
"""

import math

import pytest
import torch

import neuronx_distributed_llama3_2_amd.ops as ops
from neuronx_distributed_llama3_2_amd.ops import _ext

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


@pytest.fixture(autouse=True)
def _native():
    assert _ext.ext_available(), "HIP extension must be built for GPU tests"
    torch.manual_seed(0)
    yield


def _attn_inputs(B, Sq, Sk, Hq, Hkv, D, layout="bshd"):
    q = torch.randn(B, Sq, Hq, D, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(B, Sk, Hkv, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(B, Sk, Hkv, D, device=DEV, dtype=torch.bfloat16)
    return q, k, v


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S", [128, 333, 1024])
def test_flash_fwd(D, causal, S):
    B, Hq, Hkv = 2, 8, 2
    q, k, v = _attn_inputs(B, S, S, Hq, Hkv, D)
    o, lse = ops.flash_attn_fwd_lse(q, k, v, causal=causal)
    ro, rlse = ops.attention_reference(q, k, v, causal=causal)
    assert (o.float() - ro).abs().max().item() < 2e-2
    assert (lse - rlse).abs().max().item() < 1e-2


def test_flash_fwd_forced_rescale():
    # rule 26: force the online-softmax max to jump late in the key sweep
    B, S, Hq, Hkv, D = 1, 512, 4, 1, 128
    q, k, v = _attn_inputs(B, S, S, Hq, Hkv, D)
    k[:, 400] = q[:, 450, 0] * 4  # spike key 400 against query 450
    o, lse = ops.flash_attn_fwd_lse(q, k, v, causal=True)
    ro, rlse = ops.attention_reference(q, k, v, causal=True)
    assert (o.float() - ro).abs().max().item() < 3e-2
    assert (lse - rlse).abs().max().item() < 2e-2


def test_flash_fwd_cross_lengths():
    B, Sq, Sk, Hq, Hkv, D = 2, 100, 300, 8, 8, 64
    q, k, v = _attn_inputs(B, Sq, Sk, Hq, Hkv, D)
    o, lse = ops.flash_attn_fwd_lse(q, k, v, causal=True)  # bottom-right aligned
    ro, rlse = ops.attention_reference(q, k, v, causal=True)
    assert (o.float() - ro).abs().max().item() < 2e-2


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S", [128, 257, 1024])
def test_flash_bwd(D, causal, S):
    B, Hq, Hkv = 2, 8, 2
    q, k, v = _attn_inputs(B, S, S, Hq, Hkv, D)
    q.requires_grad_(True)
    k.requires_grad_(True)
    v.requires_grad_(True)
    o = ops.flash_attn_func(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ro, _ = ops.attention_reference(qf, kf, vf, causal=causal)
    ro.backward(do.float())
    assert _rel(q.grad, qf.grad) < 2e-2
    assert _rel(k.grad, kf.grad) < 2e-2
    assert _rel(v.grad, vf.grad) < 2e-2


def _bwd_check(B, Sq, Sk, Hq, Hkv, D, causal):
    q, k, v = _attn_inputs(B, Sq, Sk, Hq, Hkv, D)
    for t in (q, k, v):
        t.requires_grad_(True)
    o = ops.flash_attn_func(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ro, _ = ops.attention_reference(qf, kf, vf, causal=causal)
    ro.backward(do.float())
    assert _rel(q.grad, qf.grad) < 2e-2
    assert _rel(k.grad, kf.grad) < 2e-2
    assert _rel(v.grad, vf.grad) < 2e-2


@pytest.mark.parametrize("D", [64, 128])
def test_flash_bwd_chunked_items(D):
    # one kv head (TP=8 head count): each 256-key block's query sweep is cut into several work
    # items whose dK/dV partials meet in the fp32 atomics workspace
    _bwd_check(1, 4096, 4096, 4, 1, D, True)


@pytest.mark.parametrize("slab", [0, 1])
def test_flash_bwd_dkdv_slab_mode(slab):
    # dK/dV of the work items of one key block summed through per-item slabs (plain stores +
    # convert pass) instead of f32 atomics: same numerics, every shape class
    ext = ops.ext()
    ext.flash_attn_set_knob(5, slab)
    try:
        _bwd_check(1, 4096, 4096, 4, 1, 128, True)
        _bwd_check(1, 2048, 2048, 8, 2, 64, True)
        _bwd_check(2, 100, 300, 4, 2, 64, True)
        _bwd_check(1, 300, 100, 2, 2, 128, False)
        _bwd_check(2, 1024, 1024, 8, 2, 128, False)
    finally:
        ext.flash_attn_set_knob(5, -1)


def test_flash_bwd_cross_lengths():
    _bwd_check(2, 100, 300, 4, 2, 64, True)  # bottom-right aligned causal, Sk not a block multiple
    _bwd_check(1, 300, 100, 2, 2, 128, False)


def test_rope_attention_fused_qkv():
    S, B, nq, nkv, D = 256, 2, 8, 2, 128
    W = (nq + 2 * nkv) * D
    inv = ops.llama3_inv_freq(D, 500000.0, 8.0, 1.0, 4.0, 8192)
    cos_t, sin_t = ops.rope_tables(inv, 1024, device=DEV)
    qkv0 = torch.randn(S, B, W, device=DEV, dtype=torch.bfloat16)
    qkv = qkv0.clone().requires_grad_(True)
    o = ops.rope_attention(qkv.clone(), cos_t, sin_t, nq, nkv, D)
    # reference on the CPU path (plain torch ops)
    qr = qkv0.detach().cpu().float().requires_grad_(True)
    ro = ops.rope_attention(qr, cos_t.cpu(), sin_t.cpu(), nq, nkv, D)
    assert _rel(o.cpu(), ro) < 2e-2
    do = torch.randn_like(o)
    o.backward(do)
    ro.backward(do.cpu().float())
    assert _rel(qkv.grad.cpu(), qr.grad) < 3e-2


@pytest.mark.parametrize("H", [2048, 4096, 8192])
def test_rmsnorm(H):
    x = torch.randn(37, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(37, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    y, h = ops.rms_norm(x, w, 1e-5, residual=r)
    xf, rf, wf = (t.detach().float().requires_grad_(True) for t in (x, r, w))
    hf = xf + rf
    yf = ops.rms_norm_reference(hf, wf, 1e-5)
    assert _rel(y, yf) < 1e-2
    assert _rel(h, hf) < 1e-2
    dy = torch.randn_like(y)
    dh = torch.randn_like(h)
    (y.float() * dy.float()).sum().add((h.float() * dh.float()).sum()).backward()
    (yf * dy.float()).sum().add((hf * dh.float()).sum()).backward()
    assert _rel(x.grad, xf.grad) < 2e-2
    assert _rel(r.grad, rf.grad) < 2e-2
    assert _rel(w.grad, wf.grad) < 2e-2


@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_bwd_many_rows(with_res):
    """More rows than backward workgroups (512): every workgroup strides over several rows with the
    next row's loads in flight (rmsnorm.hip PIPE) -- dx, dres pass-through and dw against fp32."""
    T, H = 1537, 4096
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    y, h = ops.rms_norm(x, w, 1e-5, residual=r)
    xf, wf = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    rf = r.detach().float().requires_grad_(True) if with_res else None
    hf = xf + rf if with_res else xf
    yf = ops.rms_norm_reference(hf, wf, 1e-5)
    dy = torch.randn_like(y)
    loss = (y.float() * dy.float()).sum()
    loss_f = (yf * dy.float()).sum()
    if with_res:
        dh = torch.randn_like(h)
        loss = loss + (h.float() * dh.float()).sum()
        loss_f = loss_f + (hf * dh.float()).sum()
    loss.backward()
    loss_f.backward()
    assert _rel(x.grad, xf.grad) < 2e-2
    assert _rel(w.grad, wf.grad) < 2e-2
    if with_res:
        assert _rel(r.grad, rf.grad) < 2e-2


def test_rope_inplace():
    T, nh, D = 64, 6, 128
    W = nh * D + 256
    buf = torch.randn(T, W, device=DEV, dtype=torch.bfloat16)
    ref = buf.clone().cpu().float()
    inv = ops.llama3_inv_freq(D, 10000.0)
    c, s = ops.rope_tables(inv, 128, device=DEV)
    pos = torch.randint(0, 128, (T,), device=DEV)
    ops.rope_inplace_(buf, 0, nh, D, c, s, pos)
    x = ref[:, : nh * D].view(T, nh, D)
    out = ops.apply_rotary_reference(x, c.cpu(), s.cpu(), pos.cpu())
    assert _rel(buf[:, : nh * D].cpu().view(T, nh, D), out) < 1e-2
    assert torch.equal(buf[:, nh * D:].cpu().float(), ref[:, nh * D:])
    ops.rope_inplace_(buf, 0, nh, D, c, s, pos, sign=-1.0)
    assert _rel(buf[:, : nh * D].cpu(), ref[:, : nh * D]) < 2e-2


def test_swiglu():
    gu = torch.randn(65, 2 * 1792, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    h = ops.swiglu(gu)
    gf = gu.detach().float().requires_grad_(True)
    hf = ops.swiglu_reference(gf)
    assert _rel(h, hf) < 1e-2
    dh = torch.randn_like(h)
    h.backward(dh)
    hf.backward(dh.float())
    assert _rel(gu.grad, gf.grad) < 2e-2


@pytest.mark.parametrize("rows,I", [(128, 1792), (8192, 1792), (192, 448)])
def test_swiglu_bwd_dual_layout(rows, I):
    """Dual-layout SwiGLU backward: the row-major d(gate_up) matches the plain kernel bit for bit
    and vs fp32, and the second output is exactly its transpose."""
    C = _ext.ext()
    gu = torch.randn(rows, 2 * I, device=DEV, dtype=torch.bfloat16)
    dh = torch.randn(rows, I, device=DEV, dtype=torch.bfloat16)
    ref = torch.empty_like(gu)
    C.swiglu_bwd(gu, dh, ref)
    dgu = torch.empty_like(gu)
    dgu_t = torch.full((2 * I, rows), float("nan"), device=DEV, dtype=torch.bfloat16)
    C.swiglu_bwd_dual(gu, dh, dgu, dgu_t)
    torch.cuda.synchronize()
    assert torch.equal(dgu, ref)
    assert torch.equal(dgu_t, dgu.t())
    gf = gu.float().requires_grad_(True)
    ops.swiglu_reference(gf).backward(dh.float())
    assert _rel(dgu, gf.grad) < 2e-2


def test_swiglu_transposed_grad_reaches_gate_up_wgrad(monkeypatch):
    """The SwiGLU backward's token-contiguous d(gate_up) is what the gate_up weight gradient
    consumes (no separate transpose), with the same fp32 main_grad as the transposing path."""
    from neuronx_distributed_llama3_2_amd.ops import activations, gemm
    from neuronx_distributed_llama3_2_amd.parallel_layers import layers

    monkeypatch.setattr(gemm, "_WGRAD_T", "2")   # TN layout at this small size too
    seen = []
    orig = gemm.wgrad_accumulate_

    def spy(mg, go2, x2, go_t=None, x_t=None):
        seen.append(go_t is not None)
        return orig(mg, go2, x2, go_t=go_t, x_t=x_t)

    monkeypatch.setattr(gemm, "wgrad_accumulate_", spy)
    torch.manual_seed(0)
    T, H, I = 256, 512, 1024
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(2 * I, H, device=DEV)).to(torch.bfloat16)
    dh = torch.randn(T, I, device=DEV, dtype=torch.bfloat16)
    grads = []
    for dual in (True, False):
        monkeypatch.setattr(activations, "_DUAL", dual)
        wp = torch.nn.Parameter(w.clone())
        wp.main_grad = torch.zeros(2 * I, H, device=DEV, dtype=torch.float32)
        gu = layers.LinearWithAsyncCommunication.apply(x, wp, None, False, False, True, object())  # no TP group
        ops.swiglu(gu, token_major=True).backward(dh)
        grads.append(wp.main_grad.clone())
    assert seen == [True, False], seen
    assert torch.equal(grads[0], grads[1])


def test_swiglu_forward_token_major_copy_feeds_down_wgrad(monkeypatch):
    """SwiGLU forward under autograd writes h token-major; the down projection saves that copy
    instead of h and its weight gradient equals the transposing path's bit for bit."""
    from neuronx_distributed_llama3_2_amd.ops import activations, gemm
    from neuronx_distributed_llama3_2_amd.parallel_layers import layers

    monkeypatch.setattr(gemm, "_WGRAD_T", "2")
    C = _ext.ext()
    gu0 = torch.randn(2, 192, 2 * 448, device=DEV, dtype=torch.bfloat16)
    h_ref = torch.empty(2, 192, 448, device=DEV, dtype=torch.bfloat16)
    h_t = torch.empty(448, 384, device=DEV, dtype=torch.bfloat16)
    C.swiglu_fwd_dual(gu0, h_ref, h_t)
    torch.cuda.synchronize()
    assert torch.equal(h_t, h_ref.reshape(-1, 448).t())
    assert _rel(h_ref, ops.swiglu_reference(gu0.float())) < 1e-2
    seen = []
    orig = gemm.wgrad_accumulate_

    def spy(mg, go2, x2, go_t=None, x_t=None):
        seen.append((x2 is None, x_t is not None))
        return orig(mg, go2, x2, go_t=go_t, x_t=x_t)

    monkeypatch.setattr(gemm, "wgrad_accumulate_", spy)
    w = (0.05 * torch.randn(256, 448, device=DEV)).to(torch.bfloat16)
    dy = torch.randn(2, 192, 256, device=DEV, dtype=torch.bfloat16)
    grads, outs = [], []
    for dual in (True, False):
        monkeypatch.setattr(activations, "_DUAL_FWD", dual)
        gu = gu0.clone().requires_grad_(True)
        wp = torch.nn.Parameter(w.clone())
        wp.main_grad = torch.zeros(256, 448, device=DEV, dtype=torch.float32)
        h = ops.swiglu(gu, token_major=True)
        assert hasattr(h, "_nxd_t") == dual
        y = layers.LinearWithAsyncCommunication.apply(h, wp, None, False, False, True, object())
        y.backward(dy)
        outs.append((y.detach().clone(), gu.grad.clone()))
        grads.append(wp.main_grad.clone())
    assert seen == [(True, True), (False, False)], seen
    assert torch.equal(grads[0], grads[1])
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("smooth", [0.0, 0.1])
def test_cross_entropy(dtype, smooth):
    N, V = 77, 16032
    logits = (3 * torch.randn(N, V, device=DEV)).to(dtype).requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[5] = -100
    loss = ops.vocab_parallel_cross_entropy(logits, labels, label_smoothing=smooth)
    lf = logits.detach().float().requires_grad_(True)
    rl = ops.parallel_cross_entropy_reference(lf, labels, label_smoothing=smooth)
    assert (loss - rl).abs().max().item() < 1e-3 * max(1.0, rl.abs().max().item())
    g = torch.rand(N, device=DEV)
    loss.backward(g)
    rl.backward(g)
    assert _rel(logits.grad, lf.grad) < 2e-2


def test_embedding():
    V, H, T = 1000, 512, 300
    w = torch.randn(V, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    ids = torch.randint(0, 2 * V, (3, T // 3), device=DEV)
    out = ops.vocab_parallel_embedding(ids, w, vocab_start=V // 2)
    local = ids - V // 2
    mask = (local >= 0) & (local < V)
    ref = w.detach()[local.clamp(0, V - 1)] * mask[..., None]
    assert torch.equal(out, ref)
    d = torch.randn_like(out)
    out.backward(d)
    refg = torch.zeros(V, H, device=DEV)
    refg.index_add_(0, local.clamp(0, V - 1).view(-1), (d.float() * mask[..., None]).view(-1, H))
    assert _rel(w.grad, refg) < 1e-2


def test_flat_reduce_and_adamw():
    n = 1_000_003
    g = torch.randn(n, device=DEV, dtype=torch.bfloat16)
    s = ops.flat_sumsq(g)
    assert abs(s.item() - g.float().pow(2).sum().item()) / s.item() < 1e-4
    mx = ops.flat_absmax(g)
    assert mx.item() == g.float().abs().max().item()
    p = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    p16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    pr, mr, vr = p.clone().cpu(), m.clone().cpu(), v.clone().cpu()
    coef = ops.clip_coefficient(s, 1.0)
    for step in (1, 2):
        ops.adamw_flat_(p, g, m, v, p16, 1e-3, 0.9, 0.95, 1e-8, 0.1, step, grad_scale=coef)
        ops.adamw_flat_(pr, g.cpu(), mr, vr, None, 1e-3, 0.9, 0.95, 1e-8, 0.1, step, grad_scale=coef.cpu())
    assert _rel(p.cpu(), pr) < 1e-5
    assert torch.equal(p16.cpu(), p.cpu().to(torch.bfloat16))


@pytest.mark.parametrize("D", [64, 128])
def test_decode_attention_and_cache(D):
    B, Hq, Hkv, L, T = 3, 32, 8, 700, 2
    kc = torch.zeros(B, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc[:, :, :600] = torch.randn(B, Hkv, 600, D, device=DEV, dtype=torch.bfloat16)
    vc[:, :, :600] = torch.randn(B, Hkv, 600, D, device=DEV, dtype=torch.bfloat16)
    knew = torch.randn(B, T, Hkv, D, device=DEV, dtype=torch.bfloat16)
    vnew = torch.randn(B, T, Hkv, D, device=DEV, dtype=torch.bfloat16)
    pos = torch.tensor([100, 333, 598], device=DEV, dtype=torch.int32)
    ops.kv_cache_write(knew, vnew, kc, vc, pos)
    for b in range(B):
        assert torch.equal(kc[b, :, pos[b]:pos[b] + T], knew[b].transpose(0, 1))
    q = torch.randn(B, T, Hq, D, device=DEV, dtype=torch.bfloat16)
    seq = pos + T
    o = ops.decode_attention(q, kc, vc, seq)
    kc_c, vc_c = kc.cpu(), vc.cpu()
    ro = ops.decode_attention(q.cpu(), kc_c, vc_c, seq.cpu())
    assert _rel(o.cpu(), ro) < 2e-2


def test_sampling():
    B, V = 4, 128256
    x = torch.randn(B, V, device=DEV)
    assert torch.equal(ops.argmax_rows(x), torch.argmax(x, -1))
    u = torch.rand(B, device=DEV)
    tok, vals, idx = ops.topk_sample(x, 50, 1.0, u, return_topk=True)
    rv, ri = torch.topk(x, 50, -1)
    assert torch.allclose(vals, rv)
    assert torch.equal(idx, ri)
    rt = ops.topk_sample(x.cpu(), 50, 1.0, u.cpu())
    assert torch.equal(tok.cpu(), rt)


@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (1, 1000, 512), (8192, 1024, 4096)])
def test_tuned_gemm_variants(M, N, K):
    from neuronx_distributed_llama3_2_amd.ops import gemm

    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    ref = x.float() @ w.float().t()
    y = gemm.linear(x, w)
    torch.testing.assert_close(y.float(), ref, atol=2e-2 * ref.abs().max().item(), rtol=2e-2)
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    dx = gemm.matmul(g, w)
    torch.testing.assert_close(dx.float(), g.float() @ w.float(), atol=2e-2 * (g.float() @ w.float()).abs().max().item(),
                               rtol=2e-2)
    mg = torch.randn(N, K, device="cuda", dtype=torch.float32)
    exp = mg + g.float().t() @ x.float()
    gemm.wgrad_accumulate_(mg, g, x)
    torch.testing.assert_close(mg, exp, atol=1e-3 * exp.abs().max().item(), rtol=1e-3)


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("wtype", ["bf16", "int8_tensor", "int8_channel"])
@pytest.mark.parametrize("glu", [False, True])
def test_gemv_skinny(M, wtype, glu):
    from neuronx_distributed_llama3_2_amd.ops.gemv import dequantize_weight, skinny_linear
    from neuronx_distributed_llama3_2_amd.quantization import quantize_symmetric

    torch.manual_seed(M)
    K, N = 2048, 1536
    Nw = 2 * N if glu else N
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    wf = torch.randn(Nw, K, device="cuda") * 0.02
    bias = torch.randn(Nw, device="cuda", dtype=torch.bfloat16) * 0.1
    if wtype == "bf16":
        w, s = wf.to(torch.bfloat16), None
        wref = w.float()
    else:
        w, s = quantize_symmetric(wf, 0 if wtype == "int8_channel" else None)
        wref = w.float() * s.reshape(-1, 1) if s.numel() > 1 else w.float() * s
        torch.testing.assert_close(dequantize_weight(w, s).float(), wref, atol=1e-2, rtol=1e-2)
    ref = x.float() @ wref.t() + bias.float()
    if glu:
        g, u = ref.chunk(2, dim=-1)
        ref = torch.nn.functional.silu(g) * u
    y = skinny_linear(x, w, s, bias, glu=glu)
    assert y.shape == (M, N)
    torch.testing.assert_close(y.float(), ref, atol=2e-2 * ref.abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("D,Hq,Hkv,T,L", [(64, 32, 8, 1, 20000), (128, 64, 8, 8, 3000), (128, 32, 8, 1, 130)])
def test_decode_attention_long_and_repeated(D, Hq, Hkv, T, L):
    """many splits (>64: LDS split-weight table), M = 64 rows, and back-to-back calls (counter reset)."""
    B = 2
    torch.manual_seed(1)
    kc = torch.randn(B, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(B, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    seq = torch.tensor([L - 5, L // 3], device=DEV, dtype=torch.int32)
    kc_c, vc_c = kc.cpu(), vc.cpu()
    for it in range(3):
        q = torch.randn(B, T, Hq, D, device=DEV, dtype=torch.bfloat16)
        o = ops.decode_attention(q, kc, vc, seq)
        ro = ops.decode_attention(q.cpu(), kc_c, vc_c, seq.cpu())
        assert _rel(o.cpu(), ro) < 2e-2, it


def test_argmax_large_vocab():
    x = torch.randn(3, 128256, device=DEV).to(torch.bfloat16)
    x[1, 77777] = 50.0
    x[2, 5] = x[2, 128255] = 60.0  # tie -> smallest index
    a = ops.argmax_rows(x)
    assert a.tolist() == [int(x[0].float().argmax()), 77777, 5]


@pytest.mark.parametrize("tr", [True, False])
@pytest.mark.parametrize("R,C", [(64, 64), (8, 8), (8192, 4096), (1000, 72), (72, 1000), (4096, 14336), (136, 8200)])
def test_transpose_bf16(R, C, tr):
    """Both transpose kernels (csrc/transpose.hip: ds_read_b64_tr_b16 tile, and the 16-bit LDS one)
    bit-exact against torch, with partial edge tiles and a source row stride wider than C."""
    from neuronx_distributed_llama3_2_amd import _C
    from neuronx_distributed_llama3_2_amd.ops import gemm

    _C.transpose_set_variant(tr)
    try:
        x = torch.randn(R, C + 8, device=DEV, dtype=torch.bfloat16)[:, :C]   # row stride C + 8
        y = gemm.transpose(x)
        assert torch.equal(y, x.t().contiguous())
        x2 = torch.randn(R, C, device=DEV, dtype=torch.bfloat16)
        assert torch.equal(gemm.transpose(x2), x2.t().contiguous())
    finally:
        _C.transpose_set_variant(True)


def test_dgrad_kmajor_weight_refreshes():
    """dX = dY W through the cached K-major weight copy; stale copies are refreshed after an
    optimizer-kernel update (epoch), an in-place torch write (version) and a .data swap."""
    from neuronx_distributed_llama3_2_amd.ops import gemm

    w = torch.nn.Parameter(torch.randn(768, 512, device=DEV, dtype=torch.bfloat16))
    g = torch.randn(256, 768, device=DEV, dtype=torch.bfloat16)
    ref = lambda: (g.float() @ w.detach().float())
    assert _rel(gemm.dgrad(g, w), ref()) < 1e-2
    # optimizer kernel writes the bf16 weights behind autograd
    p32 = w.detach().float().reshape(-1).clone()
    grad = torch.randn_like(p32)
    ops.adamw_flat_(p32, grad, torch.zeros_like(p32), torch.zeros_like(p32), w.data.view(-1), 1e-1, 0.9, 0.95, 1e-8,
                    0.0, 1)
    assert _rel(gemm.dgrad(g, w), ref()) < 1e-2
    with torch.no_grad():
        w.mul_(-1.0)   # in-place torch write: version counter
    assert _rel(gemm.dgrad(g, w), ref()) < 1e-2
    w.data = torch.randn_like(w.data)   # new storage
    assert _rel(gemm.dgrad(g, w), ref()) < 1e-2


@pytest.mark.parametrize("mode", ["0", "2"])
def test_wgrad_accumulate_layouts(mode, monkeypatch):
    """fp32 main_grad += dY^T X through the NT GEMM (mode 0) and the transposed-operand TN GEMM
    (mode 2) against an fp32 reference, accumulating over two micro-batches."""
    from neuronx_distributed_llama3_2_amd.ops import gemm

    monkeypatch.setattr(gemm, "_WGRAD_T", mode)
    T, N, K = 512, 768, 256
    mg = torch.zeros(N, K, device=DEV, dtype=torch.float32)
    ref = torch.zeros(N, K, device=DEV, dtype=torch.float32)
    for _ in range(2):
        go = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
        x = torch.randn(T, K, device=DEV, dtype=torch.bfloat16)
        gemm.wgrad_accumulate_(mg, go, x)
        ref += go.float().t() @ x.float()
    assert _rel(mg, ref) < 1e-3


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("Hq,Hkv,T", [(32, 8, 1), (8, 1, 2), (64, 8, 2), (16, 2, 1)])
@pytest.mark.parametrize("L", [384, 1024, 5000])
def test_decode_attention_mfma_groups(D, Hq, Hkv, T, L):
    """MFMA flash-decoding kernel (decode_attn.hip, M = Hq/Hkv * T <= 16): one split up to 1024 keys,
    split + merge beyond; ragged lengths incl. a single visible key and chunk-boundary lengths."""
    B = 4
    torch.manual_seed(2)
    kc = torch.randn(B, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(B, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    seq = torch.tensor([L, max(T, 1), min(L, 64 + T), max(T, L // 2 + 17)], device=DEV, dtype=torch.int32)
    q = torch.randn(B, T, Hq, D, device=DEV, dtype=torch.bfloat16) * 2
    o = ops.decode_attention(q, kc, vc, seq)
    ro = ops.decode_attention(q.cpu(), kc.cpu(), vc.cpu(), seq.cpu())
    assert torch.isfinite(o.float()).all()
    assert _rel(o.cpu(), ro) < 2e-2
    # cache rows through cache_idx (continuous batching)
    idx = torch.tensor([3, 0, 2, 1], device=DEV, dtype=torch.int32)
    o2 = ops.decode_attention(q, kc, vc, seq, idx)
    ro2 = ops.decode_attention(q.cpu(), kc.cpu(), vc.cpu(), seq.cpu(), idx.cpu())
    assert _rel(o2.cpu(), ro2) < 2e-2


def test_adamw_stochastic_rounding_matches_reference():
    """bf16 copy-out with stochastic rounding: kernel bit-identical to the CPU emulation, unbiased."""
    n = 1 << 20
    p = (1.0 + torch.rand(n, device=DEV) * 2 ** -6)
    g = torch.randn(n, device=DEV) * 1e-3
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    p16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    pc, gc, mc, vc = p.cpu().clone(), g.cpu(), m.cpu().clone(), v.cpu().clone()
    p16c = torch.empty(n, dtype=torch.bfloat16)
    ops.adamw_flat_(p, g, m, v, p16, 1e-3, 0.9, 0.95, 1e-8, 0.01, 1, sr_seed=987654321)
    ops.adamw_flat_(pc, gc, mc, vc, p16c, 1e-3, 0.9, 0.95, 1e-8, 0.01, 1, sr_seed=987654321)
    assert torch.allclose(p.cpu(), pc, rtol=0, atol=1e-6)
    # the kernel's bf16 copy-out == the emulation applied to the kernel's own fp32 masters, bit for bit
    assert torch.equal(p16.cpu(), ops.stochastic_round_bf16(p.cpu(), 987654321))
    # unbiased: masters 1/8 bf16-ulp above 1.0 (tiny lr keeps them there) round to nearest as 1.0
    # (bias -1/8 ulp = -9.8e-4) but stochastically to 1.0 / 1.0078 with mean error ~0
    q = torch.full((n,), 1.0 + 2 ** -10, device=DEV)
    q16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ops.adamw_flat_(q, torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), q16,
                    1e-12, 0.9, 0.95, 1e-8, 0.0, 1, sr_seed=12345)
    err = (q16.float() - q).mean().item()
    assert abs(err) < 1e-4, err


@pytest.mark.parametrize("H", [512, 1536, 3072, 4096, 6144, 8192])
@pytest.mark.parametrize("T", [1, 9, 2049, 5003])
def test_rmsnorm_rows_path_vs_fp32(H, T):
    """Row-per-wave RMSNorm kernels (H % 512 == 0, H <= 8192 -- two waves per row above 4096, the 70B
    width; csrc/rmsnorm.hip fwd_rows / bwd_rows /
    colsum4): rows below and above the grid's 8 x 256 rows per round (grid-stride), residual fused,
    dw accumulated into a nonzero fp32 main_grad -- against fp32 torch, and against the one-row-per-
    workgroup kernels."""
    from neuronx_distributed_llama3_2_amd import _C

    g = torch.Generator(device=DEV).manual_seed(T * 7 + H)
    x, r, dy, dres = (torch.randn(T, H, device=DEV, generator=g).to(torch.bfloat16) for _ in range(4))
    w = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(torch.bfloat16)
    mg0 = torch.randn(H, device=DEV, generator=g)
    outs = {}
    try:
        for path in (True, False):
            _C.rmsnorm_set_rows_path(path)
            y, h, rstd = torch.empty_like(x), torch.empty_like(x), torch.empty(T, device=DEV)
            _C.rmsnorm_fwd(x, r, w, y, h, rstd, 1e-5)
            dx, mg = torch.empty_like(x), mg0.clone()
            _C.rmsnorm_bwd(dy, h, w, rstd, dres, dx, mg, True)
            outs[path] = (y, h, rstd, dx, mg)
    finally:
        _C.rmsnorm_set_rows_path(True)
    y, h, rstd, dx, mg = outs[True]
    hf = h.float().requires_grad_(True)   # the stored (bf16-rounded) h is what the backward reads
    wf = w.float().requires_grad_(True)
    yf = ops.rms_norm_reference(hf, wf, 1e-5)
    yf.backward(dy.float())
    assert torch.equal(h, (x.float() + r.float()).to(torch.bfloat16))
    assert _rel(y, yf) < 1e-2
    assert _rel(rstd, torch.rsqrt(h.float().pow(2).mean(-1) + 1e-5)) < 1e-5
    assert _rel(dx, hf.grad + dres.float()) < 2e-2
    assert _rel(mg - mg0, wf.grad) < 1e-3
    for a, b in zip(outs[True], outs[False]):
        assert _rel(a, b) < 1e-2


@pytest.mark.parametrize("M", [1, 2, 4, 8])
@pytest.mark.parametrize("N,K", [(2048, 2048), (4096, 8192), (1000, 520)])
@pytest.mark.parametrize("path", ["fma", "dot2", "mfma", "mfma_split"])
def test_dgemv_plain_matches_fp32(M, N, K, path):
    """Decode GEMV y = x W^T (PLAIN epilogue, with and without the RMSNorm prologue) on every body:
    VALU with widened FMAs / v_dot2c_f32_bf16, and the MFMA tiles of 2-8 rows (K split inside the
    workgroup, or also over workgroups), against fp32."""
    C = _ext.ext()
    C.decode_set_knob(7, 2 if path.startswith("mfma") else 0)
    C.decode_set_knob(8, 1 if path == "mfma_split" else 0)
    dot2 = 0 if path == "fma" else 1
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
    try:
        C.decode_set_knob(6, dot2)
        y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        C.dgemv(0, x, None, 0.0, w, y, 0, 0, 0, None, None, None, 1, None, None, None)
        ref = x.float() @ w.float().t()
        assert _rel(y, ref) < 1e-2
        # split-K launches sum their parts in a fixed order: a repeat is bit-identical
        y2 = torch.empty_like(y)
        C.dgemv(0, x, None, 0.0, w, y2, 0, 0, 0, None, None, None, 1, None, None, None)
        assert torch.equal(y, y2)
        if M * K > 32768:   # the RMSNorm prologue holds the normalised rows in 64 KiB of LDS
            return
        yn = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        C.dgemv(0, x, nw, 1e-5, w, yn, 0, 0, 0, None, None, None, 1, None, None, None)
        xf = x.float()
        h = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)).to(torch.bfloat16).float() * nw.float()
        assert _rel(yn, h.to(torch.bfloat16).float() @ w.float().t()) < 1e-2
    finally:
        C.decode_set_knob(6, 1)
        C.decode_set_knob(7, 4)
        C.decode_set_knob(8, 0)
