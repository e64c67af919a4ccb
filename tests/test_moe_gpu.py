"""MoE on the MI355X: grouped-GEMM HIP kernels (forward, input grad, fp32 weight grad) against an
fp32 PyTorch reference on ragged / empty expert groups, and a dropless MoE layer's forward +
backward running with no device->host synchronisation."""

import os

import pytest
import torch

import neuronx_distributed_llama3_2_amd.ops as ops
from neuronx_distributed_llama3_2_amd.ops import _ext
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _native():
    assert _ext.ext_available(), "HIP extension must be built for GPU tests"
    torch.manual_seed(0)
    yield


def _offs(counts):
    o = [0]
    for c in counts:
        o.append(o[-1] + c)
    return torch.tensor(o, dtype=torch.int32, device=DEV)


def _ref_fwd(x, w, offs):
    b = offs.tolist()
    y = torch.zeros(x.shape[0], w.shape[2], device=DEV)
    for e in range(w.shape[0]):
        y[b[e]:b[e + 1]] = x[b[e]:b[e + 1]].float() @ w[e].float()
    return y


@pytest.mark.parametrize("counts,K,N", [
    ([300, 0, 17, 128, 1, 555, 0, 40], 256, 384),     # ragged + empty groups, 128-aligned dims
    ([64, 200, 0, 3], 264, 392),                       # k / n tails (multiples of 8 only)
    ([0, 0, 0, 0], 128, 128),                          # no rows at all
    ([4096], 512, 640),                                # one big group
])
def test_grouped_gemm_fwd_dgrad_wgrad(counts, K, N):
    E = len(counts)
    M = sum(counts)
    offs = _offs(counts)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(E, K, N, device=DEV) / K ** 0.5).to(torch.bfloat16)
    dy = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    C = ops.ext()
    y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    C.grouped_gemm(0, x, w, offs, y, False)
    ref = _ref_fwd(x, w, offs)
    if M:
        assert torch.isfinite(y.float()).all()
        assert ((y.float() - ref).abs().max() / (ref.abs().max() + 1e-6)).item() < 1e-2
    dx = torch.full((M, K), float("nan"), device=DEV, dtype=torch.bfloat16)
    C.grouped_gemm(1, dy, w, offs, dx, False)
    ref_dx = _ref_fwd(dy, w.transpose(1, 2).contiguous(), offs)
    if M:
        assert ((dx.float() - ref_dx).abs().max() / (ref_dx.abs().max() + 1e-6)).item() < 1e-2
    dw = torch.full((E, K, N), 3.0, device=DEV)
    C.grouped_gemm(2, x, dy, offs, dw, True)      # accumulate onto 3.0
    b = offs.tolist()
    for e in range(E):
        r = x[b[e]:b[e + 1]].float().t() @ dy[b[e]:b[e + 1]].float() + 3.0
        err = (dw[e] - r).abs().max().item()
        assert err <= 1e-3 * (r.abs().max().item() + 1.0), (e, err)
    dw0 = torch.full((E, K, N), float("nan"), device=DEV)
    C.grouped_gemm(2, x, dy, offs, dw0, False)    # overwrite: empty groups get exact zeros
    for e in range(E):
        if b[e] == b[e + 1]:
            assert (dw0[e] == 0).all()
    assert torch.isfinite(dw0).all()


def test_grouped_gemm_asymmetric_exact():
    # small-integer operands: exact in bf16/fp32, catches any row/col swap of the C layout
    counts = [5, 130, 0, 77]
    E, K, N = 4, 64, 136
    offs = _offs(counts)
    M = sum(counts)
    x = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
    w = torch.randint(-3, 4, (E, K, N), device=DEV).to(torch.bfloat16)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.ext().grouped_gemm(0, x, w, offs, y, False)
    assert torch.equal(y.float(), _ref_fwd(x, w, offs))


def _single():
    import torch.distributed as dist

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29641")
        dist.init_process_group("gloo", rank=0, world_size=1)
    if not ps.model_parallel_is_initialized():
        ps.initialize_model_parallel(1)


def _moe(E=8, k=2, H=512, I=768, dtype=torch.bfloat16):
    from neuronx_distributed_llama3_2_amd.modules.moe import MoE, ExpertMLPs, RouterTopK

    torch.manual_seed(1)
    r = RouterTopK(E, k, H)
    mlps = ExpertMLPs(E, k, H, I, "silu", True, None, normalize_top_k_affinities=True, dtype=dtype)
    return MoE(r, mlps, return_router_logits=True)


def test_dropless_moe_matches_fp32_and_has_no_host_sync():
    _single()
    layer = _moe()
    ref_layer = _moe(dtype=torch.float32)               # same init, fp32, CPU reference path
    ref_layer.load_state_dict({k: v.float() for k, v in layer.state_dict().items()})
    layer = layer.to(DEV)
    layer.train()
    ref_layer.train()
    x = torch.randn(1024, 1, 512).to(torch.bfloat16).float()   # identical router inputs on both paths
    xg = x.to(DEV).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")               # any device->host sync raises
    try:
        out, _ = layer(xg.to(torch.bfloat16))
        out.float().square().mean().backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    out_r, _ = ref_layer(xr)
    out_r.square().mean().backward()
    o, r = out.float().cpu(), out_r.detach()
    assert ((o - r).abs().max() / r.abs().max()).item() < 3e-2
    gx, gr = xg.grad.float().cpu(), xr.grad
    assert ((gx - gr).abs().max() / gr.abs().max()).item() < 5e-2
    for name in ["expert_mlps.mlp_op.gate_up_proj.weight", "expert_mlps.mlp_op.down_proj.weight"]:
        g = dict(layer.named_parameters())[name].grad.float().cpu()
        g_ref = dict(ref_layer.named_parameters())[name].grad
        assert ((g - g_ref).abs().max() / g_ref.abs().max()).item() < 5e-2, name
