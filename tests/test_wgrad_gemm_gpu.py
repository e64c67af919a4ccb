"""Numerics of the hand-written weight-gradient GEMM (csrc/wgrad_gemm.hip) against an fp64 PyTorch
reference: main_grad [M, N] += dy [T, M]^T x [T, N] with token-major bf16 operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ext():
    from neuronx_distributed_llama3_2_amd.ops._ext import ext

    return ext()


@pytest.mark.parametrize("T,M,N,splits", [
    (256, 512, 256, 1),      # one tile row, exact tiles
    (1024, 768, 512, 4),     # token splits (fp32 atomics from 4 workgroups per element)
    (512, 264, 136, 0),      # partial tiles on both output dims, auto splits
    (2048, 256, 1024, 0),    # skinny output, auto split count
])
def test_wgrad_gemm_matches_fp64(T, M, N, splits):
    torch.manual_seed(T + M + N)
    dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    mg = torch.randn(M, N, device="cuda", dtype=torch.float32)
    ref = mg.double() + dy.double().t() @ x.double()
    _ext().wgrad_gemm(mg, dy, x, splits)
    torch.cuda.synchronize()
    scale = (dy.double().abs().t() @ x.double().abs())   # sum |a b| per element
    err = (mg.double() - ref).abs()
    assert torch.all(err <= 2e-6 * scale + 1e-5), float((err / (scale + 1)).max())


def test_wgrad_gemm_strided_operands_and_accumulation():
    """Row-strided views (e.g. the q|k|v slices of a fused projection) and repeated accumulation."""
    torch.manual_seed(0)
    T, M, N = 512, 384, 256
    big_dy = torch.randn(T, M + 128, device="cuda", dtype=torch.bfloat16)
    big_x = torch.randn(T, N + 64, device="cuda", dtype=torch.bfloat16)
    dy, x = big_dy[:, 64:64 + M], big_x[:, 32:32 + N]
    mg = torch.zeros(M, N, device="cuda", dtype=torch.float32)
    for _ in range(3):
        _ext().wgrad_gemm(mg, dy, x, 0)
    ref = 3 * (dy.double().t() @ x.double())
    scale = 3 * (dy.double().abs().t() @ x.double().abs())
    assert torch.all((mg.double() - ref).abs() <= 2e-6 * scale + 1e-5)


def test_wgrad_gemm_rejects_bad_shapes():
    dy = torch.randn(48, 64, device="cuda", dtype=torch.bfloat16)   # T not a multiple of 32
    x = torch.randn(48, 64, device="cuda", dtype=torch.bfloat16)
    mg = torch.zeros(64, 64, device="cuda")
    with pytest.raises(RuntimeError):
        _ext().wgrad_gemm(mg, dy, x, 0)


def test_framework_wgrad_dispatch_takes_kernel_on_skinny_shards():
    """ops.gemm.wgrad_accumulate_ routes the TP=8-like skinny shards (q|k|v: 768 x 4096) and the
    vocabulary-wide lm_head shard without producer copies (16032 x 4096) to the hand-written kernel
    and keeps hipBLASLt for the large TP=1 shapes; both accumulate correctly."""
    from neuronx_distributed_llama3_2_amd.ops import gemm as G

    torch.manual_seed(1)
    for (T, M, N, copy, want) in [(512, 768, 4096, False, True), (512, 4096, 4096, False, False),
                                  (512, 4096, 4096, True, False), (256, 16032, 4096, False, True),
                                  (256, 16032, 4096, True, False)]:
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        mg = torch.randn(M, N, device="cuda", dtype=torch.float32)
        go_t = dy.t().contiguous() if copy else None   # as the SwiGLU backward writes it
        assert G._use_wgrad_kernel(mg, dy, x, has_copy=copy) == (want and G._WG_KERNEL != "0")
        ref = mg.double() + dy.double().t() @ x.double()
        G.wgrad_accumulate_(mg, dy, x, go_t=go_t)
        scale = dy.double().abs().t() @ x.double().abs()
        assert torch.all((mg.double() - ref).abs() <= 1e-5 * scale + 1e-4)
