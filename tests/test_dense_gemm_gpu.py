"""Hand-written dense GEMM (csrc/dense_gemm.hip) against fp32 torch: NT (forward / input gradient on
the K-major weight copy) and TN (token-major weight gradient), bf16 / fp32-accumulate / split-K
atomic epilogues, full and ragged tiles."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from neuronx_distributed_llama3_2_amd.ops import ext  # noqa: E402


def _rel(got, ref):
    return ((got.float() - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (300, 264, 192), (1024, 768, 4096), (257, 1032, 64)])
def test_dense_gemm_nt_bf16(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    c = torch.full((M, N), float("nan"), device="cuda").to(torch.bfloat16)
    ext().dense_gemm(0, 0, a, b, c)
    ref = a.float() @ b.float().t()
    assert _rel(c, ref) < 1e-2


@pytest.mark.parametrize("epi,splits", [(1, 1), (2, 0), (2, 3)])
@pytest.mark.parametrize("T,M,N", [(512, 256, 256), (384, 264, 520), (4096, 768, 1024)])
def test_dense_gemm_tn_fp32(T, M, N, epi, splits):
    g = torch.Generator(device="cuda").manual_seed(T + M + N + epi)
    dy = torch.randn(T, M, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(T, N, device="cuda", generator=g).to(torch.bfloat16)
    c0 = torch.randn(M, N, device="cuda", generator=g)
    c = c0.clone()
    ext().dense_gemm(1, epi, dy, x, c, splits)
    ref = c0.double() + dy.double().t() @ x.double()
    assert _rel(c, ref) < 1e-5


def test_dense_gemm_nt_fp32_acc_and_strided():
    # row strides larger than the logical width (a view into a wider buffer)
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randn(640, 448, device="cuda", generator=g).to(torch.bfloat16)[:, :384]
    b = torch.randn(520, 392, device="cuda", generator=g).to(torch.bfloat16)[:, :384]
    c0 = torch.randn(640, 520, device="cuda", generator=g)
    c = c0.clone()
    ext().dense_gemm(0, 1, a, b, c)
    ref = c0.double() + a.double() @ b.double().t()
    assert _rel(c, ref) < 1e-5


def test_dense_gemm_tn_bf16_out():
    g = torch.Generator(device="cuda").manual_seed(9)
    dy = torch.randn(256, 512, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(256, 264, device="cuda", generator=g).to(torch.bfloat16)
    c = torch.empty(512, 264, device="cuda", dtype=torch.bfloat16)
    ext().dense_gemm(1, 0, dy, x, c)
    assert _rel(c, dy.float().t() @ x.float()) < 1e-2


def test_dense_gemm_rejects_bad_shapes():
    a = torch.randn(64, 100, device="cuda").to(torch.bfloat16)
    b = torch.randn(64, 100, device="cuda").to(torch.bfloat16)
    c = torch.empty(64, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ext().dense_gemm(0, 0, a, b, c)   # K % 64 != 0


def test_framework_wgrad_routes_skinny_shards_to_dense_tn():
    """ops.gemm.wgrad_accumulate_ sends the tensor-parallel shards and the TP=1 o_proj (no producer copy,
    M N / (M + N) < 2200) to the hand-written TN kernel -- RMW epilogue when one K split fills the chip,
    split-K atomics otherwise -- and keeps hipBLASLt for the wide TP=1 shapes; all accumulate like fp64."""
    from neuronx_distributed_llama3_2_amd.ops import gemm as G

    torch.manual_seed(3)
    for (T, M, N, copy, want) in [(512, 768, 4096, False, True), (1024, 4096, 512, False, True),
                                  (512, 4096, 4096, False, True), (512, 6144, 4096, False, False),
                                  (512, 768, 4096, True, False), (288, 768, 4096, False, False)]:
        dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        mg = torch.randn(M, N, device="cuda", dtype=torch.float32)
        go_t = dy.t().contiguous() if copy else None
        assert G._use_dense_wgrad(mg, dy, x, has_copy=copy) == (want and G._DENSE_WG != "0"), (T, M, N, copy)
        ref = mg.double() + dy.double().t() @ x.double()
        G.wgrad_accumulate_(mg, dy, x, go_t=go_t)
        scale = dy.double().abs().t() @ x.double().abs()
        assert torch.all((mg.double() - ref).abs() <= 1e-5 * scale + 1e-4)
