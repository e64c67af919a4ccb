"""Tensor / sequence-parallel layers on N CPU ranks (gloo) vs a single-device torch reference
(the reference's ti/parallel_layers/test_layers.py strategy, run without accelerators)."""

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

TOL = dict(atol=1e-4, rtol=1e-4)


def test_meshes():
    dp, edp, tp_m, dp_m, pp_m, ep_m, edp_m = ps._build_meshes(32, 8, 4, 1)
    assert dp == 1 and tp_m[0] == list(range(8)) and pp_m[0] == [0, 8, 16, 24]
    dp, edp, tp_m, dp_m, pp_m, ep_m, edp_m = ps._build_meshes(16, 2, 1, 4)
    assert dp == 8 and edp == 2
    assert dp_m[0] == [0, 2, 4, 6, 8, 10, 12, 14]
    assert ep_m[0] == [0, 2, 4, 6] and edp_m[0] == [0, 8]
    with pytest.raises(RuntimeError):
        ps._build_meshes(12, 8, 1, 1)


def _w_column_row(rank, world, sp):
    from neuronx_distributed_llama3_2_amd.parallel_layers import ColumnParallelLinear, RowParallelLinear
    from neuronx_distributed_llama3_2_amd.parallel_layers.mappings import (
        gather_from_sequence_parallel_region,
        scatter_to_sequence_parallel_region,
    )

    ps.initialize_model_parallel(world)
    torch.manual_seed(0)
    col = ColumnParallelLinear(16, 32, bias=not sp, gather_output=False, sequence_parallel_enabled=sp,
                               keep_master_weight=True)
    torch.manual_seed(1)
    row = RowParallelLinear(32, 16, bias=True, input_is_parallel=True, sequence_parallel_enabled=sp,
                            keep_master_weight=True)
    S, B = 8, 3
    torch.manual_seed(2)
    x = torch.randn(S, B, 16)
    xr = x.clone().requires_grad_(True)
    xin = scatter_to_sequence_parallel_region(x.clone().requires_grad_(True)) if sp else x.clone().requires_grad_(True)
    xin.retain_grad()
    y = row(F.gelu(col(xin)))
    if sp:
        y = gather_from_sequence_parallel_region(y, to_model_parallel=False)
    # reference
    Wc, Wr = col.master_weight, row.master_weight
    bc = None
    if not sp:
        bc_full = [torch.zeros(16) for _ in range(world)]
        dist.all_gather(bc_full, col.bias.detach().contiguous())
        bc = torch.cat(bc_full)
    yr = F.linear(F.gelu(F.linear(xr, Wc, bc)), Wr, row.bias.detach())
    torch.testing.assert_close(y, yr, **TOL)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    # weight grads: this rank's shard of the full grad (Wc split rows, Wr split cols)
    gWc = torch.zeros_like(Wc)
    gWr = torch.zeros_like(Wr)
    Wc_ = Wc.clone().requires_grad_(True)
    Wr_ = Wr.clone().requires_grad_(True)
    F.linear(F.gelu(F.linear(x, Wc_, bc)), Wr_, row.bias.detach()).backward(g)
    n = 32 // world
    torch.testing.assert_close(col.weight.grad, Wc_.grad[rank * n:(rank + 1) * n], **TOL)
    torch.testing.assert_close(row.weight.grad, Wr_.grad[:, rank * n:(rank + 1) * n], **TOL)
    if sp:
        rb = row.bias.grad.clone()
        dist.all_reduce(rb)  # sequence-parallel bias grads are partial over TP
        torch.testing.assert_close(rb, g.sum((0, 1)), **TOL)
    _ = gWc, gWr


@pytest.mark.parametrize("sp", [False, True])
def test_column_row_parallel(sp):
    run_distributed(_w_column_row, 2, sp)


def _w_embedding_xent(rank, world):
    from neuronx_distributed_llama3_2_amd.parallel_layers import ParallelEmbedding, parallel_cross_entropy

    ps.initialize_model_parallel(world)
    torch.manual_seed(0)
    V, H = 64, 8
    emb = ParallelEmbedding(V, H)
    full = [torch.zeros_like(emb.weight) for _ in range(world)]
    dist.all_gather(full, emb.weight.detach().contiguous())
    Wf = torch.cat(full)
    ids = torch.randint(0, V, (5, 7))
    out = emb(ids)
    torch.testing.assert_close(out, F.embedding(ids, Wf))
    # vocab-parallel cross entropy
    torch.manual_seed(3)
    logits_full = torch.randn(6, V, requires_grad=True)
    n = V // world
    local = logits_full.detach()[:, rank * n:(rank + 1) * n].clone().requires_grad_(True)
    tgt = torch.randint(0, V, (6,))
    tgt[2] = -100
    for eps in (0.0, 0.1):
        loss = parallel_cross_entropy(local, tgt, label_smoothing=eps)
        ref = F.cross_entropy(logits_full, tgt.clamp(min=0), reduction="none", label_smoothing=eps)
        ref = torch.where(tgt == -100, torch.zeros_like(ref), ref)
        torch.testing.assert_close(loss, ref, **TOL)
        local.grad = None
        logits_full.grad = None
        loss.sum().backward()
        ref.sum().backward()
        torch.testing.assert_close(local.grad, logits_full.grad[:, rank * n:(rank + 1) * n], **TOL)


def test_embedding_and_cross_entropy():
    run_distributed(_w_embedding_xent, 2)


def _w_qkv(rank, world, mult):
    from neuronx_distributed_llama3_2_amd.modules.qkv_linear import GQAQKVColumnParallelLinear

    ps.initialize_model_parallel(world)
    torch.manual_seed(0)
    H, D, nq = 16, 4, 4
    nkv = 1 if mult > 1 else 2
    lin = GQAQKVColumnParallelLinear(H, [nq * D, nkv * D], bias=False, gather_output=False, kv_size_multiplier=mult)
    torch.manual_seed(0)  # the layer drew q, k, v full weights in this order from the same seed
    ref_q = torch.empty(nq * D, H)
    ref_k = torch.empty(nkv * D, H)
    ref_v = torch.empty(nkv * D, H)
    import math

    for w in (ref_q, ref_k, ref_v):
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    x = torch.randn(3, 2, H)
    q, k, v = lin(x)
    qn = nq * D // world
    torch.testing.assert_close(q, F.linear(x, ref_q)[..., rank * qn:(rank + 1) * qn])
    kr = torch.cat([ref_k] * mult)
    kn = kr.shape[0] // world
    torch.testing.assert_close(k, F.linear(x, kr)[..., rank * kn:(rank + 1) * kn])
    # gradient: replicas of a kv head end with identical weight grads
    (q.sum() + (k * 2).sum() + v.sum()).backward()
    g = lin.weight_qkv.grad[qn:qn + kn].clone()
    gs = [torch.zeros_like(g) for _ in range(world)]
    dist.all_gather(gs, g)
    if mult > 1:
        torch.testing.assert_close(gs[0], gs[1])


@pytest.mark.parametrize("mult", [1, 2])
def test_gqa_qkv(mult):
    run_distributed(_w_qkv, 2, mult)


def _tag(over):
    return f"_h{over['num_attention_heads']}kv{over['num_key_value_heads']}" if over else ""


def _w_tiny_llama(rank, world, sp, over=None):
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config

    ps.initialize_model_parallel(world)
    cfg = llama_config("tiny", sequence_parallel_enabled=sp, **(over or {}))
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=torch.float32)
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 32))
    loss = model(ids, labels=ids).loss
    loss.backward()
    gn = torch.stack([p.grad.float().norm() ** 2 for p in model.parameters() if getattr(p, "tensor_model_parallel", False)]).sum()
    dist.all_reduce(gn)
    dup = torch.stack([p.grad.float().norm() ** 2 for p in model.parameters() if not getattr(p, "tensor_model_parallel", False)]).sum()
    if sp:
        # sequence-parallel norm grads are partial sums over TP ranks
        parts = [p.grad.clone() for p in model.parameters() if not getattr(p, "tensor_model_parallel", False)]
        for t in parts:
            dist.all_reduce(t)
        dup = torch.stack([t.norm() ** 2 for t in parts]).sum()
    torch.save({"loss": loss.detach(), "gn": (gn + dup).detach()}, f"/tmp/nxd_tiny_llama_{world}_{sp}_{rank}{_tag(over)}.pt")


@pytest.mark.parametrize("sp", [False, True])
def test_tiny_llama_tp2_matches_tp1(sp):
    """BASELINE config 1: tiny-Llama 2-layer, TP=2 on CPU/gloo == TP=1 (loss and grad norm)."""
    run_distributed(_w_tiny_llama, 1, False)
    run_distributed(_w_tiny_llama, 2, sp)
    r1 = torch.load(f"/tmp/nxd_tiny_llama_1_False_0.pt")
    r2 = torch.load(f"/tmp/nxd_tiny_llama_2_{sp}_0.pt")
    torch.testing.assert_close(r1["loss"], r2["loss"], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(r1["gn"], r2["gn"], atol=1e-3, rtol=1e-3)


def test_tiny_llama_tp4_sp_matches_tp1():
    """TP=4 with sequence parallelism (default 2 SP chunks at TP4, vs 4 at TP2) == TP=1."""
    over = {"num_attention_heads": 8, "num_key_value_heads": 4}
    run_distributed(_w_tiny_llama, 1, False, over)
    run_distributed(_w_tiny_llama, 4, True, over)
    r1 = torch.load(f"/tmp/nxd_tiny_llama_1_False_0{_tag(over)}.pt")
    r4 = torch.load(f"/tmp/nxd_tiny_llama_4_True_0{_tag(over)}.pt")
    torch.testing.assert_close(r1["loss"], r4["loss"], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(r1["gn"], r4["gn"], atol=1e-3, rtol=1e-3)


def test_tiny_llama_tp8_sp_matches_tp1():
    """The headline layout in miniature: TP=8 + SP (1 kv head per rank, 2 SP chunks) == TP=1."""
    over = {"num_attention_heads": 8, "num_key_value_heads": 8}
    run_distributed(_w_tiny_llama, 1, False, over)
    run_distributed(_w_tiny_llama, 8, True, over)
    r1 = torch.load(f"/tmp/nxd_tiny_llama_1_False_0{_tag(over)}.pt")
    r8 = torch.load(f"/tmp/nxd_tiny_llama_8_True_0{_tag(over)}.pt")
    torch.testing.assert_close(r1["loss"], r8["loss"], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(r1["gn"], r8["gn"], atol=1e-3, rtol=1e-3)


def _w_kv_replicated_training(rank, world, out):
    """TP > #kv heads: replicated kv heads (q head groups reshuffled as the reference converter does)
    train exactly like the unsharded model, clip norm included (replicated K/V rows count once)."""
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params

    ps.initialize_model_parallel(world)
    cfg = llama_config("tiny", sequence_parallel_enabled=world > 1, max_position_embeddings=512)
    torch.manual_seed(0)
    model = LlamaForCausalLM(cfg, dtype=torch.float32, device=torch.device("cpu"))
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=2e-3, grad_clipping=True, max_grad_norm=1.0,
                                  shared_param_ids=find_shared_params(model))
    torch.manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (2, 64))
    res = []
    for _ in range(3):
        loss = model(ids, labels=ids).loss
        loss.backward()
        opt.step()
        opt.zero_grad()
        res.append((float(loss), float(opt.grad_norm)))
    if rank == 0:
        torch.save(res, out)


def test_kv_replicated_tp4_trains_like_tp1():
    import os
    import tempfile

    d = tempfile.mkdtemp()
    run_distributed(_w_kv_replicated_training, 1, os.path.join(d, "a.pt"))
    run_distributed(_w_kv_replicated_training, 4, os.path.join(d, "b.pt"))   # tiny: 2 kv heads, m = 2
    a, b = torch.load(os.path.join(d, "a.pt")), torch.load(os.path.join(d, "b.pt"))
    for (la, ga), (lb, gb) in zip(a, b):
        assert abs(la - lb) < 1e-4 and abs(ga - gb) < 1e-4 * ga, (a, b)
