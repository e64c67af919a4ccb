"""Weight-layout optimisation (reference: trace/model_builder.py:457-586 -- weights transformed
once at load to the layout chosen for the priority bucket).  On the CPU the measured pass keeps
every weight as stored, so these tests force the packed K-major layout and check that the outputs
do not change, that the map round-trips through compile()/load(), and that the ModelBuilder
priority hook and the parallel-linear override serve no-grad calls from the packed copy."""

import os

import torch

from test_inference import _hf_model, _inf_model, _tiny_cfg
from neuronx_distributed_llama3_2_amd.trace import weight_layout as wl


def test_packed_layout_inference_matches_and_round_trips(tmp_path):
    cfg = _tiny_cfg()
    hf = _hf_model(cfg, seed=2)
    m = _inf_model(cfg, hf.state_dict())
    torch.manual_seed(5)
    ids = torch.randint(3, cfg.vocab_size, (2, 12))
    ref = m._context_encode(ids)
    names = [n for n, _ in wl._weights(m.model)]
    assert any(n.endswith("qkv_proj") for n in names) and any(n.endswith("down_proj") for n in names)
    layouts = {n: "kn" for n in names}
    assert wl.apply_layouts(m.model, layouts) == len(names)
    mods = dict(wl._weights(m.model))
    for n in names:
        w = wl._weight_of(mods[n])
        assert mods[n]._nxd_packed_kn.shape == (w.shape[1], w.shape[0]) and mods[n]._nxd_packed_kn.is_contiguous()
    out = m._context_encode(ids)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    # CPU measurement keeps the stored layout everywhere
    assert set(wl.choose_layouts(m.model, 64).values()) == {"nk"}
    # map file round trip, then back to the stored layout
    wl.save_layouts(str(tmp_path), layouts)
    assert wl.load_layouts(str(tmp_path)) == layouts
    wl.apply_layouts(m.model, {n: "nk" for n in names})
    assert all(not hasattr(mods[n], "_nxd_packed_kn") for n in names)
    torch.testing.assert_close(m._context_encode(ids), ref, atol=0, rtol=0)


def test_weight_layout_compile_load(tmp_path):
    from neuronx_distributed_llama3_2_amd.inference import LlamaForCausalLMInference

    cfg = _tiny_cfg()
    hf = _hf_model(cfg, seed=3)
    m = _inf_model(cfg, hf.state_dict(), weight_layout_optimization=True)
    assert m.weight_layouts and set(m.weight_layouts.values()) == {"nk"}
    m.compile(str(tmp_path))
    assert os.path.exists(tmp_path / wl.LAYOUT_FILE)
    # a compiled map is reused (not re-measured) at load: force one weight to the packed layout
    layouts = dict(m.weight_layouts)
    key = next(k for k in layouts if k.endswith("down_proj"))
    layouts[key] = "kn"
    wl.save_layouts(str(tmp_path), layouts)
    m2 = LlamaForCausalLMInference.load(str(tmp_path), dtype=torch.float32)
    assert m2.weight_layouts == layouts
    assert dict(wl._weights(m2.model))[key]._nxd_layout == "kn"
    ids = torch.randint(3, cfg.vocab_size, (1, 9))
    torch.testing.assert_close(m2._context_encode(ids), m._context_encode(ids), atol=1e-5, rtol=1e-5)


def _w_packed_parallel(rank, world):
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.parallel_layers.layers import ColumnParallelLinear, RowParallelLinear

    ps.initialize_model_parallel(tensor_model_parallel_size=world)
    torch.manual_seed(0)
    net = torch.nn.Sequential(ColumnParallelLinear(16, 32, bias=True, gather_output=True),
                              RowParallelLinear(32, 8, bias=False, input_is_parallel=False))
    torch.manual_seed(1)
    x = torch.randn(3, 5, 16)
    with torch.no_grad():
        ref = net(x)
    wl.apply_layouts(net, {"0": "kn", "1": "kn"})
    assert isinstance(net[0]._forward_impl, wl._PackedForward)
    calls = []
    orig = wl._gemm.matmul
    wl._gemm.matmul = lambda a, b, out=None: calls.append(tuple(b.shape)) or orig(a, b)
    try:
        with torch.no_grad():
            out = net(x)
        y = net(x)                   # autograd path keeps the stored weight
    finally:
        wl._gemm.matmul = orig
    assert calls == [(16, 32 // world), (32 // world, 8)], calls
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    y.sum().backward()
    assert net[0].weight.grad is not None and net[0].weight.grad.shape == (32 // world, 16)
    wl.apply_layouts(net, {"0": "nk", "1": "nk"})
    assert not isinstance(net[0]._forward_impl, wl._PackedForward)


def test_parallel_linear_packed_forward_and_priority_hook():
    """TP=2 column/row-parallel linears serve no-grad calls from the packed copy (same output),
    autograd calls from the stored weight; priority-bucket token count."""
    from dist_utils import run_distributed
    from neuronx_distributed_llama3_2_amd.trace.model_builder import _bucket_tokens

    run_distributed(_w_packed_parallel, 2)
    # priority bucket GEMM rows: ids [B, S] -> B*S; activations [B, S, H] -> B*S
    assert _bucket_tokens((torch.zeros(2, 128, dtype=torch.long),)) == 256
    assert _bucket_tokens((torch.zeros(4, 16, 64),)) == 64
