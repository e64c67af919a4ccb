"""ZeRO-1 optimizer checkpoints in the reference's torch_xla layout (optimizer/zero_layout.py):
written at DP=2, merged with an independent re-implementation of the reference converter's merge
(src/neuronx_distributed/optimizer/convert_zero_checkpoints.py:54-99: concatenate each parameter's
dim-0 shards, drop the padding), re-sharded by our converter for DP=1 and DP=4, and resumed there
with the optimizer state restored bit-exactly."""

import os
import shutil
import tempfile

import torch
import torch.distributed as dist

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

STEPS = 6


def _batches(vocab):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, vocab, (4, 32), generator=g) for _ in range(STEPS)]


def _w(rank, world, ckpt_dir, resume, out):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config

    cfg_nxd = nxd.neuronx_distributed_config(optimizer_config={"zero_one_enabled": True, "grad_clipping": True,
                                                               "max_grad_norm": 1.0})
    cfg = llama_config("tiny")
    torch.manual_seed(0)
    model = nxd.initialize_parallel_model(cfg_nxd, LlamaForCausalLM, cfg, torch.float32)
    opt = nxd.initialize_parallel_optimizer(cfg_nxd, torch.optim.AdamW, model.parameters(), lr=3e-3,
                                            betas=(0.9, 0.95), weight_decay=0.01)
    dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
    start, losses = 0, []
    rec = {}
    if resume:
        start = nxd.load_checkpoint(ckpt_dir, model=model, optimizer=opt)["step"]
        rec["loaded"] = opt.state_dict()          # this DP size's reference-layout shards
    batches = _batches(cfg.vocab_size)
    for step in range(start, STEPS):
        local = batches[step].chunk(dp)[dpr]
        o = model(local, labels=local)
        o.loss.backward()
        opt.step()
        opt.zero_grad()
        lo = o.loss.detach().clone()
        dist.all_reduce(lo)
        losses.append(float(lo) / world)
        if not resume and step == 2:
            nxd.save_checkpoint(ckpt_dir, "step_3", model=model, optimizer=opt, user_content={"step": 3})
    nxd.finalize_checkpoint()
    rec["losses"] = losses
    torch.save(rec, f"{out}.{rank}")


def _ref_merge(shards):
    """Independent re-implementation of the reference merge semantics."""
    full = {}
    for k, shape in shards[0]["shape_info"].items():
        ent = {}
        for key in ("exp_avg", "exp_avg_sq"):
            ent[key] = torch.cat([s["base_state"][k][key] for s in shards])[:shape[0]]
        ent["master"] = torch.cat([s["sharded_master_weights"][k] for s in shards])[:shape[0]]
        full[k] = ent
    return full


def test_reference_layout_dp2_to_dp1_and_dp4_bit_exact():
    from neuronx_distributed_llama3_2_amd.optimizer.convert_zero_checkpoints import main as zmain

    d = tempfile.mkdtemp()
    ck = os.path.join(d, "ck")
    run_distributed(_w, 2, ck, False, os.path.join(d, "dp2"))
    optim = os.path.join(ck, "step_3", "optim")
    files = sorted(os.listdir(optim))
    assert files == ["dp_rank_00_tp_rank_00_pp_rank_00.pt", "dp_rank_01_tp_rank_00_pp_rank_00.pt"], files
    shards = [torch.load(os.path.join(optim, f), weights_only=True) for f in files]
    s0 = shards[0]
    assert set(s0) >= {"state", "param_groups", "base_state", "shape_info", "sharded_master_weights"}, set(s0)
    assert s0["state"] == {}
    for k, shape in s0["shape_info"].items():   # dim-0 padded to a multiple of the DP size, chunk per rank
        ent = s0["base_state"][k]
        assert set(ent) == {"step", "exp_avg", "exp_avg_sq"} and float(ent["step"]) == 3.0
        assert ent["exp_avg"].shape[0] == -(-shape[0] // 2) and ent["exp_avg"].shape[1:] == shape[1:]
    n_params = len(s0["shape_info"])
    assert sorted(i for g in s0["param_groups"] for i in g["params"]) == list(range(n_params))
    ref_full = _ref_merge(shards)

    zmain(["--input_dir", os.path.join(ck, "step_3"), "--output_dir", os.path.join(d, "full"), "--convert_to_full"])
    ours = torch.load(os.path.join(d, "full", "optim", "full_tp_rank_00_pp_rank_00.pt"), weights_only=True)
    for k, ent in ref_full.items():
        assert torch.equal(ours["base_state"][k]["exp_avg"], ent["exp_avg"])
        assert torch.equal(ours["base_state"][k]["exp_avg_sq"], ent["exp_avg_sq"])
        assert torch.equal(ours["sharded_master_weights"][k], ent["master"])

    cont = torch.load(os.path.join(d, "dp2.0"))["losses"]
    for new_dp in (1, 4):
        nck = os.path.join(d, f"ck{new_dp}")
        shutil.copytree(ck, nck)
        shutil.rmtree(os.path.join(nck, "step_3", "optim"))
        zmain(["--input_dir", os.path.join(d, "full"), "--output_dir", os.path.join(nck, "step_3"),
               "--convert_to_sharded", "--dp_size", str(new_dp)])
        assert len(os.listdir(os.path.join(nck, "step_3", "optim"))) == new_dp
        run_distributed(_w, new_dp, nck, True, os.path.join(d, f"r{new_dp}"))
        loaded = [torch.load(os.path.join(d, f"r{new_dp}.{r}"))["loaded"] for r in range(new_dp)]
        back = _ref_merge(loaded)      # state after loading at the new DP size == the saved state
        for k, ent in ref_full.items():
            for key in ("exp_avg", "exp_avg_sq", "master"):
                assert torch.equal(back[k][key], ent[key]), (new_dp, k, key)
        res = torch.load(os.path.join(d, f"r{new_dp}.0"))["losses"]
        assert len(res) == STEPS - 3
        for x, y in zip(cont[3:], res):   # same global batches; DP changes only reduction order
            assert abs(x - y) < 1e-4, (new_dp, cont, res)


def _w_dcp(rank, world, path, save, out):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.zero_dcp_utils import load_optim_state_dict, save_optim_state_dict

    cfg_nxd = nxd.neuronx_distributed_config(optimizer_config={"zero_one_enabled": True, "grad_clipping": True})
    cfg = llama_config("tiny")
    torch.manual_seed(0)
    model = nxd.initialize_parallel_model(cfg_nxd, LlamaForCausalLM, cfg, torch.float32)
    opt = nxd.initialize_parallel_optimizer(cfg_nxd, torch.optim.AdamW, model.parameters(), lr=3e-3)
    inner = opt.optimizer
    if save:
        dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
        for step in range(2):
            local = _batches(cfg.vocab_size)[step].chunk(dp)[dpr]
            model(local, labels=local).loss.backward()
            opt.step()
            opt.zero_grad()
        save_optim_state_dict(path, inner)
    else:
        load_optim_state_dict(path, inner)
    sd = inner.state_dict()           # reference layout at this DP size
    torch.save(sd, f"{out}.{rank}")


def test_dcp_reshards_across_dp_sizes():
    """DCP optimizer checkpoint (per-parameter row-sharded tensors, reference zero_dcp_utils.py:84-140)
    saved at DP=2 loads at DP=1 and DP=4 with every state element restored."""
    d = tempfile.mkdtemp()
    path = os.path.join(d, "dcp")
    run_distributed(_w_dcp, 2, path, True, os.path.join(d, "s"))
    ref = _ref_merge([torch.load(os.path.join(d, f"s.{r}")) for r in range(2)])
    for new_dp in (1, 4):
        run_distributed(_w_dcp, new_dp, path, False, os.path.join(d, f"l{new_dp}"))
        got = _ref_merge([torch.load(os.path.join(d, f"l{new_dp}.{r}")) for r in range(new_dp)])
        for k, ent in ref.items():
            for key in ("exp_avg", "exp_avg_sq", "master"):
                assert torch.equal(got[k][key], ent[key]), (new_dp, k, key)
        assert float(torch.load(os.path.join(d, f"l{new_dp}.0"))["base_state"][0]["step"]) == 2.0
