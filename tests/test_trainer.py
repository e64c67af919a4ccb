"""Trainer API + ZeRO-1 + checkpointing on CPU ranks (gloo)."""

import os
import tempfile

import pytest
import torch
import torch.distributed as dist

from dist_utils import run_distributed
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps


def _train(rank, world, tp, zero1, steps, out, ckpt_dir=None, resume=False):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config

    cfg_nxd = nxd.neuronx_distributed_config(tensor_parallel_size=tp,
                                            optimizer_config={"zero_one_enabled": zero1, "grad_clipping": True,
                                                              "max_grad_norm": 1.0})
    cfg = llama_config("tiny", sequence_parallel_enabled=tp > 1)
    torch.manual_seed(0)
    model = nxd.initialize_parallel_model(cfg_nxd, LlamaForCausalLM, cfg, torch.float32)
    opt = nxd.initialize_parallel_optimizer(cfg_nxd, torch.optim.AdamW, model.parameters(), lr=3e-3, betas=(0.9, 0.95),
                                            weight_decay=0.0)
    dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
    start = 0
    if resume:
        uc = nxd.load_checkpoint(ckpt_dir, model=model, optimizer=opt)
        start = uc["step"]
    losses = []
    g = torch.Generator().manual_seed(7)
    all_batches = [torch.randint(0, cfg.vocab_size, (4, 32), generator=g) for _ in range(2)]
    for step in range(start, steps):
        batch = all_batches[step % 2]
        local = batch.chunk(dp)[dpr]
        out_ = model(local, labels=local)
        out_.loss.backward()
        opt.step()
        opt.zero_grad()
        l = out_.loss.detach().clone()
        dist.all_reduce(l)
        losses.append(float(l) / dist.get_world_size())
        if ckpt_dir is not None and not resume and step == steps // 2 - 1:
            nxd.save_checkpoint(ckpt_dir, f"step_{step + 1}", model=model, optimizer=opt,
                                user_content={"step": step + 1}, num_kept_ckpts=2)
    if rank == 0:
        torch.save(losses, out)


def test_zero1_dp2_matches_dp1():
    d = tempfile.mkdtemp()
    run_distributed(_train, 1, 1, True, 4, os.path.join(d, "a.pt"))
    run_distributed(_train, 2, 1, True, 4, os.path.join(d, "b.pt"))
    a, b = torch.load(os.path.join(d, "a.pt")), torch.load(os.path.join(d, "b.pt"))
    # DP=2 averages per-rank losses over half batches: compare training trajectories loosely
    assert a[-1] < a[0] and b[-1] < b[0]
    for x, y in zip(a, b):
        assert abs(x - y) < 5e-2 * max(1.0, abs(x))


def test_tp2_dp2_zero1_checkpoint_resume():
    d = tempfile.mkdtemp()
    ck = os.path.join(d, "ckpt")
    run_distributed(_train, 4, 2, True, 6, os.path.join(d, "full.pt"), ck, False)
    assert os.path.exists(os.path.join(ck, "step_3", "done"))
    assert os.path.exists(os.path.join(ck, "step_3", "model", "dp_rank_00_tp_rank_01_pp_rank_00.pt"))
    assert os.path.exists(os.path.join(ck, "step_3", "optim", "dp_rank_01_tp_rank_01_pp_rank_00.pt"))
    run_distributed(_train, 4, 2, True, 6, os.path.join(d, "resumed.pt"), ck, True)
    full, res = torch.load(os.path.join(d, "full.pt")), torch.load(os.path.join(d, "resumed.pt"))
    assert len(res) == 3
    for x, y in zip(full[3:], res):
        assert abs(x - y) < 1e-5, (full, res)


def test_plain_optimizer_path():
    d = tempfile.mkdtemp()
    run_distributed(_train, 2, 2, False, 3, os.path.join(d, "p.pt"))
    p = torch.load(os.path.join(d, "p.pt"))
    assert p[-1] < p[0]


def _train_pp(rank, world, pp, steps, out):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import (
        LlamaDecoderLayer,
        LlamaForCausalLM,
        llama_config,
    )

    pcfg = {"transformer_layer_cls": LlamaDecoderLayer, "num_microbatches": 2, "input_names": ["input_ids", "labels"],
            "auto_partition": True, "broadcast_and_average_loss": True}
    cfg_nxd = nxd.neuronx_distributed_config(pipeline_parallel_size=pp, pipeline_config=pcfg,
                                            optimizer_config={"zero_one_enabled": True, "grad_clipping": True,
                                                              "max_grad_norm": 1.0})
    cfg = llama_config("tiny", num_hidden_layers=4)
    torch.manual_seed(0)
    model = nxd.initialize_parallel_model(cfg_nxd, LlamaForCausalLM, cfg, torch.float32)
    opt = nxd.initialize_parallel_optimizer(cfg_nxd, torch.optim.AdamW, model.parameters(), lr=3e-3,
                                            betas=(0.9, 0.95), weight_decay=0.0)
    dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
    g = torch.Generator().manual_seed(7)
    batches = [torch.randint(0, cfg.vocab_size, (8, 16), generator=g) for _ in range(2)]
    losses = []
    for step in range(steps):
        local = batches[step % 2].chunk(dp)[dpr]
        if pp > 1:
            loss = model.run_train(input_ids=local, labels=local)
        else:
            # same micro-batching as the pipeline: mean of two half-batch losses
            loss = 0
            for mb in local.chunk(2):
                l = model(mb, labels=mb).loss / 2
                l.backward()
                loss = loss + l.detach()
        opt.step()
        opt.zero_grad()
        l = torch.as_tensor(loss, dtype=torch.float32).clone().reshape(1)
        dist.all_reduce(l)
        losses.append(float(l) / world)
    if rank == 0:
        torch.save(losses, out)


def test_pp2_dp2_zero1_matches_dp2():
    d = tempfile.mkdtemp()
    run_distributed(_train_pp, 2, 1, 4, os.path.join(d, "ref.pt"))
    run_distributed(_train_pp, 4, 2, 4, os.path.join(d, "pp.pt"))
    a, b = torch.load(os.path.join(d, "ref.pt")), torch.load(os.path.join(d, "pp.pt"))
    assert a[-1] < a[0]
    for x, y in zip(a, b):
        assert abs(x - y) < 1e-4, (a, b)


def test_zero1_checkpoint_reshard_dp2_to_dp1():
    """ZeRO-1 optimizer checkpoint saved at DP=2 -> convert_zero_checkpoints (full and re-sharded) ->
    resume at DP=1 continues the DP=2 trajectory."""
    import shutil

    from neuronx_distributed_llama3_2_amd.optimizer.convert_zero_checkpoints import main as zmain

    d = tempfile.mkdtemp()
    ck = os.path.join(d, "ckpt")
    run_distributed(_train, 2, 1, True, 6, os.path.join(d, "full.pt"), ck, False)
    src = os.path.join(ck, "step_3")
    full_dir = os.path.join(d, "full_tag")
    zmain(["--input_dir", src, "--output_dir", full_dir, "--convert_to_full"])
    assert os.path.exists(os.path.join(full_dir, "optim", "full_tp_rank_00_pp_rank_00.pt"))
    new = os.path.join(d, "ckpt1")
    shutil.copytree(ck, new)
    shutil.rmtree(os.path.join(new, "step_3", "optim"))
    zmain(["--input_dir", full_dir, "--output_dir", os.path.join(new, "step_3"), "--convert_to_sharded", "--dp_size", "1"])
    run_distributed(_train, 1, 1, True, 6, os.path.join(d, "res.pt"), new, True)
    full, res = torch.load(os.path.join(d, "full.pt")), torch.load(os.path.join(d, "res.pt"))
    assert len(res) == 3
    for x, y in zip(full[3:], res):
        assert abs(x - y) < 1e-4, (full, res)


def _dcp(rank, world, path, out):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.zero_dcp_utils import load_optim_state_dict, save_optim_state_dict

    cfg_nxd = nxd.neuronx_distributed_config(optimizer_config={"zero_one_enabled": True, "grad_clipping": True,
                                                               "max_grad_norm": 1.0})
    cfg = llama_config("tiny")
    torch.manual_seed(0)
    model = nxd.initialize_parallel_model(cfg_nxd, LlamaForCausalLM, cfg, torch.float32)
    opt = nxd.initialize_parallel_optimizer(cfg_nxd, torch.optim.AdamW, model.parameters(), lr=3e-3)
    g = torch.Generator().manual_seed(7)
    batch = torch.randint(0, cfg.vocab_size, (4, 32), generator=g)
    local = batch.chunk(world)[rank]
    for _ in range(2):
        model(local, labels=local).loss.backward()
        opt.step()
        opt.zero_grad()
    inner = opt.optimizer if hasattr(opt, "optimizer") else opt
    save_optim_state_dict(path, inner)
    snap = [(b.master.clone(), b.exp_avg_sq.clone()) for b in inner.buffers]
    for b in inner.buffers:
        b.master.zero_()
        b.exp_avg_sq.zero_()
    load_optim_state_dict(path, inner)
    for (m, v), b in zip(snap, inner.buffers):
        assert torch.equal(m, b.master) and torch.equal(v, b.exp_avg_sq)
    assert inner.step_count == 2
    if rank == 0:
        torch.save(True, out)


def test_zero1_dcp_save_load():
    d = tempfile.mkdtemp()
    run_distributed(_dcp, 2, os.path.join(d, "dcp"), os.path.join(d, "ok.pt"))
    assert torch.load(os.path.join(d, "ok.pt"))


def _tied_step(rank, world, out):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config

    cfg_nxd = nxd.neuronx_distributed_config(tensor_parallel_size=1,
                                            optimizer_config={"zero_one_enabled": True, "grad_clipping": False})
    cfg = llama_config("tiny", tie_word_embeddings=True)
    torch.manual_seed(0)
    model = nxd.initialize_parallel_model(cfg_nxd, LlamaForCausalLM, cfg, torch.float32)
    # the optimizer is built WITHOUT the model: the tie must still be honoured
    opt = nxd.initialize_parallel_optimizer(cfg_nxd, torch.optim.AdamW, model.parameters(), lr=1e-2, weight_decay=0.0)
    dp, dpr = ps.get_data_parallel_size(), ps.get_data_parallel_rank()
    g = torch.Generator().manual_seed(11)
    for _ in range(2):
        micro = [torch.randint(0, cfg.vocab_size, (4, 32), generator=g) for _ in range(2)]
        for i, batch in enumerate(micro):
            opt.set_grad_sync(i == len(micro) - 1)   # backward-overlapped reduction armed on the last micro
            local = batch.chunk(dp)[dpr]
            (model(local, labels=local).loss / len(micro)).backward()
        opt.step()
        opt.zero_grad()
    if rank == 0:
        sd = {k: v.detach().clone() for k, v in model.module.state_dict().items()} if hasattr(model, "module") \
            else {k: v.detach().clone() for k, v in model.state_dict().items()}
        torch.save(sd, out)


def test_tied_embedding_dp2_matches_dp1():
    d = tempfile.mkdtemp()
    run_distributed(_tied_step, 1, os.path.join(d, "a.pt"))
    run_distributed(_tied_step, 2, os.path.join(d, "b.pt"))
    a, b = torch.load(os.path.join(d, "a.pt")), torch.load(os.path.join(d, "b.pt"))
    emb = [k for k in a if "embed_tokens" in k][0]
    for k in a:
        torch.testing.assert_close(b[k], a[k], rtol=0, atol=2e-4, msg=k)
    assert not torch.equal(a[emb], torch.zeros_like(a[emb]))


def test_foreign_subdir_survives_checkpoint_gc():
    """Only directories with the `checkpoint` begin marker are tags: a user directory under the
    checkpoint dir is never treated as an interrupted save and deleted."""
    from neuronx_distributed_llama3_2_amd.trainer.checkpoint_storage import FilesysCheckpointStorage
    from neuronx_distributed_llama3_2_amd.trainer.checkpoint import _determine_remove_tags

    d = tempfile.mkdtemp()
    os.makedirs(os.path.join(d, "tensorboard"))
    open(os.path.join(d, "tensorboard", "events"), "w").write("x")
    for i, tag in enumerate(["step_1", "step_2", "step_3"]):
        os.makedirs(os.path.join(d, tag))
        open(os.path.join(d, tag, "checkpoint"), "w").write("1")
        if tag != "step_2":
            open(os.path.join(d, tag, "done"), "w").write("1")
        t = 1000 + i
        os.utime(os.path.join(d, tag, "checkpoint"), (t, t))
    st = FilesysCheckpointStorage(d)
    assert st.list_checkpoint_tags() == ["step_1", "step_2", "step_3"]
    assert sorted(_determine_remove_tags(st, 1, current="step_3")) == ["step_1", "step_2"]
    assert st.get_latest_tag() == "step_3"
