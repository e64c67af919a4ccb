"""PyTorch-Lightning path (reference: src/neuronx_distributed/lightning/*, examples/training/llama/
lightning/*): NeuronXLAStrategy / NeuronLTModule / NeuronCheckpointIO / NeuronXLAPrecisionPlugin /
NeuronTensorBoardLogger / NeuronTQDMProgressBar and the example scripts, run on gloo ranks under a
stand-in of the `lightning.pytorch` API (tests/fake_lightning.py -- Lightning itself is not
installed, so parity with real Lightning is unpinned; what is pinned: the Lightning-driven run
takes exactly the steps of the framework's own training API, logs and checkpoints from the right
ranks, and the checkpoint holds the sharded model + reference-layout ZeRO-1 state)."""

import json
import os
import sys

import torch
import torch.distributed as dist

from dist_utils import run_distributed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LDIR = os.path.join(ROOT, "examples", "training", "llama", "lightning")
STEPS = 6
ARGS = ["--model", "tiny", "--tensor_parallel_size", "2", "--use_zero1_optimizer", "1", "--seq_len", "64",
        "--train_batch_size", "2", "--grad_accum_usteps", "2", "--max_steps", str(STEPS), "--warmup_steps", "2",
        "--lr", "3e-3", "--cpu", "--save_load_xser", "0"]


def _w_ptl(rank, world, out):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import fake_lightning

    fake_lightning.install()
    sys.path.insert(0, LDIR)
    import run_llama_nxd_ptl as ex

    a = ex.build_args(ARGS + ["--checkpoint_dir", os.path.join(out, "ck"), "--checkpoint_freq", "3",
                              "--tb_dir", os.path.join(out, "tb")])
    torch.manual_seed(a.seed)
    hist = ex.train_llama(a)
    torch.save(hist, os.path.join(out, f"hist.{rank}"))


def _w_plain(rank, world, out):
    """The same run through the framework's training API, no Lightning."""
    from types import SimpleNamespace

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import fake_lightning

    fake_lightning.install()   # the data module subclasses LightningDataModule
    sys.path.insert(0, LDIR)
    import run_llama_nxd_ptl as ex
    from data_module import NeuronLlamaDataModule

    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.utils.training_utils import (get_learning_rate_scheduler,
                                                                        get_param_groups_by_weight_decay)

    a = ex.build_args(ARGS)
    torch.manual_seed(a.seed)
    cfg = ex._model_config(a)
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=2, sequence_parallel=cfg.sequence_parallel_enabled,
        optimizer_config={"zero_one_enabled": True, "grad_clipping": True, "max_grad_norm": 1.0})
    model = nxd.initialize_parallel_model(nxd_config, LlamaForCausalLM, cfg, dtype=torch.float32)
    opt = nxd.initialize_parallel_optimizer(nxd_config, torch.optim.AdamW,
                                            get_param_groups_by_weight_decay(model, 0.01),
                                            lr=a.lr, betas=(a.beta1, a.beta2), weight_decay=a.weight_decay)
    sch = get_learning_rate_scheduler(opt, SimpleNamespace(lr_schedule="cosine", warmup_steps=a.warmup_steps,
                                                           max_steps=a.max_steps, min_lr=a.min_lr))
    dm = NeuronLlamaDataModule(None, a.seq_len, cfg.vocab_size, a.train_batch_size * a.grad_accum_usteps, seed=a.seed)
    dm.trainer = SimpleNamespace(strategy=SimpleNamespace(distributed_sampler_kwargs={
        "num_replicas": ps.get_data_parallel_size(), "rank": ps.get_data_parallel_rank()}))
    dm.setup()
    loader = dm.train_dataloader()
    loader.sampler.set_epoch(0)
    losses = []
    for step, batch in enumerate(loader):
        if step == STEPS:
            break
        tot = 0.0
        for i in range(a.grad_accum_usteps):
            opt.set_grad_sync(i == a.grad_accum_usteps - 1)
            mb = {k: v.chunk(a.grad_accum_usteps)[i] for k, v in batch.items()}
            o = model(**mb)
            (o.loss / a.grad_accum_usteps).backward()
            tot += float(o.loss)
        opt.step()
        opt.zero_grad()
        sch.step()
        losses.append(tot / a.grad_accum_usteps)
    torch.save(losses, os.path.join(out, f"plain.{rank}"))


def test_run_llama_nxd_ptl_matches_training_api(tmp_path):
    """examples/training/llama/lightning/run_llama_nxd_ptl.py on TP2 x DP2 with ZeRO-1 + SP."""
    out = str(tmp_path)
    run_distributed(_w_ptl, 4, out)
    run_distributed(_w_plain, 4, out)
    hist = torch.load(os.path.join(out, "hist.0"))
    assert [h[0] for h in hist] == list(range(1, STEPS + 1)), hist
    for r in (1, 2, 3):   # only the loss owner (last PP stage, tp 0, dp 0) records / logs
        assert torch.load(os.path.join(out, f"hist.{r}")) == []
    plain = torch.load(os.path.join(out, "plain.0"))
    for (_, lt, _), lp in zip(hist, plain):
        assert abs(lt - lp) < 1e-5 * abs(lp), (hist, plain)
    logs = sorted(os.listdir(os.path.join(out, "tb")))
    assert logs == ["metrics.0.jsonl"], logs
    rows = [json.loads(x) for x in open(os.path.join(out, "tb", "metrics.0.jsonl"))]
    assert [r["step"] for r in rows] == list(range(1, STEPS + 1))
    assert {"loss", "lr", "global_norm", "throughput_tokens_per_s"} <= set(rows[-1])
    for step in (3, 6):   # ModelCheckpoint every 3 steps; one shard per (dp, tp) rank
        d = os.path.join(out, "ck", f"step={step}.ckpt")
        files = sorted(os.listdir(d))
        assert files == [f"dp_rank_{dp:02d}_tp_rank_{tp:02d}_pp_rank_00.pt" for dp in range(2) for tp in range(2)]
        ck = torch.load(os.path.join(d, files[0]), weights_only=True)
        assert ck["global_step"] == step
        osd = ck["optimizer_states"][0]
        assert set(osd) >= {"base_state", "shape_info", "sharded_master_weights"}   # torch_xla ZeRO-1 layout
        assert float(next(iter(osd["base_state"].values()))["step"]) == step
        assert any("qkv" in k for k in ck["state_dict"])


def _w_ft(rank, world, hf_dir, data, out):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import fake_lightning

    fake_lightning.install()
    sys.path.insert(0, LDIR)
    import tp_llama_hf_finetune_ptl as ex

    before, after = ex.main(["--hf_model_dir", hf_dir, "--data_file", data, "--tensor_parallel_size", "2",
                             "--seq_len", "64", "--max_steps", "40", "--lr", "1e-2", "--warmup_steps", "2",
                             "--test_size", "4", "--use_zero_1", "--sequence_parallel_enabled",
                             "--checkpoint_dir", os.path.join(out, "ck")], cpu=True)
    dist.barrier()
    if rank == 0:
        torch.save((before, after), os.path.join(out, "ft.pt"))


def test_tp_llama_hf_finetune_ptl(tmp_path):
    """examples/training/llama/lightning/tp_llama_hf_finetune_ptl.py: HF checkpoint -> TP2 shards
    -> Lightning fine-tune -> held-out response loss drops; Lightning checkpoint written per rank."""
    from test_examples import _finetune_fixture

    hf_dir, data = _finetune_fixture(tmp_path)
    run_distributed(_w_ft, 2, hf_dir, data, str(tmp_path))
    before, after = torch.load(tmp_path / "ft.pt")
    assert after < 0.6 * before, (before, after)
    names = [f"dp_rank_00_tp_rank_{t:02d}_pp_rank_00.pt" for t in range(2)]   # xser: index + tensor dir
    files = set(os.listdir(tmp_path / "ck" / "step_40"))
    assert set(names + [n + ".tensors" for n in names]) <= files and all("tp_rank_0" in f for f in files), files
