"""Native token loader (csrc/dataloader.cpp): windows, labels, DP sharding (disjoint, complete),
epoch reshuffle, exact resume via state; plus training_utils schedules / meters."""

import os
import tempfile

import numpy as np
import torch

from neuronx_distributed_llama3_2_amd.utils.data_loader import DevicePrefetcher, TokenDataLoader, write_token_file


def _corpus(n=10_001, tb=4):
    d = tempfile.mkdtemp()
    p = os.path.join(d, "c.bin")
    toks = np.arange(n) % 60000
    write_token_file(p, [toks[:5000], toks[5000:]], token_bytes=tb)
    return p, toks


def test_windows_sharding_resume():
    seq, B = 16, 3
    for tb in (2, 4):
        p, toks = _corpus(tb=tb)
        ld = TokenDataLoader(p, seq, B, dp_rank=0, dp_size=1, seed=7, token_bytes=tb, threads=3)
        nsamp = (len(toks) - 1) // seq
        steps = ld.steps_per_epoch
        assert steps == nsamp // B
        seen = []
        for _ in range(steps):
            b = next(ld)
            assert b.shape == (B, seq + 1) and b.dtype == torch.int64
            for row in b:
                i0 = int(row[0])   # tokens are arange: the window start identifies the sample
                assert i0 % seq == 0 and torch.equal(row, torch.arange(i0, i0 + seq + 1) % 60000)
                seen.append(i0 // seq)
        assert len(set(seen)) == len(seen) == steps * B
    # DP: two ranks see disjoint samples of the same permutation
    p, toks = _corpus()
    a = TokenDataLoader(p, seq, 2, dp_rank=0, dp_size=2, seed=1, threads=2)
    b = TokenDataLoader(p, seq, 2, dp_rank=1, dp_size=2, seed=1, threads=2)
    sa = {int(r[0]) for _ in range(a.steps_per_epoch) for r in next(a)}
    sb = {int(r[0]) for _ in range(b.steps_per_epoch) for r in next(b)}
    assert not (sa & sb) and len(sa) == len(sb)
    # resume: state after k steps reproduces the same next batches
    c = TokenDataLoader(p, seq, 2, seed=3, threads=4)
    for _ in range(5):
        next(c)
    st = c.state_dict()
    ref = [next(c).clone() for _ in range(4)]
    d = TokenDataLoader(p, seq, 2, seed=3, threads=1)
    d.load_state_dict(st)
    got = [next(d).clone() for _ in range(4)]
    assert all(torch.equal(x, y) for x, y in zip(ref, got))
    # epoch boundary reshuffles
    e = TokenDataLoader(p, seq, 2, seed=3)
    ep0 = [next(e)[:, 0].clone() for _ in range(e.steps_per_epoch)]
    ep1 = [next(e)[:, 0].clone() for _ in range(e.steps_per_epoch)]
    assert len(set(torch.cat(ep0).tolist())) == len(torch.cat(ep0)) == len(set(torch.cat(ep1).tolist()))
    assert not all(torch.equal(x, y) for x, y in zip(ep0, ep1))
    pf = DevicePrefetcher(TokenDataLoader(p, seq, 2, seed=3))
    bt = next(pf)
    assert bt["input_ids"].shape == (2, seq)


def test_training_utils():
    from neuronx_distributed_llama3_2_amd.utils.training_utils import (CosineAnnealing, Throughput, TrainingMetrics,
                                                                          create_partition, get_learning_rate_scheduler)

    p = torch.nn.Parameter(torch.zeros(2))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = CosineAnnealing(opt, max_steps=100, min_lr=0.1, warmup_steps=10)
    lrs = []
    for _ in range(100):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    assert abs(lrs[0] - 0.1) < 1e-6 and abs(lrs[9] - 1.0) < 1e-6 and abs(lrs[-1] - 0.1) < 0.01
    assert all(lrs[i] >= lrs[i + 1] - 1e-9 for i in range(10, 99))

    class A:
        warmup_steps, max_steps = 4, 20

    opt2 = torch.optim.SGD([p], lr=2.0)
    s2 = get_learning_rate_scheduler(opt2, A())
    for _ in range(3):
        opt2.step()
        s2.step()
    assert abs(opt2.param_groups[0]["lr"] - 2.0) < 1e-6
    assert create_partition(32, 4) == ["model.layers.7", "model.layers.15", "model.layers.23"]
    assert create_partition(10, 4) == ["model.layers.1", "model.layers.3", "model.layers.6"]
    t = Throughput(batch_size=2, world_size=4, grad_accum_usteps=2, seq_len=128)
    assert t.get_throughput() > 0
    f = os.path.join(tempfile.mkdtemp(), "m.json")
    m = TrainingMetrics(f)
    m.store_parameters({"lr": 1e-4})
    from neuronx_distributed_llama3_2_amd.utils.training_utils import Metric

    m.store_metrics([Metric("Throughput", 12.5, "seq/s")])
    m.store_metrics([Metric("Loss", 2.0, "")])
    import json

    d = json.load(open(f))
    assert d["results"]["parameters"]["lr"] == 1e-4 and len(d["results"]["metrics"]) == 2
