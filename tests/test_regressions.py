"""Regression tests for the round-2 advisor findings: stale K-major dgrad weights after
DP=1 optimizer writes, single-writer xser saves on object stores, EP clip norms without ZeRO-1,
stale producer-written transposes, and pipeline exchange retirement by identity."""

import os
import tempfile

import torch
import torch.distributed as dist

from dist_utils import run_distributed


def _w_epoch(rank, world):
    from neuronx_distributed_llama3_2_amd.ops import gemm
    from neuronx_distributed_llama3_2_amd.optimizer.zero_redundancy_optimizer import NeuronZero1Optimizer
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    ps.initialize_model_parallel(tensor_model_parallel_size=1)
    assert ps.get_data_parallel_size() == 1
    lin = torch.nn.Linear(16, 8, bias=False)
    opt = NeuronZero1Optimizer(lin.parameters(), torch.optim.SGD, lr=0.1)
    lin(torch.randn(4, 16)).sum().backward()
    e0 = gemm._weight_epoch[0]
    opt.step()   # SGD through _GenericZero1 at DP=1: param_data written behind autograd's back
    assert gemm._weight_epoch[0] > e0, "K-major dgrad copies not invalidated by a DP=1 ZeRO-1 step"
    e1 = gemm._weight_epoch[0]
    opt.load_state_dict(opt.state_dict())
    assert gemm._weight_epoch[0] > e1
    lin2 = torch.nn.Linear(16, 8, bias=False)
    flat = FlatMixedPrecisionAdamW(lin2.parameters(), lr=0.1)
    e2 = gemm._weight_epoch[0]
    flat.load_state_dict(flat.state_dict())
    assert gemm._weight_epoch[0] > e2


def test_dp1_optimizer_writes_invalidate_kmajor_weights():
    run_distributed(_w_epoch, 1)


def _w_objstore(rank, world, root):
    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.trainer import checkpoint as ck
    from neuronx_distributed_llama3_2_amd.trainer.checkpoint_storage import (BaseCheckpointStorage,
                                                                             FilesysCheckpointStorage)

    class ObjectStore(BaseCheckpointStorage):
        """An S3-like store (not a filesystem): whole objects per key, last writer wins."""

        def __init__(self, d):
            super().__init__(d)
            self.fs = FilesysCheckpointStorage(d)

        def __getattribute__(self, name):
            if name in ("save_object",):
                def rec(obj, fn):
                    with open(os.path.join(root, f"writes.{dist.get_rank()}"), "a") as f:
                        f.write(fn + "\n")
                    return object.__getattribute__(self, "fs").save_object(obj, fn)
                return rec
            if name in ("file_exists", "dir_exists", "is_dir", "find_files", "save_text", "load_object",
                        "create_dir", "remove_dir", "remove_file", "list_checkpoint_tags", "get_latest_tag",
                        "is_checkpoint_xser"):
                return getattr(object.__getattribute__(self, "fs"), name)
            return object.__getattribute__(self, name)

    ck.create_checkpoint_storage = lambda d: ObjectStore(d)
    ps.initialize_model_parallel(tensor_model_parallel_size=1)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 32))
    nxd.save_checkpoint(os.path.join(root, "ck"), "t1", model=model, use_xser=True)
    nxd.finalize_checkpoint()


def test_xser_on_object_store_has_one_complete_writer():
    """DP-deduplicated xser writes only apply to filesystems; on an object store
    every replica would upload a partial object to the same key."""
    d = tempfile.mkdtemp()
    run_distributed(_w_objstore, 2, d)
    writes = {r: open(os.path.join(d, f"writes.{r}")).read().split() if os.path.exists(os.path.join(d, f"writes.{r}"))
              else [] for r in range(2)}
    model_writes = [(r, fn) for r, fns in writes.items() for fn in fns if "/model/" in fn]
    assert len(model_writes) == 1 and model_writes[0][0] == 0, writes
    sd = torch.load(os.path.join(d, "ck", model_writes[0][1]), weights_only=True)
    assert all(v.device.type == "cpu" for v in sd.values()), "placeholder tensors in the only object"
    assert set(sd) == {"0.weight", "0.bias", "1.weight", "1.bias"}


def _w_ep_norm(rank, world, out):
    from neuronx_distributed_llama3_2_amd.models.mixtral import MixtralForCausalLM, mixtral_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

    ps.initialize_model_parallel(tensor_model_parallel_size=1, expert_model_parallel_size=2)
    cfg = mixtral_config("tiny", capacity_factor=2.0)
    torch.manual_seed(0)
    model = MixtralForCausalLM(cfg, dtype=torch.float32)
    # master weights without ZeRO-1: whole buffers per rank, expert buffers hold this rank's experts
    opt = FlatMixedPrecisionAdamW(model.parameters(), lr=3e-3, zero1=False, grad_clipping=True, max_grad_norm=0.05)
    batch = torch.randint(0, cfg.vocab_size, (4, 32), generator=torch.Generator().manual_seed(3))
    norms = []
    for _ in range(3):
        local = batch.chunk(world)[rank]
        model(local, labels=local).loss.backward()
        opt.step()
        opt.zero_grad()
        n = torch.as_tensor(opt.grad_norm, dtype=torch.float32).reshape(1).clone()
        both = [torch.zeros(1) for _ in range(world)]
        dist.all_gather(both, n)
        norms.append([float(x) for x in both])
    # the replicated (non-expert) parameters stay identical across the EP ranks
    for name, p in model.named_parameters():
        if getattr(p, "expert_model_parallel", False):
            continue
        q = p.detach().clone()
        dist.broadcast(q, 0)
        assert torch.equal(q, p.detach()), name
    if rank == 0:
        torch.save(norms, out)


def test_ep_without_zero1_uses_one_global_norm():
    """without ZeRO-1 the expert part of the grad norm is summed over EP, so every
    EP rank clips with the same coefficient and the replicated dense params do not drift."""
    d = tempfile.mkdtemp()
    run_distributed(_w_ep_norm, 2, os.path.join(d, "n.pt"))
    for a, b in torch.load(os.path.join(d, "n.pt")):
        assert abs(a - b) <= 1e-6 * max(abs(a), 1.0), (a, b)


def test_stale_token_major_copy_is_ignored():
    """a producer-written transpose is not used once its tensor changed in place."""
    from neuronx_distributed_llama3_2_amd.ops.activations import attached_token_major
    from neuronx_distributed_llama3_2_amd.parallel_layers.layers import _token_major_copy

    h = torch.randn(8, 4)
    h._nxd_t, h._nxd_t_ver = h.t().contiguous(), h._version
    assert _token_major_copy(h) is h._nxd_t
    h.mul_(2.0)   # e.g. in-place dropout between SwiGLU and down_proj
    assert attached_token_major(h) is None and _token_major_copy(h) is None
    g = torch.randn(8, 4)
    g._nxd_t = g.t().contiguous()   # attached without a version record: never trusted
    assert attached_token_major(g) is None


def _w_p2p_empty(rank, world):
    from neuronx_distributed_llama3_2_amd.pipeline.comm import P2PGroup

    grp = P2PGroup()
    peer = 1 - rank
    bufs = []
    for i in range(3):   # three exchanges in flight, retired out of order
        t = torch.full((4,), float(rank * 10 + i))
        r = torch.empty(4)
        grp.send(t, peer)
        grp.recv(r, peer)
        grp.issue()
        bufs.append(r)
    grp.wait_for([bufs[1]])
    grp.wait_for([bufs[0]])
    grp.flush()
    for i, r in enumerate(bufs):
        assert torch.equal(r, torch.full((4,), float(peer * 10 + i)))


def test_p2p_retire_out_of_order():
    """retired exchanges are removed by identity (tuple == on emptied work lists
    would compare tensors element-wise)."""
    run_distributed(_w_p2p_empty, 2)
