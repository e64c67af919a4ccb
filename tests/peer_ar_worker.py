"""Worker of tests/test_peer_allreduce_gpu.py: one rank of W processes sharing cuda:0 (gloo for the
IPC-handle exchange only).  Checks the peer all-reduce's three modes bitwise against a local
recomputation of every rank's partial (rank-order fp32 sum), eager and inside a replayed hipGraph,
and times eager calls.  Rank 0 writes a JSON summary to argv[1]."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.parallel.peer_allreduce import PeerAllReduce  # noqa: E402


def partial(it, r, n):
    g = torch.Generator(device="cuda").manual_seed(1000 * it + r)
    return torch.randn(n, device="cuda", generator=g)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = PeerAllReduce(None, nmax=8 * 4096)
    checks = 0
    sizes = [2048, 8192, 32768, 4000, 12]
    for it in range(40):
        n = sizes[it % len(sizes)]
        parts = [partial(it, r, n) for r in range(world)]
        want = torch.zeros(n, device="cuda")
        for p in parts:
            want += p
        inp = parts[rank].clone()
        mode = it % 3
        g = torch.Generator(device="cuda").manual_seed(77 + it)
        res0 = torch.randn(n, device="cuda", generator=g).to(torch.bfloat16)
        xadd = torch.randn(n, device="cuda", generator=g)
        if mode == 0:
            out = torch.empty(n, device="cuda")
            par.sum_(inp, out, zero_in=True)
            assert torch.equal(out, want), (it, (out - want).abs().max())
            assert not inp.any()
        elif mode == 1:
            res = res0.clone()
            par.fold_residual_(inp, res, xadd)
            y = (res0.float() + xadd.to(torch.bfloat16).float()).to(torch.bfloat16)
            exp = (y.float() + want.to(torch.bfloat16).float()).to(torch.bfloat16)
            assert torch.equal(res, exp), it
        else:
            res = res0.clone()
            par.set_residual_(inp, res)
            assert torch.equal(res, want.to(torch.bfloat16)), it
        checks += 1
    # the vocab-parallel logits gather (bf16 bytes, rank order)
    for it in range(6):
        rows, C = 1 + it % 4, 1000 + 8 * it
        sl = [partial(900 + it, r, rows * C).to(torch.bfloat16).view(rows, C) for r in range(world)]
        out = torch.empty(rows, world * C, dtype=torch.bfloat16, device="cuda")
        par.gather_(sl[rank].clone(), out)
        assert torch.equal(out, torch.cat(sl, dim=1)), it
        checks += 1
    # sequence-parallel all-gather / reduce-scatter (PeerCollectives: its own region, comm stream,
    # async handles, region growth)
    from neuronx_distributed_llama3_2_amd.parallel.peer_allreduce import PeerCollectives

    pc = PeerCollectives(None)
    for it, (n, dt) in enumerate([(4096, torch.bfloat16), (1 << 19, torch.bfloat16), (8, torch.float32),
                                  (3 << 16, torch.float32), (1 << 20, torch.bfloat16)]):
        shards = [partial(700 + it, r, n).to(dt) for r in range(world)]
        out = torch.empty(world * n, dtype=dt, device="cuda")
        w = pc.all_gather(out, shards[rank].clone(), async_op=bool(it % 2))
        if w is not None:
            w.wait()
        assert torch.equal(out, torch.cat(shards)), ("ag", it)
        fulls = [partial(800 + it, r, world * n).to(dt) for r in range(world)]
        want = torch.zeros(n, device="cuda")
        for f in fulls:
            want += f[rank * n:(rank + 1) * n].float()
        rs = torch.empty(n, dtype=dt, device="cuda")
        w = pc.reduce_scatter(rs, fulls[rank].clone(), async_op=not bool(it % 2))
        if w is not None:
            w.wait()
        assert torch.equal(rs, want.to(dt)), ("rs", it)
        checks += 1
    errs_coll = pc.error_count()
    # inside a hipGraph: 4 calls per replay (an even and an odd count of calls between replays)
    n = 2048
    sin = torch.zeros(4, n, device="cuda")
    sout = torch.zeros(4, n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for k in range(3):                      # warm-up on the capture stream (odd number of calls)
            par.sum_(sin[k], sout[k])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for k in range(4):
            par.sum_(sin[k], sout[k])
    dist.barrier()
    for rep in range(10):
        for k in range(4):
            sin[k].copy_(partial(500 + 4 * rep + k, rank, n))
        torch.cuda.synchronize()
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        for k in range(4):
            want = torch.zeros(n, device="cuda")
            for r in range(world):
                want += partial(500 + 4 * rep + k, r, n)
            assert torch.equal(sout[k], want), (rep, k)
        checks += 1
        dist.barrier()
    # eager latency of back-to-back calls (both processes share the GPU here: an upper bound)
    x = torch.randn(n, device="cuda")
    out = torch.empty(n, device="cuda")
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(200):
        par.sum_(x, out)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 200 * 1e6
    errs = par.error_count() + errs_coll
    dist.barrier()
    if rank == 0:
        with open(sys.argv[1], "w") as f:
            json.dump({"world": world, "checks": checks, "errors": errs, "uncached": bool(par.uncached),
                       "eager_us_per_call_n2048": round(us, 2)}, f)
    par.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
