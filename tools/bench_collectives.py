"""Collective bandwidth on N ranks of one node: all-gather, reduce-scatter, all-reduce at 8 and
64 MiB (the SP activation sizes of Llama-3-8B at S=8192: one 64 MiB [8192, 4096] bf16 tensor per
TP collective) and a bidirectional neighbour p2p exchange (the pipeline boundary pattern).
Bus bandwidth follows the nccl-tests convention (AG/RS: algbw*(n-1)/n, AR: algbw*2(n-1)/n).

    python tools/bench_collectives.py --gpus N            # spawns N ranks (RCCL on GPUs)
    python tools/bench_collectives.py --gpus 2 --cpu      # gloo plumbing check
Rank 0 prints one JSON line per (op, size); every line records the RCCL environment in effect.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(a):
    import torch
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.parallel import comm
    from neuronx_distributed_llama3_2_amd.parallel.rccl_env import apply_rccl_env, comm_config

    apply_rccl_env()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    cuda = torch.cuda.is_available() and not a.cpu
    if cuda:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)))
    dev = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    dist.init_process_group("nccl" if cuda else "gloo", rank=rank, world_size=world,
                            device_id=dev if cuda else None)

    def sync():
        if cuda:
            torch.cuda.synchronize()
        dist.barrier()

    def timeit(fn, iters):
        fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        sync()
        return (time.perf_counter() - t0) / iters

    for mib in a.sizes:
        n = mib * 2**20 // 2   # bf16 elements of the FULL tensor
        n -= n % world
        full = torch.randn(n, dtype=torch.bfloat16, device=dev)
        shard = torch.randn(n // world, dtype=torch.bfloat16, device=dev)
        nbytes = n * 2
        res = {}
        t = timeit(lambda: comm.all_gather_into_tensor(full, shard), a.iters)
        res["all_gather"] = (t, nbytes / t, nbytes / t * (world - 1) / world)
        t = timeit(lambda: comm.reduce_scatter_tensor(shard, full), a.iters)
        res["reduce_scatter"] = (t, nbytes / t, nbytes / t * (world - 1) / world)
        t = timeit(lambda: comm.all_reduce(full), a.iters)
        res["all_reduce"] = (t, nbytes / t, nbytes / t * 2 * (world - 1) / world)
        if world > 1:
            send_buf = torch.randn(n // world, dtype=torch.bfloat16, device=dev)
            recv_l = torch.empty_like(send_buf)
            recv_r = torch.empty_like(send_buf)

            def p2p():
                ops = [dist.P2POp(dist.isend, send_buf, (rank + 1) % world),
                       dist.P2POp(dist.irecv, recv_l, (rank - 1) % world),
                       dist.P2POp(dist.isend, send_buf, (rank - 1) % world),
                       dist.P2POp(dist.irecv, recv_r, (rank + 1) % world)]
                for w in dist.batch_isend_irecv(ops):
                    w.wait()

            t = timeit(p2p, a.iters)
            pb = send_buf.numel() * 2 * 2   # bytes sent per rank (both neighbours)
            res["p2p_neighbours"] = (t, pb / t, pb / t)
        if rank == 0:
            for op, (t, alg, bus) in res.items():
                print(json.dumps({"op": op, "size_mib": mib, "ranks": world, "backend": dist.get_backend(),
                                  "us": round(t * 1e6, 1), "algbw_gbs": round(alg / 1e9, 2),
                                  "busbw_gbs": round(bus / 1e9, 2), "env": comm_config()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=2)
    ap.add_argument("--sizes", type=int, nargs="+", default=[8, 64], help="MiB of the full tensor")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    if "WORLD_SIZE" in os.environ:
        worker(a)
        return
    port = str(_free_port())
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    for p in procs:
        rc = rc or p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
