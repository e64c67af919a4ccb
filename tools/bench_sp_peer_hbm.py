"""HBM-side cost of the direct-peer sequence-parallel collectives (parallel/peer_allreduce.py
PeerCollectives, NXD_SP_PEER=1) at the TP=8 SP message sizes, with W ranks sharing ONE GPU: every
rank's publish copy and peer reads then hit the same HBM, so the per-call time over the bytes all W
ranks move is the kernel's streaming efficiency (no xGMI link is involved).  A same-size device
copy by one process is the reference rate.  RCCL cannot be A/B'd here: it refuses two ranks on one
device.

    python tools/bench_sp_peer_hbm.py --world 8          # spawns the ranks (gloo group for set-up)
Rank 0 prints one JSON line per (op, shard MiB)."""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker():
    import torch
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.parallel.peer_allreduce import PeerCollectives

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pc = PeerCollectives(None)
    reps = 10
    for mib in (1, 4, 8):   # per-rank shard: 8 MiB = one [1024, 4096] bf16 SP shard at TP=8, S=8192
        n = mib * 2**20 // 2
        shard = torch.randn(n, device="cuda").to(torch.bfloat16)
        full = torch.empty(world * n, dtype=torch.bfloat16, device="cuda")
        for op in ("all_gather", "reduce_scatter"):
            def call():
                if op == "all_gather":
                    pc.all_gather(full, shard)
                else:
                    pc.reduce_scatter(shard, full)
            call()
            torch.cuda.synchronize()
            dist.barrier()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                call()
            e.record()
            torch.cuda.synchronize()
            ms = torch.tensor([s.elapsed_time(e) / reps])
            dist.all_reduce(ms, op=dist.ReduceOp.MAX)
            pc.check() if hasattr(pc, "check") else None
            # bytes through HBM per call, all ranks: AG publish (read+write shard) + pull world shards
            # (read) + write out; RS publish world shards (read+write) + read world slices + write shard
            sb = n * 2
            per_rank = (2 * sb + world * sb + world * sb) if op == "all_gather" else (2 * world * sb + world * sb + sb)
            tot = per_rank * world
            if rank == 0:
                a = torch.empty(tot // 4, dtype=torch.uint8, device="cuda")
                b = torch.empty_like(a)
                b.copy_(a)
                torch.cuda.synchronize()
                s.record()
                for _ in range(reps):
                    b.copy_(a)
                e.record()
                torch.cuda.synchronize()
                cms = s.elapsed_time(e) / reps * 2   # a copy moves 2x its size; tot/4 copied = tot/2 moved -> x2
                print(json.dumps({"op": op, "world": world, "shard_mib": mib, "ms_per_call": round(ms.item(), 4),
                                  "hbm_bytes_all_ranks": tot, "tb_s": round(tot / ms.item() / 1e9, 2),
                                  "device_copy_same_bytes_ms": round(cms, 4)}), flush=True)
                del a, b
            dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    if "RANK" in os.environ:
        return worker()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)],
                              env=dict(os.environ, RANK=str(r), WORLD_SIZE=str(a.world), MASTER_ADDR="127.0.0.1",
                                       MASTER_PORT=port))
             for r in range(a.world)]
    rcs = [p.wait(timeout=600) for p in procs]
    sys.exit(max(abs(rc) for rc in rcs))


if __name__ == "__main__":
    main()
