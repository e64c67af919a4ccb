"""Worker of tests/test_peer_allreduce_gpu.py::test_peer_allreduce_lost_peer_raises: rank 1 silently
skips its 3rd call (NXD_PEER_AR_DROP=1:3).  Rank 0's 3rd call times out (small NXD_PEER_AR_SPIN_LIMIT):
NaN outputs and check() raises; rank 1's next call reads rank 0's poisoned flags and fails too.
Each rank writes {calls_ok, raised_at, nan_output} to argv[1].rank."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.parallel.peer_allreduce import PeerAllReduce  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = PeerAllReduce(None, nmax=4096)
    rec = {"calls_ok": 0, "raised_at": None, "nan_output": False, "error": None}
    n = 2048
    for call in range(1, 6):
        inp = torch.full((n,), float(rank + 1), device="cuda")
        out = torch.zeros(n, device="cuda")
        try:
            par.sum_(inp, out)
            torch.cuda.synchronize()
            par.check()
        except RuntimeError as e:
            rec["raised_at"] = call
            rec["nan_output"] = bool(torch.isnan(out).all().item())
            rec["error"] = str(e)[:200]
            break
        if call == 3 and rank == 1:
            # the straggler comes back late (after rank 0's bounded spin), as a hung rank would; one that
            # came back within the spin would publish the very epoch rank 0 waits for (the sequences
            # re-align by one call: undetectable by epochs alone)
            time.sleep(1.0)
        if call != 3 or rank != 1:   # rank 1's dropped call leaves out untouched
            assert torch.equal(out, torch.full((n,), float(world * (world + 1) // 2), device="cuda")), call
        rec["calls_ok"] += 1
    with open(f"{sys.argv[1]}.{rank}", "w") as f:
        json.dump(rec, f)
    # the group is unusable now: every later call raises without launching
    try:
        par.sum_(torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda"))
        raise SystemExit("a failed handle accepted another call")
    except RuntimeError:
        pass
    dist.barrier()
    par.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
