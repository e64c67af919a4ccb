"""Multi-process CPU (gloo) harness: run a function on N ranks with real torch.distributed
collectives, propagate failures (the reference has no such harness)."""

import os
import socket
import tempfile
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, errfile):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fn(rank, world, *args)
    except Exception:  # pragma: no cover - reported to parent
        with open(errfile + f".{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
        from neuronx_distributed_llama3_2_amd.modules.qkv_linear import destroy_kv_group

        ps.destroy_model_parallel()
        destroy_kv_group()
        if dist.is_initialized():
            dist.destroy_process_group()


def run_distributed(fn, world_size: int, *args):
    errfile = tempfile.mktemp(prefix="nxd_dist_err_")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, fn, args, errfile)) for r in range(world_size)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    errs = []
    for r in range(world_size):
        fn_ = errfile + f".{r}"
        if os.path.exists(fn_):
            errs.append(f"rank {r}:\n" + open(fn_).read())
            os.remove(fn_)
    for p in procs:
        if p.is_alive():
            p.kill()
            errs.append(f"rank process {p.pid} timed out")
    if errs or any(p.exitcode != 0 for p in procs):
        raise AssertionError("distributed test failed:\n" + "\n".join(errs) + f"\nexit codes {[p.exitcode for p in procs]}")
