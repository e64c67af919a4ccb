"""One tensor-parallel rank of the multi-GPU bench, emulated on ONE GPU without its peers.

torch.distributed runs on the in-process "fake" backend with world size = TP and this process as
rank 0, so the model is built and stepped exactly as `bench.py --gpus TP` builds it on a node:
the real TP shards (32/TP q heads, 8/TP kv heads, FFN and vocabulary split), sequence-parallel
activations (RMSNorm, residual adds and embeddings on S/TP rows, the chunked all-gather -> GEMM
and GEMM -> reduce-scatter pipelines of parallel_layers/sp.py), the vocabulary-parallel embedding
and cross-entropy, fp32-master AdamW with the global grad-norm clip.  Only the links are missing:
each collective is replaced by the local HBM work it does on the receiving side (an all-gather
writes the whole output buffer -- filled with copies of the local shard so values stay finite --
a reduce-scatter writes its shard, an all-reduce leaves the tensor as is).

The step time is therefore the per-rank compute floor of the N-GPU bench; tokens/s = global batch
x sequence / step time is the whole-node throughput at perfect communication overlap.  It is not
a throughput claim (the driver's node run is).

    python tools/emulate_tp_rank.py --tp 8 --steps 3 --warmup 1
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuronx_distributed_llama3_2_amd.parallel import comm  # noqa: E402


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


class _Link:
    """Optional link-time model (--link-gbps B): every collective runs on one high-priority side
    stream (RCCL's per-communicator stream) after the producer's work, as a spin of
    bytes-on-the-wire / B followed by its receiving-side write; the consumer waits on it.  Ring
    bytes per rank: all-gather / reduce-scatter (n-1)/n of the full tensor, all-reduce twice that.

    The spin is csrc/diag.hip `cu_stream`: `--link-cus K` workgroups (default 1; RCCL runs one per
    channel) stream a small buffer until the 100 MHz real-time counter has advanced by the link
    time -- wall-clock based, so it is not stretched when the shader clock drops under MFMA load
    (the round-3 model spun torch.cuda._sleep on the shader-clock cycle counter, calibrated idle).

    Buffer lifetime (--sync stash, default): the collective's tensors are held by the handle until
    wait() has made the consumer's stream wait for the link stream, then dropped -- what
    ProcessGroupNCCL does with TORCH_NCCL_AVOID_RECORD_STREAMS=1 (parallel/rccl_env.py).  --sync
    record reproduces the round-3 model: record_stream() onto the link stream, which keeps every
    freed block out of the allocator until the GPU has passed an event the CPU enqueued far ahead
    (profiles/r4_emulate_stall.jsonl measures what that did)."""

    def __init__(self, gbps: float, cus: int = 1, spin: str = "realtime"):
        from neuronx_distributed_llama3_2_amd.ops import ext

        self.C = ext()
        self.spin = spin
        if spin == "sleep":   # round-3 model: shader-clock cycles, calibrated on an idle GPU
            torch.cuda._sleep(1000)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.cuda._sleep(10_000_000)
            e1.record()
            torch.cuda.synchronize()
            self.cycles_per_s = 10_000_000 / (e0.elapsed_time(e1) / 1e3)
        self.bps = gbps * 1e9
        self.cus = max(1, int(cus))
        self.stream = torch.cuda.Stream(priority=-1)
        self.copy_stream = torch.cuda.Stream(priority=-1)
        self.src = torch.zeros(self.cus * 4096, dtype=torch.uint8, device="cuda")
        self.dst = torch.empty_like(self.src)
        self.busy_s = 0.0

    def run(self, nbytes: float, work):
        """Spin for the link time on the link stream and do the receiving-side write on a second
        side stream, both after the producer: RCCL writes the output while it transfers, so the
        write must not queue behind the spin (round-4 first traces serialised them: the copies
        added ~40 % to the link stream's busy time, profiles/r4_stream_timeline_8layers.jsonl)."""
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        self.copy_stream.wait_stream(cur)
        t = nbytes / self.bps
        self.busy_s += t
        with torch.cuda.stream(self.stream):
            if self.spin == "sleep":
                torch.cuda._sleep(max(1, int(t * self.cycles_per_s)))
            else:
                self.C.cu_stream(self.src, self.dst, 4096, self.cus, max(1, int(t * 1e8)))
        with torch.cuda.stream(self.copy_stream):
            work()
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.stream.wait_stream(self.copy_stream)   # the handle's event covers the write too
        ev2 = torch.cuda.Event()
        ev2.record(self.stream)
        return ev2


_LINK = None
_SYNC = "stash"


class _Pending:
    def __init__(self, ev, tensors):
        self.ev, self.tensors = ev, tensors

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)
            if _SYNC == "record":   # allocated on the compute stream, written on the link stream
                for t in self.tensors:
                    t.record_stream(torch.cuda.current_stream())
            self.ev = None
            self.tensors = None     # stash released: the consumer's stream is now ordered after the link
        return True

    def is_completed(self):
        return self.ev is None or self.ev.query()


def _collective(nbytes, work, async_op, tensors):
    if _LINK is None or not tensors[0].is_cuda:
        work()
        return _Done() if async_op else None
    if _SYNC == "record":
        for t in tensors:
            t.record_stream(_LINK.stream)
            t.record_stream(_LINK.copy_stream)
    h = _Pending(_LINK.run(nbytes, work), tensors)
    if async_op:
        return h
    h.wait()
    return None


def _emulate_collectives():
    """Receiving-side HBM work of each collective, no links unless --link-gbps (module docstring)."""

    def all_gather_into_tensor(out, inp, group=None, async_op=False):
        ws = dist.get_world_size(group=group)
        inp = inp.contiguous()

        def work():
            out.view((ws,) + tuple(inp.shape)).copy_(inp.unsqueeze(0).expand((ws,) + tuple(inp.shape)))

        return _collective(out.numel() * out.element_size() * (ws - 1) / ws, work, async_op, [out, inp])

    def reduce_scatter_tensor(out, inp, group=None, async_op=False, op=dist.ReduceOp.SUM):
        ws = dist.get_world_size(group=group)
        inp = inp.contiguous()

        def work():
            out.copy_(inp.view((ws,) + tuple(out.shape))[0])

        return _collective(inp.numel() * inp.element_size() * (ws - 1) / ws, work, async_op, [out, inp])

    def all_reduce(t, group=None, async_op=False, op=dist.ReduceOp.SUM):
        ws = dist.get_world_size(group=group)
        return _collective(2 * t.numel() * t.element_size() * (ws - 1) / ws, lambda: None, async_op, [t])

    def all_reduce_coalesced(tensors, group=None):
        tensors = [t for t in tensors if t.numel()]
        if tensors:
            ws = dist.get_world_size(group=group)
            nbytes = sum(2 * t.numel() * t.element_size() * (ws - 1) / ws for t in tensors)
            _collective(nbytes, lambda: None, False, tensors)

    comm.all_gather_into_tensor = all_gather_into_tensor
    comm.reduce_scatter_tensor = reduce_scatter_tensor
    comm.all_reduce = all_reduce
    comm.all_reduce_coalesced = all_reduce_coalesced


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--layers", type=int, default=None, help="override #layers (default: the full model)")
    ap.add_argument("--mbs", type=int, default=None, help="default: bench.py's MBS_BY_TP")
    ap.add_argument("--gbs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-sp", action="store_true")
    ap.add_argument("--ckpt", default=None, choices=[None, "selective", "full"], help="activation checkpointing")
    ap.add_argument("--cpu", action="store_true", help="plumbing check on the CPU (tiny models)")
    ap.add_argument("--hidden", type=int, default=None, help="(CPU plumbing) override hidden size")
    ap.add_argument("--link-gbps", type=float, default=None,
                    help="model collective time at this per-rank ring bandwidth (GB/s) on a side stream")
    ap.add_argument("--link-cus", type=int, default=1, help="workgroups the link spin occupies (RCCL channels)")
    ap.add_argument("--sync", choices=["stash", "record"], default="stash",
                    help="collective buffer lifetime: stash until wait() (RCCL default) or record_stream")
    ap.add_argument("--spin", choices=["realtime", "sleep"], default="realtime",
                    help="link spin: real-time-counter copy kernel, or round-3's torch.cuda._sleep")
    ap.add_argument("--sp-stagger", type=int, default=None, help="NXD_SP_STAGGER for this run")
    ap.add_argument("--sp-streams", type=int, default=None, help="NXD_SP_STREAMS for this run (1 = one pass, k >= 2 parts)")
    a = ap.parse_args()

    from torch.testing._internal.distributed.fake_pg import FakeStore

    import bench
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
    from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW
    from neuronx_distributed_llama3_2_amd.parallel.grad_buffer import find_shared_params
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed

    use_cuda = torch.cuda.is_available() and not a.cpu
    dev = torch.device("cuda", 0) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(0)
    dist.init_process_group("fake", rank=0, world_size=a.tp, store=FakeStore())
    _emulate_collectives()
    global _LINK, _SYNC
    _SYNC = a.sync
    if a.sp_streams is not None:
        from neuronx_distributed_llama3_2_amd.parallel_layers import stream_split

        stream_split.set_enabled(a.sp_streams >= 2, a.sp_streams)
    if a.sp_stagger is not None:
        from neuronx_distributed_llama3_2_amd.parallel_layers import stream_split

        stream_split.set_stagger(a.sp_stagger)
    if a.link_gbps and use_cuda:
        _LINK = _Link(a.link_gbps, a.link_cus, a.spin)
    ps.initialize_model_parallel(tensor_model_parallel_size=a.tp)
    model_parallel_manual_seed(1234)
    over = dict(sequence_parallel_enabled=(a.tp > 1 and not a.no_sp), max_position_embeddings=max(8192, a.seq))
    if a.layers is not None:
        over["num_hidden_layers"] = a.layers
    if a.ckpt == "full":
        over["activation_checkpoint"] = "full"
    elif a.ckpt == "selective":
        over["selective_checkpoint_enabled"] = True
    if a.hidden is not None:
        over.update(hidden_size=a.hidden, intermediate_size=4 * a.hidden, vocab_size=1024 * a.tp)
    cfg = llama_config(a.model, **over)
    mbs = a.mbs if a.mbs is not None else bench.MBS_BY_TP.get(a.tp, 1)
    accum = a.gbs // mbs
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=dev)
    model.train()
    decay = [p for n, p in model.named_parameters() if p.dim() > 1]
    no_decay = [p for n, p in model.named_parameters() if p.dim() <= 1]
    opt = FlatMixedPrecisionAdamW([{"params": decay, "weight_decay": 0.01}, {"params": no_decay, "weight_decay": 0.0}],
                                  lr=1e-5, betas=(0.9, 0.95), eps=1e-8, zero1=False, grad_clipping=True,
                                  max_grad_norm=1.0, shared_param_ids=find_shared_params(model))
    g = torch.Generator(device="cpu").manual_seed(4321)
    n_mb = (a.warmup + a.steps) * accum
    batches = torch.randint(0, cfg.vocab_size, (n_mb, mbs, a.seq), generator=g).to(dev)
    cursor = [0]

    def step():
        for i in range(accum):
            opt.set_grad_sync(i == accum - 1)
            ids = batches[cursor[0]]
            cursor[0] += 1
            out = model(ids, labels=ids)
            (out.loss / accum).backward()
        opt.step()
        opt.zero_grad()

    for _ in range(a.warmup):
        step()
    if use_cuda:
        torch.cuda.synchronize()
        ms0 = torch.cuda.memory_stats(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    if use_cuda:
        torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps
    mem = {}
    if use_cuda:
        ms1 = torch.cuda.memory_stats(dev)
        # allocator events inside the timed steps (retries = OOM -> free cached blocks -> retry,
        # each a device-wide synchronisation; device allocs = fresh hipMalloc calls)
        mem = {k: ms1.get(k, 0) - ms0.get(k, 0) for k in ("num_alloc_retries", "num_sync_all_streams",
                                                            "num_device_alloc", "num_device_free")}
        mem["num_alloc_retries_total"] = ms1.get("num_alloc_retries", 0)
        mem["peak_reserved_gib"] = round(torch.cuda.max_memory_reserved(dev) / 2**30, 1)
    rec = {"tool": "emulate_tp_rank", "tp": a.tp, "sp": over["sequence_parallel_enabled"], "model": a.model,
           "layers": cfg.num_hidden_layers, "seq": a.seq, "mbs": mbs, "gbs": a.gbs, "grad_accum": accum,
           "sp_chunks": __import__("neuronx_distributed_llama3_2_amd.parallel_layers.sp", fromlist=["x"])
           .get_sequence_parallel_chunks(a.tp), "link_gbps": a.link_gbps,
           "link_cus": a.link_cus if _LINK else None, "gemm_no_streamk": os.environ.get("NXD_GEMM_NO_STREAMK", "0"), "spin": a.spin if _LINK else None, "sync": a.sync,
           "sp_streams": __import__("neuronx_distributed_llama3_2_amd.parallel_layers.stream_split",
                                     fromlist=["x"]).parts(),
           "sp_stagger": __import__("neuronx_distributed_llama3_2_amd.parallel_layers.stream_split",
                                    fromlist=["x"])._STAGGER,
           "link_busy_ms_per_step": round(1000 * _LINK.busy_s / (a.warmup + a.steps), 2) if _LINK else None,
           "ms_per_step": round(1000 * el, 2), "ms_per_microbatch": round(1000 * el / accum, 2),
           "node_tokens_per_s_comm_free": round(a.gbs * a.seq / el, 1),
           "params_per_rank": sum(p.numel() for p in model.parameters()),
           "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if use_cuda else 0.0, **mem}
    if use_cuda:
        from neuronx_distributed_llama3_2_amd.utils.memory_planner import plan_training_memory

        plan = plan_training_memory(cfg, tp=a.tp, mbs=mbs, seq=a.seq, sequence_parallel=over["sequence_parallel_enabled"],
                                    activation_checkpoint=a.ckpt, zero1=False)
        rec["ckpt"] = a.ckpt
        rec["planner_gib"] = round(plan.total_bytes / 2**30, 1)
        rec["planner_err_pct"] = round(100 * (plan.total_bytes / 2**30 - rec["peak_mem_gib"]) / rec["peak_mem_gib"], 1)
    print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
