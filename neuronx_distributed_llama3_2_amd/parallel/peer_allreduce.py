"""One-shot peer all-reduce for latency-bound tensor-parallel messages (csrc/peer_allreduce.hip).

Tensor-parallel decode all-reduces a few KiB per row-parallel projection (o_proj, down: M x H fp32).
Through RCCL each call is a ring of 2 (W - 1) link latencies plus a launch; here every rank exports one
device region (its IPC handle exchanged once over the process group), maps every peer's, and ONE kernel
per call publishes this rank's partial, waits for the peers' flags and sums all W partials in rank
order -- identical bits on every rank, no host involvement, capturable in the decode hipGraph.

Reference: the fork's TP decode compiles its all-reduces into one SPMD graph
(examples/inference/modules/gqa.py:641-647, src/neuronx_distributed/trace/spmd.py:82-187).

    par = PeerAllReduce(group, nmax=8 * hidden)
    par.sum_(partial, out, zero_in=True)             # out = sum over ranks; partial zeroed
    par.fold_residual_(partial, res, xadd)           # res = bf16(bf16(res + bf16(xadd)) + bf16(sum))
    par.set_residual_(partial, res)                  # res = bf16(sum)
    par.gather_(logits_slice, logits_full)           # [rows, C] per rank -> [rows, world * C]

`ProcessGroupAllReduce` has the same interface on torch.distributed (RCCL or gloo), the fallback when
IPC is not available (CPU, or NXD_DECODE_PEER_AR=0).
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

SUM, FOLD_RES, SET_RES = 0, 1, 2


class PeerAllReduce:
    def __init__(self, group=None, nmax: int = 65536):
        from ..ops._ext import ext

        self.C = ext()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 8:
            raise ValueError("peer all-reduce: at most 8 ranks (one node)")
        self.nmax = int(nmax)
        self.h = None
        # every step is collective and every rank reaches every collective, so a failure on any rank
        # (no IPC for this allocation, a handle that does not open) makes ALL ranks raise together
        err = None
        mine = None
        try:
            self.h, self.uncached = self.C.peer_ar_create(self.nmax)
            mine = self.C.peer_ar_ipc_handle(self.h)
        except Exception as e:
            err = repr(e)
        handles = [None] * self.world
        dist.all_gather_object(handles, mine, group=group)
        if err is None and all(h is not None for h in handles):
            try:
                self.C.peer_ar_open(self.h, self.rank, handles)
            except Exception as e:
                err = repr(e)
        elif err is None:
            err = "a peer could not export its buffer"
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=group)
        bad = [e for e in errs if e is not None]
        if bad:
            self.close()
            raise RuntimeError(f"peer all-reduce unavailable: {bad[0]}")
        self._failed = None
        self._calls = 0
        self._drop = _drop_spec(self.rank)
        # Before first use: a per-rank pattern through the REAL kernel and the IPC mappings, checked on
        # every rank.  This is what admits the coarse-grained fallback (no uncached IPC export) for a
        # group spread over several GPUs: visibility across devices then rests on the system-scope
        # fences alone, so it must be shown, not assumed.
        ok = self._self_test()
        oks = [None] * self.world
        dist.all_gather_object(oks, ok, group=group)
        if not all(oks):
            self.close()
            raise RuntimeError(f"peer all-reduce self-test failed on rank(s) {[r for r, o in enumerate(oks) if not o]} "
                               f"(uncached={bool(self.uncached)}); refusing the peer path")

    def _self_test(self) -> bool:
        n = min(self.nmax, 4096) // 4 * 4
        i = torch.arange(n, device="cuda", dtype=torch.float32)
        pat = lambda r: (r + 1) * 1000.0 + (i % 61)   # noqa: E731
        inp = pat(self.rank)
        out = torch.empty(n, device="cuda")
        self.C.peer_ar_set_spin_limit(self.h, 1 << 26)   # first launches may be far apart
        self.C.peer_ar_run(self.h, inp, False, SUM, out, None, None)
        torch.cuda.current_stream().synchronize()
        self.C.peer_ar_set_spin_limit(self.h, -1)
        want = sum(pat(r) for r in range(self.world))
        return bool(torch.equal(out, want)) and int(self.C.peer_ar_error(self.h)) == 0

    def _run(self, inp: torch.Tensor, zero_in: bool, mode: int, out=None, res=None, xadd=None):
        if inp.numel() > self.nmax or inp.numel() % 4:
            raise ValueError(f"peer all-reduce: {inp.numel()} elements (max {self.nmax}, multiple of 4)")
        if self._failed:
            raise RuntimeError(self._failed)
        self._calls += 1
        if self._drop is not None and self._calls == self._drop:
            return   # test hook (NXD_PEER_AR_DROP): this rank skips one call -- its peers must notice
        self.C.peer_ar_run(self.h, inp, zero_in, mode, out, res, xadd)

    def sum_(self, inp: torch.Tensor, out: torch.Tensor, zero_in: bool = False) -> torch.Tensor:
        self._run(inp, zero_in, SUM, out=out)
        return out

    def fold_residual_(self, inp: torch.Tensor, res: torch.Tensor, xadd: torch.Tensor, zero_in: bool = False):
        self._run(inp, zero_in, FOLD_RES, res=res, xadd=xadd)
        return res

    def set_residual_(self, inp: torch.Tensor, res: torch.Tensor, zero_in: bool = False):
        self._run(inp, zero_in, SET_RES, res=res)
        return res

    def gather_(self, inp: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """out [rows, world * C] = every rank's inp [rows, C] side by side (rank order); any dtype with
        16-byte rows (the vocab-parallel decode logits)."""
        if inp.numel() * inp.element_size() // 4 > self.nmax:
            raise ValueError("peer gather: slice larger than the exported region")
        self.C.peer_ar_gather(self.h, inp, out, self.world)
        return out

    def error_count(self) -> int:
        """Non-zero once some call lost a peer (bounded spin expired, or the peers' call sequences
        diverged).  A pinned host word: free to read, covers every call that has completed on the GPU."""
        return int(self.C.peer_ar_error(self.h)) if self.h else 0

    def check(self) -> None:
        """Raise if any completed call lost a peer.  Such a call wrote NaN outputs and the ranks' epochs
        no longer agree, so the handle stays failed: every later call raises too."""
        if self._failed:
            raise RuntimeError(self._failed)
        if self.error_count():
            self._failed = (f"peer all-reduce: a peer of rank {self.rank} never arrived or skipped a call (world "
                            f"{self.world}); the results of this step are invalid (NaN) and the group is unusable")
            raise RuntimeError(self._failed)

    def close(self) -> None:
        if getattr(self, "h", None):
            self.C.peer_ar_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


class ProcessGroupAllReduce:
    """The same operations on torch.distributed (RCCL graph-capturable; gloo host-staged)."""

    def __init__(self, group=None):
        self.group = group

    def sum_(self, inp: torch.Tensor, out: torch.Tensor, zero_in: bool = False) -> torch.Tensor:
        dist.all_reduce(inp, group=self.group)
        out.copy_(inp)
        if zero_in:
            inp.zero_()
        return out

    def fold_residual_(self, inp: torch.Tensor, res: torch.Tensor, xadd: torch.Tensor, zero_in: bool = False):
        dist.all_reduce(inp, group=self.group)
        y = (res.float() + xadd.reshape(res.shape).to(torch.bfloat16).float()).to(torch.bfloat16)
        res.copy_((y.float() + inp.reshape(res.shape).to(torch.bfloat16).float()).to(torch.bfloat16))
        if zero_in:
            inp.zero_()
        return res

    def set_residual_(self, inp: torch.Tensor, res: torch.Tensor, zero_in: bool = False):
        dist.all_reduce(inp, group=self.group)
        res.copy_(inp.reshape(res.shape))
        if zero_in:
            inp.zero_()
        return res

    def gather_(self, inp: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        parts = [torch.empty_like(inp) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(parts, inp.contiguous(), group=self.group)
        out.copy_(torch.cat(parts, dim=-1))
        return out

    def error_count(self) -> int:
        return 0

    def check(self) -> None:
        pass

    def close(self) -> None:
        pass


def _drop_spec(rank: int):
    """NXD_PEER_AR_DROP="r:k": rank r silently skips its k-th peer all-reduce call (the error-path
    tests inject a lost peer with it)."""
    import os

    spec = os.environ.get("NXD_PEER_AR_DROP", "")
    if not spec:
        return None
    r, k = spec.split(":")
    return int(k) if int(r) == rank else None


def make_decode_all_reduce(group, nmax: int, device: Optional[torch.device] = None, prefer_peer: bool = True):
    """The peer all-reduce when IPC works on this node, else the process-group one."""
    if prefer_peer and device is not None and torch.device(device).type == "cuda":
        try:
            return PeerAllReduce(group, nmax)
        except Exception as e:  # no IPC (e.g. a runtime without it): fall back, loudly
            from ..utils.logger import get_logger

            get_logger().warning("peer all-reduce unavailable (%s); decode all-reduces go through the process group", e)
    return ProcessGroupAllReduce(group)


class _PeerWork:
    """Async handle of a peer collective launched on the group's comm stream: wait() orders the
    current stream after it; the tensors stay referenced until then."""

    def __init__(self, event, keep):
        self.event, self.keep = event, keep

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        self.keep = None
        return True

    def is_completed(self):
        return self.event.query()


class PeerCollectives:
    """Sequence-parallel all-gather / reduce-scatter over the peer region (csrc/peer_allreduce.hip
    peer_coll_kernel): every rank publishes its input once and reads each peer's slot directly, so a
    node's 7 xGMI links all carry the gather at once, where a ring moves one hop per link
    step.  All calls of a group run on ONE comm stream (the host issue order, identical on every rank,
    is the execution order the epoch protocol relies on).  The region grows collectively -- every rank
    meets the same-sized first call at the same point -- after a device sync and a group barrier.
    Opt-in (NXD_SP_PEER=1, parallel/comm.py): measured on ranks sharing one GPU only."""

    def __init__(self, group=None):
        self.group = group
        self.par = None
        self.cap = 0
        self.stream = None

    def _ensure(self, nbytes: int) -> PeerAllReduce:
        if self.par is None or nbytes > self.cap:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("peer collectives: the region must be sized before graph capture "
                                   f"({nbytes} B requested, {self.cap} B mapped)")
            # every rank grows at the same call (same shapes everywhere); agree on the largest request
            # so no rank maps a smaller region than a peer will write
            probe = torch.tensor([int(nbytes)], dtype=torch.int64,
                                 device="cuda" if dist.get_backend(self.group) == "nccl" else "cpu")
            dist.all_reduce(probe, op=dist.ReduceOp.MAX, group=self.group)
            nbytes = int(probe.item())
            cap = max(1 << 20, 1 << (int(nbytes) - 1).bit_length())
            if self.par is not None:
                torch.cuda.synchronize()
                dist.barrier(group=self.group)
                self.par.check()
                self.par.close()
            self.par = PeerAllReduce(self.group, nmax=cap // 4)
            self.cap = cap
            if self.stream is None:
                self.stream = torch.cuda.Stream(priority=-1)
        return self.par

    def _launch(self, inp, out, mode, nbytes, async_op):
        par = self._ensure(nbytes)
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            par.C.peer_coll(par.h, inp, out, mode)
        if async_op:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            return _PeerWork(ev, (inp, out))
        cur.wait_stream(self.stream)
        return None

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        inp = inp.contiguous()
        return self._launch(inp, out, 0, inp.numel() * inp.element_size(), async_op)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        inp = inp.contiguous()
        return self._launch(inp, out, 1, inp.numel() * inp.element_size(), async_op)

    def error_count(self) -> int:
        return self.par.error_count() if self.par is not None else 0

    def check(self) -> None:
        if self.par is not None:
            self.par.check()
