"""Two-stream micro-batch interleaving for tensor + sequence parallel training.

Why: at TP = 8 the SP collectives of one Llama-3-8B layer move as many bytes per token as the
layer's GEMMs take time (8 all-gathers / reduce-scatters of hidden x 2 B per token and layer), and
inside ONE sequence the chunked GEMM <-> collective pipelines of `sp.py` can only hide a
collective behind the GEMM that consumes or produces it -- attention, norms and SwiGLU leave the
links idle and the next collective waits for them.  An emulated TP=8 rank with a 400 GB/s link
model (tools/emulate_tp_rank.py --link-gbps 400) spends 603 ms per step against 388 ms of compute
and 305 ms of link time.

How: the micro-batch is split into two halves whose forward passes are issued alternately, one
collective-bearing op at a time, each half on its own HIP stream.  The single RCCL stream then
carries A's all-gather, B's all-gather, A's reduce-scatter, ... while the compute streams run the
other half's attention / MLP.  Autograd runs every backward op on its forward op's stream and
orders the ready ops by creation, so the backward interleaves the same way with no extra code.

Shared state the two streams write is serialised here:
* fp32 `main_grad` accumulation (weight-gradient GEMMs with beta = 1, RMSNorm dw): a per-parameter
  event orders the two halves' read-modify-writes (`accumulate_begin` / `accumulate_end`);
* the lazily built K-major weight copies and the wgrad transposes' scratch (ops/gemm.py) and the
  hipBLASLt workspace (csrc/gemm.cpp) are per stream or event-ordered;
* `join()` makes the caller's stream wait for both halves (the optimizer step calls it).

Active only while training with TP > 1, sequence parallelism, DP = 1 (the backward-overlapped DP
bucket reduction counts one gradient report per parameter) and no full activation checkpointing;
NXD_SP_STREAMS=k (k >= 2) turns it on with k parts of the micro-batch on k streams (the largest
divisor of the micro-batch <= k); off (1) by default until it has run on a multi-GPU node.  Checked:
fp32 CPU parity with the one-pass step (tests/test_stream_split.py, TP=2 and TP=4 replicated kv);
on the GPU kernels (one-GPU gloo rehearsal, TP=4 replicated kv, 4 AdamW steps, three runs each)
bit-identical from run to run and within 3e-4 of the one-pass losses / grad norms
(profiles/r3_sp_streams_noise_default_gemm.jsonl).  The run-to-run variation first seen there came
from the (then unvalidated) exhaustive GEMM search, not from the streams
(profiles/r3_sp_streams_noise_nosk_exhaustive.jsonl).
"""

from __future__ import annotations

import os
from typing import Generator, List, Sequence

import torch

_MODE = os.environ.get("NXD_SP_STREAMS", "1")
# phase offset between the parts: part i starts after part 0 has taken i * STAGGER steps (one step =
# one collective-bearing op of a decoder layer: qkv all-gather, o_proj reduce-scatter, gate_up
# all-gather, down reduce-scatter).  0 = strict alternation; 2 (default) puts one part's MLP beside
# the other part's attention.  Emulated ranks, stagger 2 vs 0 (profiles/r4_emulate_sp_stagger.jsonl):
# TP=8 at 400 GB/s 516 vs 518 ms, without links 386 vs 397; TP=4 at 200 GB/s 898 vs 931; TP=2 at
# 70 GB/s 1,753 vs 1,801.
_STAGGER = int(os.environ.get("NXD_SP_STAGGER", "2") or 0)
_active = False           # inside an interleaved forward/backward (set until join())
_streams = {}             # device index -> [stream A, stream B]


_NO_SP = os.environ.get("NXD_SP_STREAMS_NO_SP", "0") == "1"
# NXD_SP_RESERVE_CUS=n: the parts' streams are CU-masked to leave n CUs (spread over the XCDs) to the
# collectives, whose kernels otherwise wait for a compute workgroup to retire before they can start
# (every heavy kernel holds whole CUs: 256-thread workgroups at the register / LDS maximum).
# Measured slower, off: emulated TP=8 without links 387 -> 467 ms with 8 CUs masked off (far more
# than the 3 % of CUs), 518 -> 557 at 400 GB/s (profiles/r4_emulate_cu_masked_streams.jsonl).
_RESERVE = int(os.environ.get("NXD_SP_RESERVE_CUS", "0") or 0)


def reserved_cus(n: int, ncu: int = 256) -> List[int]:
    """n CU indices spread over the 8 XCDs whether the mask bits are XCD-major (32 per XCD) or
    XCD-interleaved (bit i on XCD i % 8): index 32 j + j (+ 8 k) lands on XCD j either way."""
    per = ncu // 8
    out = []
    for k in range((n + 7) // 8):
        for j in range(8):
            if len(out) < n:
                out.append(per * j + j + 8 * k)
    return out


def without_sp() -> bool:
    """NXD_SP_STREAMS_NO_SP=1: also split micro-batches that run without sequence parallelism
    at TP = 1: the parts' kernels then only share the GPU, no collectives to hide.  Only taken at
    TP = 1 (modeling_llama checks it): TP > 1 without SP keeps the one-pass step."""
    return _NO_SP


def parts() -> int:
    """Streams (micro-batch parts) requested: 1 = off."""
    try:
        return max(1, int(_MODE))
    except ValueError:
        return 1


def enabled() -> bool:
    return parts() >= 2


def set_enabled(on, n: int = None) -> None:
    """set_enabled(True) -> 2 parts; set_enabled(True, n) or set_enabled(n) -> n parts; False -> off."""
    global _MODE
    if n is None and not isinstance(on, bool):
        n = int(on)
    k = (n if n is not None else 2) if on else 1
    _MODE = str(max(1, int(k)))


def active() -> bool:
    return _active


def streams_for(device: torch.device, n: int = 2) -> List[torch.cuda.Stream]:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.setdefault(idx, [])
    while len(s) < n:
        if _RESERVE > 0:
            from ..ops._ext import ext

            with torch.cuda.device(idx):
                ncu = torch.cuda.get_device_properties(idx).multi_processor_count
                h = ext().cu_masked_stream(reserved_cus(_RESERVE, ncu))
                s.append(torch.cuda.ExternalStream(h, device=torch.device("cuda", idx)))
        else:
            s.append(torch.cuda.Stream(device=idx))
    return s[:n]


def set_stagger(n: int) -> None:
    global _STAGGER
    _STAGGER = max(0, int(n))


def run_interleaved(gens: Sequence[Generator], device: torch.device) -> list:
    """Drive the generators alternately (one step each in turn) until all return; generator i
    runs on stream i (GPU) or inline (CPU), and joins the rotation once generator 0 has taken
    i * stagger steps (NXD_SP_STAGGER).  Returns their return values."""
    global _active
    results = [None] * len(gens)
    live = list(range(len(gens)))
    cuda = device.type == "cuda"
    if cuda:
        main = torch.cuda.current_stream(device)
        ss = streams_for(device, len(gens))
        for s in ss:
            s.wait_stream(main)   # weights / zeroed grads / inputs written on the caller's stream
        _active = True
    steps0 = 0
    while live:
        for i in list(live):
            if i > 0 and 0 in live and steps0 <= i * _STAGGER:
                continue   # part i has not joined the rotation yet
            if i == 0:
                steps0 += 1
            try:
                if cuda:
                    with torch.cuda.stream(ss[i]):
                        next(gens[i])
                else:
                    next(gens[i])
            except StopIteration as e:
                results[i] = e.value
                live.remove(i)
    if cuda:
        for s in ss:
            main.wait_stream(s)
    return results


def join() -> None:
    """Make the current stream wait for both halves' streams (their backward ends there)."""
    global _active
    if not _active:
        return
    main = torch.cuda.current_stream()
    for ss in _streams.values():
        for s in ss:
            main.wait_stream(s)
    _active = False


def accumulate_begin(p: torch.Tensor) -> None:
    """Before a read-modify-write of p's fp32 main_grad: wait for the other stream's last one."""
    if not _active:
        return
    ev = getattr(p, "_nxd_acc_ev", None)
    if ev is not None:
        torch.cuda.current_stream().wait_event(ev)


def accumulate_end(p: torch.Tensor) -> None:
    if not _active:
        return
    ev = getattr(p, "_nxd_acc_ev", None)
    if ev is None:
        ev = p._nxd_acc_ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream())
