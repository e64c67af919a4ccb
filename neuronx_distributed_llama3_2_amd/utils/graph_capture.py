"""hipGraph capture with Python's cyclic garbage collector held off.

Root cause of the round-4 decode abort (profiles/r4_decode_attn_trace_abort.txt): the cyclic GC ran
INSIDE a capture (`the captured Python code allocates and can trigger a collection mid-capture) and finalised a `torch.cuda.CUDAGraph` of an earlier model
that had become unreachable in a reference cycle (torch 2.10's `torch.cuda.graph` no longer collects
at entry unless torch.compiler.config.force_cudagraph_gc, so such a cycle from an earlier model
survives into the next capture).  Its destructor destroys a HIP graph, which is not
permitted while a stream captures (hipErrorStreamCaptureUnsupported); the exception escapes a C++
destructor, std::terminate aborts, and Python reports only "Fatal Python error: Aborted ... Garbage-
collecting".  The native backtrace from _C's SIGABRT handler showed `at::cuda::CUDAGraph::~CUDAGraph`
raising (gpurun_out/r5b, round 5).  Any code change that shifts allocation counts moves the GC
trigger point, which is why an unrelated trailing kernel-argument field seemed to cause it.

`graph_capture(graph, **kw)` = `torch.cuda.graph(graph, **kw)` after a full collection (outside the
capture, where destroying old graphs is legal), with `gc.disable()` for the capture (restored after).
"""

from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def graph_capture(graph: "torch.cuda.CUDAGraph", **kwargs):
    was_enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(graph, **kwargs):
            yield graph
    finally:
        if was_enabled:
            gc.enable()
