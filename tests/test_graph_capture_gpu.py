"""Regression test for the decode abort of rounds 4-5 (profiles/r4_decode_attn_trace_abort.txt): a
torch.cuda.CUDAGraph left in an unreachable reference cycle is finalised by Python's cyclic GC while
another graph captures -> its destructor destroys a HIP graph during capture
(hipErrorStreamCaptureUnsupported) -> std::terminate -> "Fatal Python error: Aborted ... Garbage-
collecting".  torch.cuda.graph no longer collects at entry by default (torch 2.10:
torch.compiler.config.force_cudagraph_gc), so a dead cycle from an earlier model survives into the
next capture.  Runs in a child process (an abort must not take pytest down)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import gc, sys
import torch
sys.path.insert(0, {root!r})
from neuronx_distributed_llama3_2_amd.utils.graph_capture import graph_capture
x = torch.zeros(1024, device="cuda")
class Holder:
    pass
gc.disable()
h = Holder()
h.me = h                                   # a reference cycle: only the cyclic GC frees it
h.g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    x.add_(1)
torch.cuda.synchronize()
with torch.cuda.graph(h.g):
    h.z = x * 3                            # the graph's private memory pool holds an allocation
del h
gc.enable()
gc.set_threshold(50)
g2 = torch.cuda.CUDAGraph()
ctx = graph_capture(g2) if {use_guard} else torch.cuda.graph(g2)
with ctx:
    y = x * 2
    keep = []
    for i in range(5000):                  # live container allocations: trigger gen-0 collections
        keep.append([i])
g2.replay()
torch.cuda.synchronize()
print("capture ok")
'''


def test_gc_during_capture_is_held_off():
    """A dead graph (with pool memory) in a reference cycle plus enough live allocations inside the
    capture to trigger collections: graph_capture completes and the captured graph replays.  (The
    plain-torch.cuda.graph arm of this script did not abort on the box -- the destructor's failing HIP
    call depends on the old graph's state -- so the evidence of the failure mode is the native stack
    recorded in profiles/r5_decode_abort_native_backtrace.txt.)"""
    code = SCRIPT.format(root=ROOT, use_guard=True)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, NXD_ABORT_BACKTRACE="1"))
    assert r.returncode == 0 and "capture ok" in r.stdout, r.stderr[-3000:]
