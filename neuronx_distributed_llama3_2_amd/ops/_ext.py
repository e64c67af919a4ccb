"""Loader for the in-tree CDNA4 extension and the native-vs-reference dispatch rule.

Rule: a tensor on the GPU ALWAYS runs the hand-written HIP kernel; if the extension is missing the
op raises (never a silent eager fallback).  CPU tensors run the plain-PyTorch fp32 reference of
the same op, which is what the CPU/gloo test-suite and the numerics tests compare against.
`NXD_FORCE_REFERENCE=1` forces the reference path on the GPU (debugging / A-B only).
"""

from __future__ import annotations

import os

import torch

_C = None
_ERR = None


def ext():
    """Return the `_C` extension module, building nothing; raise loudly if it is unavailable."""
    global _C, _ERR
    if _C is not None:
        return _C
    # The shipped exhaustive hipBLASLt table (tuned/gemm_gfx950.txt, tools/tune_gemm.py) is opt-in
    # (NXD_GEMM_TABLE=<path>): measured in the full 1-GPU bench, the in-process top-24 tuning of
    # the first step picks faster solutions (16.8k vs 16.3k tokens/s, profiles/r1_gemm_table_ab.txt).
    try:
        from .. import _C as c  # noqa: WPS433
    except ImportError as e:  # pragma: no cover - depends on the build
        _ERR = e
        raise RuntimeError(
            "neuronx_distributed_llama3_2_amd HIP extension (_C) is not built; run "
            "`python -m neuronx_distributed_llama3_2_amd._build` (hipcc --offload-arch=gfx950)"
        ) from e
    _C = c
    return _C


def ext_available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


def use_native(*tensors: torch.Tensor) -> bool:
    """True when the op must run its HIP kernel (all tensors on the GPU)."""
    if os.environ.get("NXD_FORCE_REFERENCE", "0") == "1":
        return False
    ts = [t for t in tensors if t is not None]
    return bool(ts) and all(t.is_cuda for t in ts)
