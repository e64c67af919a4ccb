"""Weight-layout optimisation (reference: trace/model_builder.py:457-586 -- the compiler suggests a
layout for every weight at the PRIORITY model's shapes, a layout-transformation program rewrites
the weights on device once at load, and every other bucket uses the transformed weights).

MI355X form: the "compiler suggestion" is a measurement.  For each distinct projection shape of
the model, the priority bucket's token count M is run through both GEMM layouts the framework can
serve -- "nk" (weight as stored, [N, K]: y = x W^T) and "kn" (a pre-packed K-major copy, [K, N]:
y = x Wkn) -- and the faster one (by more than `min_gain`) is kept.  `apply_layouts` then packs
the chosen weights on the device once; inference projections (`packed_linear`) use the packed copy
for prefill-sized inputs (decode-sized inputs keep the [N, K] rows the GEMV streams).  The layout
map is a small JSON file saved next to the compiled shards, so a later load repeats the packing
without re-measuring.

Measured on MI355X (profiles/r2_weight_layout_prefill_ab.jsonl, Llama-3.2-1B prefill): hipBLASLt
serves both layouts at nearly the same speed, so the pass keeps 64-65 of 65 weights as stored at
128 and 2048 tokens and prefill latency does not change (1.74 / 1.63 ms, 5.26 / 5.26 ms).  It is
therefore opt-in (`InferenceConfig(weight_layout_optimization=True)`, ModelBuilder
`priority_model_idx`).  A first version that timed each layout once, stored layout first, picked
the packed layout for every weight at 128 tokens and made prefill 15 % slower: the layouts are now
timed in alternating rounds.
"""

from __future__ import annotations

import json
import os
from typing import Dict, Iterable, Optional, Tuple

import torch

from ..ops import gemm as _gemm

LAYOUT_FILE = "weight_layout.json"


def _weights(model: torch.nn.Module) -> Iterable[Tuple[str, torch.nn.Module]]:
    for name, mod in model.named_modules():
        w = getattr(mod, "weight", None)
        if isinstance(w, torch.Tensor) and w.dim() == 2 and w.is_floating_point() and \
                type(mod).__name__ in ("ColumnParallelLinear", "RowParallelLinear", "Linear", "OutputChannelParallelConv2d"):
            yield name, mod
        wq = getattr(mod, "weight_qkv", None)
        if isinstance(wq, torch.Tensor) and wq.dim() == 2 and wq.is_floating_point():
            yield name, mod


def _weight_of(mod) -> torch.Tensor:
    if hasattr(mod, "_fused_weight_bias"):
        return mod._fused_weight_bias()[0]
    return mod.weight


def _time(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def choose_layouts(model: torch.nn.Module, tokens: int, reps: int = 20, min_gain: float = 0.05,
                   rounds: int = 3) -> Dict[str, str]:
    """Measured layout per weight at M = tokens (priority bucket): the two layouts are timed in
    alternating rounds (min per layout), so clock ramp and cache warmth do not favour the one timed
    second.  On the CPU every weight keeps 'nk'."""
    out: Dict[str, str] = {}
    by_shape: Dict[tuple, str] = {}
    for name, mod in _weights(model):
        w = _weight_of(mod)
        key = (tuple(w.shape), w.dtype, str(w.device))
        if key not in by_shape:
            layout = "nk"
            if w.is_cuda and w.dtype in (torch.bfloat16, torch.float16):
                x = torch.randn(tokens, w.shape[1], dtype=w.dtype, device=w.device)
                wkn = w.detach().t().contiguous()
                t_nk = t_kn = float("inf")
                for _ in range(rounds):
                    t_nk = min(t_nk, _time(lambda: _gemm.linear(x, w), reps))
                    t_kn = min(t_kn, _time(lambda: _gemm.matmul(x, wkn), reps))
                layout = "kn" if t_kn < t_nk * (1.0 - min_gain) else "nk"
                del x, wkn
            by_shape[key] = layout
        out[name] = by_shape[key]
    return out


def apply_layouts(model: torch.nn.Module, layouts: Dict[str, str]) -> int:
    """Pack the weights whose layout is 'kn' (once, on their device); returns how many were packed."""
    n = 0
    mods = dict(_weights(model))
    for name, layout in layouts.items():
        mod = mods.get(name)
        if mod is None:
            continue
        if layout == "kn":
            with torch.no_grad():
                mod._nxd_packed_kn = _weight_of(mod).detach().t().contiguous()
            if "_forward_impl" in mod.__dict__ and not isinstance(mod._forward_impl, _PackedForward) and \
                    not getattr(mod, "sequence_parallel_enabled", False):
                mod._forward_impl = _PackedForward(mod, mod._forward_impl)
            n += 1
        else:
            mod.__dict__.pop("_nxd_packed_kn", None)
            if isinstance(mod.__dict__.get("_forward_impl"), _PackedForward):
                mod._forward_impl = mod._forward_impl.orig
        mod._nxd_layout = layout
    return n


class _PackedForward:
    """Replaces a parallel linear's `_forward_impl` (parallel_layers/layers.py) so that no-grad
    calls (ModelBuilder / inference) read the packed K-major weight; autograd calls keep the
    original path.  The module's TP collectives around `_forward_impl` are unchanged."""

    def __init__(self, mod, orig):
        self.mod_ref = mod
        self.orig = orig

    def __call__(self, input, weight, bias, *args, **kwargs):
        wkn = getattr(self.mod_ref, "_nxd_packed_kn", None)
        if torch.is_grad_enabled() or wkn is None or weight is not self.mod_ref.weight:
            return self.orig(input, weight, bias, *args, **kwargs)
        y = _gemm.matmul(input, wkn)
        return y + bias if bias is not None else y


def packed_linear(mod, x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x W^T through the module's packed K-major copy when its layout is 'kn'."""
    wkn = getattr(mod, "_nxd_packed_kn", None)
    if wkn is not None and getattr(mod, "_nxd_layout", "nk") == "kn":
        y = _gemm.matmul(x, wkn)
        return y + bias if bias is not None else y
    return _gemm.linear(x, w, bias)


def save_layouts(path: str, layouts: Dict[str, str]) -> None:
    with open(os.path.join(path, LAYOUT_FILE), "w") as f:
        json.dump(layouts, f, indent=1, sort_keys=True)


def load_layouts(path: str) -> Optional[Dict[str, str]]:
    p = os.path.join(path, LAYOUT_FILE)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def optimize_weight_layout(model: torch.nn.Module, tokens: int, path: Optional[str] = None,
                           save: bool = False) -> Dict[str, str]:
    """Reuse the saved map from `path` (or measure one), apply it, and optionally save it there."""
    layouts = load_layouts(path) if path else None
    if layouts is None:
        layouts = choose_layouts(model, tokens)
        if path and save:
            os.makedirs(path, exist_ok=True)
            save_layouts(path, layouts)
    apply_layouts(model, layouts)
    return layouts
