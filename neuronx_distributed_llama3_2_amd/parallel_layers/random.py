"""Model-parallel RNG state tracking (reference: src/neuronx_distributed/parallel_layers/random.py:20-127).

Dropout / init inside tensor-parallel regions must differ across TP ranks but be identical across
DP replicas; everything else uses the default (DP-shared) generator.  States are the device
generator states (HIP RNG on the GPU, the CPU generator otherwise).
"""

from __future__ import annotations

import contextlib

import torch

from .parallel_state import get_data_parallel_rank, get_pipeline_model_parallel_rank, get_tensor_model_parallel_rank

_MODEL_PARALLEL_RNG_TRACKER_NAME = "model-parallel-rng"


def _get_state():
    return torch.cuda.get_rng_state() if torch.cuda.is_available() else torch.get_rng_state()


def _set_state(state):
    if torch.cuda.is_available():
        torch.cuda.set_rng_state(state)
    else:
        torch.set_rng_state(state)


class RNGStatesTracker:
    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def get_states(self):
        return dict(self.states_)

    def set_states(self, states):
        self.states_ = dict(states)

    def add(self, name, seed):
        if seed in self.seeds_:
            raise Exception(f"seed {seed} already exists")
        self.seeds_.add(seed)
        if name in self.states_:
            raise Exception(f"rng state {name} already exists")
        orig = _get_state()
        torch.manual_seed(seed)
        self.states_[name] = _get_state()
        _set_state(orig)

    @contextlib.contextmanager
    def fork(self, name=_MODEL_PARALLEL_RNG_TRACKER_NAME):
        if name not in self.states_:
            # lazily seeded trackers behave like the default generator
            yield
            return
        orig = _get_state()
        _set_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _get_state()
            _set_state(orig)


# reference name kept for API parity
XLARNGStatesTracker = RNGStatesTracker
_RNG_STATE_TRACKER = RNGStatesTracker()


def get_rng_tracker() -> RNGStatesTracker:
    return _RNG_STATE_TRACKER


def get_xla_rng_tracker() -> RNGStatesTracker:
    return _RNG_STATE_TRACKER


def model_parallel_manual_seed(seed: int) -> None:
    """Default generator: `seed` + 100 * pp_rank (DP/TP-shared);  TP regions: seed + 2718 + tp_rank."""
    offset = seed + 2718
    tp_seed = offset + get_tensor_model_parallel_rank()
    data_seed = seed + 100 * get_pipeline_model_parallel_rank()
    _RNG_STATE_TRACKER.reset()
    torch.manual_seed(data_seed)
    _RNG_STATE_TRACKER.add(_MODEL_PARALLEL_RNG_TRACKER_NAME, tp_seed)
    _ = get_data_parallel_rank


model_parallel_xla_manual_seed = model_parallel_manual_seed
