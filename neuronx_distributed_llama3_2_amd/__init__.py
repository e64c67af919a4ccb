"""MI355X-native distributed training / inference library with the capabilities and public API of
AWS neuronx-distributed (NxD) — PyTorch-ROCm + hand-written CDNA4 HIP kernels + RCCL over xGMI.

Top-level API parity with the reference package root (src/neuronx_distributed/__init__.py:1-13).
"""

from ._version import __version__  # noqa: F401
from . import ops, parallel_layers, utils  # noqa: F401
from .trainer.checkpoint import (  # noqa: F401
    CheckpointIOState,
    finalize_checkpoint,
    has_checkpoint,
    load_checkpoint,
    save_checkpoint,
)
from .trainer.trainer import (  # noqa: F401
    initialize_parallel_model,
    initialize_parallel_optimizer,
    neuronx_distributed_config,
)


def __getattr__(name):
    # lazily import heavier subpackages (pipeline / trace / kernels / modules / inference)
    import importlib

    if name in ("pipeline", "trace", "kernels", "modules", "quantization", "optimizer", "inference", "models",
                "lightning", "scripts", "trainer", "parallel"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
