"""PyTorch-Lightning integration (reference: src/neuronx_distributed/lightning/*).

MI355X mapping: the XLA strategy / accelerator / launcher become a strategy over one process per
GPU (torchrun or Lightning's own subprocess launcher) that initialises the NxD process-group mesh
(TP/PP/EP/DP over RCCL), hands out DP-rank data shards, leaves DP gradient reduction to the
framework's flat-buffer optimizer (no DDP wrapper), and checkpoints through the NxD sharded
checkpoint API.  Lightning is an optional dependency: `lightning` (2.x) or `pytorch_lightning`
must be importable; it is NOT installed in this build environment, so these classes are written
against its public API and import-gated.  tests/test_lightning_examples.py drives them (and the
examples under examples/training/llama/lightning/) on gloo ranks through a stand-in of that API
(tests/fake_lightning.py): the Lightning-driven run equals the training-API run step for step;
behaviour against real Lightning stays unpinned.
"""

from ._compat import HAVE_LIGHTNING, require_lightning  # noqa: F401
from .launcher import NeuronLauncher  # noqa: F401  (no Lightning dependency)

_EXPORTS = {
    "NeuronXLAStrategy": ".strategy", "NxDStrategy": ".strategy",
    "NeuronXLAAccelerator": ".accelerator", "NeuronCheckpointIO": ".checkpoint_io",
    "NeuronLTModule": ".module", "NeuronXLAPrecisionPlugin": ".precision_plugin",
    "NeuronTQDMProgressBar": ".progress_bar", "NeuronTensorBoardLogger": ".logger",
    "_NeuronXLALauncher": ".launcher",
}


def __getattr__(name):
    if name in _EXPORTS:
        require_lightning()
        import importlib

        return getattr(importlib.import_module(_EXPORTS[name], __name__), name)
    raise AttributeError(name)
