"""Precision plugin (reference: lightning/precision_plugin.py): parameters are already bf16 with
fp32 master weights inside the NxD optimizer, so no autocast / loss scaling is applied."""

from ._compat import Precision, require_lightning

require_lightning()


class NeuronXLAPrecisionPlugin(Precision):
    def __init__(self, mixed_precision_enabled: bool = False) -> None:
        super().__init__()
        self.mixed_precision_enabled = mixed_precision_enabled

    def optimizer_step(self, optimizer, model, closure, **kwargs):
        closure()                      # forward + backward
        return optimizer.step(**kwargs)
