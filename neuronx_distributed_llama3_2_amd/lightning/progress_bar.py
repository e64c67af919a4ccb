"""Progress bar shown only on the rank that owns the loss (last PP stage, tp 0, dp 0)
(reference: lightning/progress_bar.py)."""

from ..parallel_layers import parallel_state as ps
from ._compat import TQDMProgressBar, require_lightning

require_lightning()


class NeuronTQDMProgressBar(TQDMProgressBar):
    def setup(self, trainer, pl_module, stage: str) -> None:
        super().setup(trainer, pl_module, stage)
        owner = (ps.get_pipeline_model_parallel_rank() == ps.get_pipeline_model_parallel_size() - 1
                 and ps.get_tensor_model_parallel_rank() == 0 and ps.get_data_parallel_rank() == 0)
        if not owner:
            self.disable()
