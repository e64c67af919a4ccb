"""TensorBoard logger that writes only from the loss-owning rank (last PP stage, tp 0, dp 0)
(reference: lightning/logger.py NeuronTensorBoardLogger)."""

from ..parallel_layers import parallel_state as ps
from ._compat import TensorBoardLogger, require_lightning

require_lightning()


class NeuronTensorBoardLogger(TensorBoardLogger):
    def __init__(self, log_rank0: bool = False, **kwargs):
        super().__init__(**kwargs)
        self.log_rank0 = log_rank0

    @property
    def should_print(self) -> bool:
        if self.log_rank0:
            import torch.distributed as dist

            return not dist.is_initialized() or dist.get_rank() == 0
        return (ps.get_pipeline_model_parallel_rank() == ps.get_pipeline_model_parallel_size() - 1
                and ps.get_tensor_model_parallel_rank() == 0 and ps.get_data_parallel_rank() == 0)

    def log_metrics(self, metrics, step=None) -> None:
        if self.should_print:
            super().log_metrics(metrics, step)

    def log_hyperparams(self, params, metrics=None) -> None:
        if self.should_print:
            super().log_hyperparams(params, metrics)
