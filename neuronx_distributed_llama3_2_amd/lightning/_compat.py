"""Lightning import shim: `lightning.pytorch` (2.x) or `pytorch_lightning`."""

try:  # pragma: no cover - depends on the environment
    import lightning.pytorch as pl  # type: ignore
    from lightning.pytorch.accelerators import CUDAAccelerator  # type: ignore
    from lightning.pytorch.callbacks import TQDMProgressBar  # type: ignore
    from lightning.pytorch.loggers import TensorBoardLogger  # type: ignore
    from lightning.pytorch.plugins.io import CheckpointIO  # type: ignore
    from lightning.pytorch.plugins.precision import Precision  # type: ignore
    from lightning.pytorch.strategies import DDPStrategy  # type: ignore
    HAVE_LIGHTNING = True
except ImportError:  # pragma: no cover
    try:
        import pytorch_lightning as pl  # type: ignore
        from pytorch_lightning.accelerators import CUDAAccelerator  # type: ignore
        from pytorch_lightning.callbacks import TQDMProgressBar  # type: ignore
        from pytorch_lightning.loggers import TensorBoardLogger  # type: ignore
        from pytorch_lightning.plugins.io import CheckpointIO  # type: ignore
        from pytorch_lightning.plugins.precision import Precision  # type: ignore
        from pytorch_lightning.strategies import DDPStrategy  # type: ignore
        HAVE_LIGHTNING = True
    except ImportError:
        pl = CUDAAccelerator = TQDMProgressBar = TensorBoardLogger = CheckpointIO = Precision = DDPStrategy = None
        HAVE_LIGHTNING = False


def require_lightning():
    if not HAVE_LIGHTNING:
        raise ImportError("neuronx_distributed_llama3_2_amd.lightning needs PyTorch Lightning "
                          "(`lightning` >= 2.0 or `pytorch_lightning`), which is not installed")
