"""Accelerator: the ROCm GPU through Lightning's CUDA accelerator (HIP is exposed as torch.cuda)
(reference: lightning/accelerator.py NeuronXLAAccelerator)."""

from ._compat import CUDAAccelerator, require_lightning

require_lightning()


class NeuronXLAAccelerator(CUDAAccelerator):
    @staticmethod
    def name() -> str:
        return "mi355x"

    def get_device_stats(self, device):
        import torch

        return {"max_memory_allocated_gib": torch.cuda.max_memory_allocated(device) / 2**30}
