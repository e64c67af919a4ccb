"""Pipeline parallelism (reference: src/neuronx_distributed/pipeline/)."""

from .model import NxDPPModel
from .partition import create_partitions
from .scheduler import InferenceSchedule, Train1F1BSchedule, TrainInterleavedSchedule, TrainSchedule

__all__ = ["NxDPPModel", "create_partitions", "InferenceSchedule", "Train1F1BSchedule", "TrainInterleavedSchedule",
           "TrainSchedule"]
