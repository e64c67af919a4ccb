"""Utilities: logging, timeline, serialization, activation checkpointing, model init, sampling,
speculative decoding (reference: src/neuronx_distributed/utils/)."""
