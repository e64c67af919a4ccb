"""utils/memory_planner.py: parameter accounting matches the model, the plan reproduces the measured
1-GPU bench peak, and the 288 GB sizing conclusions for Llama-3-70B TP=8 + SP hold."""

import pytest
import torch

from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
from neuronx_distributed_llama3_2_amd.utils.memory_planner import (GIB, largest_micro_batch, params_per_rank,
                                                                    plan_training_memory)


def test_params_per_rank_matches_model_and_stages():
    cfg = llama_config("tiny")
    m = LlamaForCausalLM(cfg, dtype=torch.float32, device=torch.device("cpu"))
    assert params_per_rank(cfg) == sum(p.numel() for p in m.parameters())
    c8 = llama_config("llama3-8b")
    assert abs(params_per_rank(c8) - 8.03e9) < 0.01e9
    # stages of a 4-stage pipeline add up to the whole model
    total = sum(params_per_rank(c8, pp=4, stage=s) for s in range(4))
    assert total == params_per_rank(c8)


def test_plan_matches_measured_bench_peak():
    p = plan_training_memory(llama_config("llama3-8b"), tp=1, mbs=1, seq=8192)
    assert abs(p.total_bytes / GIB - 189.0) / 189.0 < 0.05    # profiles/r2_bench_1gpu_v4.log
    assert p.fits


def test_llama3_70b_tp8_fits_one_node():
    c70 = llama_config("llama3-70b")
    p1 = plan_training_memory(c70, tp=8, mbs=1)
    assert p1.fits and p1.total_bytes / GIB < 210
    # sequence parallelism divides the hidden-sized activations by TP
    assert plan_training_memory(c70, tp=8, sequence_parallel=False).total_bytes > p1.total_bytes
    # full recompute shrinks activations; ZeRO-1 over DP shrinks the optimizer state
    assert plan_training_memory(c70, tp=8, activation_checkpoint="full").activation_bytes < p1.activation_bytes
    assert plan_training_memory(c70, tp=8, dp=4).resident_bytes < p1.resident_bytes
    assert largest_micro_batch(c70, tp=8) >= 2
    # re-gathering the column-parallel inputs in backward (instead of saving them) trades comm for memory
    assert plan_training_memory(c70, tp=8, save_gathered_input=False).total_bytes < p1.total_bytes
    assert not plan_training_memory(c70, tp=1).fits   # 70B needs model parallelism
    with pytest.raises(ValueError):
        plan_training_memory(c70, activation_checkpoint="bogus")
