"""utils/profiling.py: parameter / FLOP accounting used for bench.py's MFU, phase timer, and the
torch.profiler step capture (CPU activities here; HIP activities on the GPU box)."""

import os
import tempfile

import torch

from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config
from neuronx_distributed_llama3_2_amd.utils import profiling


def test_param_count_and_flops():
    assert profiling.llama_num_params(llama_config("llama3-8b")) == 8_030_261_248
    cfg = llama_config("llama3-8b", num_hidden_layers=2, hidden_size=64, intermediate_size=128,
                       num_attention_heads=4, num_key_value_heads=2, vocab_size=256)
    m = LlamaForCausalLM(cfg, dtype=torch.float32, device=torch.device("cpu"))
    assert profiling.llama_num_params(cfg) == sum(p.numel() for p in m.parameters())
    f = profiling.model_flops_per_token(8.03e9, 32, 4096, 8192)
    assert abs(f - (6 * 8.03e9 + 6 * 32 * 4096 * 8192)) < 1
    assert abs(profiling.mfu(1000.0, 2.5e12, 1) - 1e-0) < 1e-9


def test_phase_timer_and_profile_steps():
    t = profiling.PhaseTimer()
    x = torch.randn(64, 64)
    for _ in range(2):
        with t.phase("mm"):
            x = x @ x.t() / 64
        with t.phase("add"):
            x = x + 1
    s = t.summary()
    assert set(s) == {"mm", "add"} and all(v >= 0 for v in s.values())
    d = tempfile.mkdtemp()

    def step():
        with profiling.annotate("step"):
            torch.randn(32, 32) @ torch.randn(32, 32)

    table = profiling.profile_steps(step, steps=2, warmup=1, out_dir=d, tag="t")
    assert "aten::mm" in table or "aten::matmul" in table
    assert os.path.getsize(os.path.join(d, "t_trace.json")) > 0
