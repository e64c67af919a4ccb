"""The training LlamaForCausalLM on its HIP kernels (bf16: flash attention, fused RMSNorm,
in-place RoPE, SwiGLU, vocab-parallel cross entropy, hipBLASLt GEMMs with fp32 wgrad) against
HuggingFace's fp32 Llama on the same weights: loss and parameter gradients within bf16 tolerance
(reference pattern: test/integration/parallel_layers/test_layers.py:44-101)."""

import json
import os
import tempfile

import pytest
import torch
import torch.distributed as dist

from neuronx_distributed_llama3_2_amd.ops import _ext
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps

pytestmark = pytest.mark.gpu


def test_llama_hip_kernels_match_hf_fp32():
    from transformers import LlamaConfig
    from transformers import LlamaForCausalLM as HF

    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM
    from neuronx_distributed_llama3_2_amd.scripts.checkpoint_converter import main as convert

    assert _ext.ext_available()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29577")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ps.initialize_model_parallel(1)
    cfg = LlamaConfig(hidden_size=512, intermediate_size=1536, num_hidden_layers=2, num_attention_heads=4,
                      num_key_value_heads=2, vocab_size=4096, max_position_embeddings=1024, rope_theta=500000.0,
                      rms_norm_eps=1e-5, head_dim=128)
    torch.manual_seed(0)
    hf = HF(cfg).float()
    sd = {k: v.detach().clone() for k, v in hf.state_dict().items()}
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump(cfg.to_dict(), f)
    torch.save(sd, os.path.join(d, "checkpoint.pt"))
    convert(["--input_dir", d, "--output_dir", os.path.join(d, "tp1"), "--config", os.path.join(d, "config.json"),
             "--tp_size", "1", "--convert_from_full_state"])
    shard = torch.load(os.path.join(d, "tp1", "model", "dp_rank_00_tp_rank_00_pp_rank_00.pt"), weights_only=True)
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device("cuda", 0))
    missing, _ = model.load_state_dict({k: v.to(torch.bfloat16) for k, v in shard.items()}, strict=False)
    assert not [m for m in missing if "rope" not in m], missing
    # HF in fp32 on the bf16-rounded weights (the same numbers our model holds)
    hf.load_state_dict({k: v.to(torch.bfloat16).float() for k, v in sd.items()})
    hf = hf.cuda()
    torch.manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (2, 512), device="cuda")
    ref = hf(ids, labels=ids)
    ref.loss.backward()
    out = model(ids, labels=ids)
    out.loss.backward()
    assert abs(float(out.loss) - float(ref.loss)) < 2e-2 * float(ref.loss), (float(out.loss), float(ref.loss))
    hp = dict(hf.named_parameters())
    pairs = {
        "model.layers.1.mlp.down_proj.weight": "model.layers.1.mlp.down_proj.weight",
        "model.layers.0.self_attn.o_proj.weight": "model.layers.0.self_attn.o_proj.weight",
        "model.norm.weight": "model.norm.weight",
        "model.layers.0.input_layernorm.weight": "model.layers.0.input_layernorm.weight",
        "model.embed_tokens.weight": "model.embed_tokens.weight",
        "lm_head.weight": "lm_head.weight",
    }
    mp = dict(model.named_parameters())
    for ours, theirs in pairs.items():
        g = mp[ours].grad.float()
        rg = hp[theirs].grad.float()
        rel = ((g - rg).norm() / rg.norm()).item()
        assert rel < 5e-2, (ours, rel)
    # fused QKV gradient against HF's separate q/k/v gradients
    gq = mp["model.layers.0.self_attn.qkv_proj.weight_qkv"].grad.float()
    rq = torch.cat([hp[f"model.layers.0.self_attn.{n}_proj.weight"].grad for n in "qkv"]).float()
    assert ((gq - rq).norm() / rq.norm()).item() < 5e-2
    ps.destroy_model_parallel()
    dist.destroy_process_group()
