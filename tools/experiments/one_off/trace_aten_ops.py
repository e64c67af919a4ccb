"""Which PyTorch (non-native) ops run in one Llama-3-8B layer fwd+bwd on the GPU, and from where.

Profiles 2 decoder layers with torch.profiler (CPU op view + python stacks) and prints every aten
elementwise/copy op with its input shapes and the innermost python frame of this repo that issued
it.  Used to hunt down glue kernels around the hand-written ones.
"""
import os
import sys
from collections import Counter

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29544")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ps.initialize_model_parallel(1)
    cfg = llama_config("llama3-8b", num_hidden_layers=2)
    model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=torch.device("cuda", 0))
    ids = torch.randint(0, cfg.vocab_size, (1, 8192), device="cuda")
    for _ in range(2):
        model(ids, labels=ids).loss.backward()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], record_shapes=True,
                                with_stack=True) as prof:
        model(ids, labels=ids).loss.backward()
        torch.cuda.synchronize()
    cnt = Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.name in ("aten::empty", "aten::view", "aten::as_strided",
                                                           "aten::empty_strided", "aten::t", "aten::transpose",
                                                           "aten::reshape", "aten::_reshape_alias", "aten::detach",
                                                           "aten::slice", "aten::select", "aten::permute",
                                                           "aten::expand", "aten::alias", "aten::lift_fresh",
                                                           "aten::unsqueeze", "aten::squeeze", "aten::contiguous",
                                                           "aten::result_type", "aten::resolve_conj", "aten::resolve_neg",
                                                           "aten::empty_like", "aten::chunk", "aten::split",
                                                           "aten::narrow", "aten::_to_copy", "aten::to", "aten::item",
                                                           "aten::_local_scalar_dense", "aten::is_nonzero", "aten::numel"):
            continue
        frames = [f for f in (ev.stack or []) if "neuronx_distributed_llama3_2_amd" in f or "torch/autograd" in f]
        where = frames[0] if frames else "(autograd engine)"
        cnt[(ev.name, str(ev.input_shapes)[:60], where[-90:])] += 1
    for (name, shp, where), n in cnt.most_common(40):
        print(f"{n:4d}  {name:28s} {shp:60s} {where}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
