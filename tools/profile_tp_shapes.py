"""Per-GPU compute time of one Llama-3-8B training micro-batch at TP=N *shapes*, on ONE GPU with
no communication (heads, kv heads, FFN width and vocab divided by N; sequence 8192).  Tells how
well the kernels keep up when TP shrinks every GEMM / attention problem — the compute floor of
the N-GPU bench.  Not a throughput claim (SP elementwise work is done on all S rows here).

    python tools/profile_tp_shapes.py --tp 1 2 4 8
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaForCausalLM, llama_config  # noqa: E402
from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--mbs", type=int, nargs="+", default=[1], help="micro-batch sizes (sequences) to time")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ps.initialize_model_parallel(tensor_model_parallel_size=1)
    dev = torch.device("cuda", 0)
    for tp in a.tp:
        cfg = llama_config("llama3-8b", num_attention_heads=32 // tp, num_key_value_heads=max(1, 8 // tp),
                           intermediate_size=14336 // tp, head_dim=128, vocab_size=128256 // tp,
                           num_hidden_layers=a.layers, max_position_embeddings=max(8192, a.seq))
        model = LlamaForCausalLM(cfg, dtype=torch.bfloat16, device=dev)
        model.train()
        # the flat fp32 gradient buffers of the real training step (main_grad, hipBLASLt fp32
        # in-place wgrad) -- never stepped, just zeroed between micro-batches
        from neuronx_distributed_llama3_2_amd.optimizer.flat_optimizer import FlatMixedPrecisionAdamW

        opt = FlatMixedPrecisionAdamW(model.parameters(), lr=0.0)
        for mbs in a.mbs:
            ids = torch.randint(0, cfg.vocab_size, (mbs, a.seq), device=dev)

            def mb():
                out = model(ids, labels=ids)
                out.loss.backward()
                opt.zero_grad()

            mb()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                mb()
            torch.cuda.synchronize()
            ms = 1000 * (time.perf_counter() - t0) / a.iters
            print(json.dumps({"tp_shapes": tp, "mbs": mbs, "seq": a.seq, "layers": a.layers,
                              "ms_per_microbatch_fwd_bwd": round(ms, 2),
                              "tokens_per_s_per_gpu_compute_only": round(mbs * a.seq / ms * 1000, 1),
                              "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)}), flush=True)
            del ids
            torch.cuda.reset_peak_memory_stats(dev)
        del model, opt
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
