"""Llama-3.2-1B bf16 inference benchmark on MI355X (BASELINE config 2; reference flow:
examples/inference/llama3_2_inference.ipynb cells 8/13 -> runner.benchmark_sampling).

Random-init weights of the Llama-3.2-1B architecture (no checkpoints offline), synthetic prompt
tokens.  Reports the reference `benchmark_report.json` schema for the end-to-end generate call
(prompt of --prompt tokens, --new tokens greedy), plus context-encoding latency and the per-token
decode latency of the hipGraph token loop.  TP > 1: launch one process per GPU with torchrun.

    python bench_inference.py [--prompt 2048 --new 256 --batch 1 --runs 10]
"""

from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.2-1b")
    ap.add_argument("--prompt", type=int, default=2048)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--graph-steps", type=int, default=16)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--gloo-gpu", action="store_true",
                    help="TP rehearsal on a one-GPU box: every rank on cuda:0, gloo process group (the decode "
                         "all-reduces and vocabulary gather run on the one-shot peer kernels over IPC, so decode is "
                         "still captured in hipGraphs); prefill eager")
    ap.add_argument("--quantized", default=None, choices=[None, "per_tensor_symmetric", "per_channel_symmetric"])
    ap.add_argument("--report", default="gpurun_out/benchmark_report.json")
    ap.add_argument("--weight-layout", action="store_true",
                    help="measured weight-layout pass at the prompt size (trace/weight_layout.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = 0 if args.gloo_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        if args.gloo_gpu:
            dist.init_process_group("gloo")   # prefill eager; decode graphs when the peer kernels carry it
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from neuronx_distributed_llama3_2_amd.inference import InferenceConfig, LlamaForCausalLMInference
    from neuronx_distributed_llama3_2_amd.inference.benchmark import Benchmark, generate_report
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import llama_config

    mcfg = llama_config(args.model)
    seq_len = args.prompt + args.new
    icfg = InferenceConfig(tp_degree=world, batch_size=args.batch, seq_len=seq_len, max_context_length=args.prompt,
                           decode_graph_steps=args.graph_steps, use_hip_graphs=not args.no_graphs,
                           quantized=args.quantized is not None,
                           quantization_type=args.quantized or "per_tensor_symmetric")
    torch.manual_seed(0)
    model = LlamaForCausalLMInference(mcfg, icfg, dtype=torch.bfloat16)
    layouts = None
    if args.weight_layout:
        from neuronx_distributed_llama3_2_amd.trace.weight_layout import optimize_weight_layout

        layouts = optimize_weight_layout(model.model, args.prompt * args.batch)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(10, mcfg.vocab_size, (args.batch, args.prompt), generator=g)
    mask = torch.ones_like(ids)

    def e2e():
        return model.generate(ids, mask, max_new_tokens=args.new, eos_token_id=-1)

    report = {}
    b = Benchmark(e2e, (), icfg, num_runs=args.runs)
    b.run()
    report["e2e_model"] = generate_report(b.latency_list, icfg, max_length=seq_len, batch_size=args.batch)
    cte = Benchmark(model.context_encoding_model, (ids, mask), icfg, num_runs=args.runs)
    cte.run()
    report["context_encoding_model"] = generate_report(cte.latency_list, icfg, max_length=args.prompt,
                                                       batch_size=args.batch)
    # per-token decode latency of the graph loop: (e2e - prefill) / (new - 1)
    e2e_ms = report["e2e_model"]["latency_ms_p50"]
    cte_ms = report["context_encoding_model"]["latency_ms_p50"]
    report["token_generation"] = {"ms_per_token_p50": (e2e_ms - cte_ms) / max(1, args.new - 1),
                                  "tokens_per_s_per_seq": 1000.0 * max(1, args.new - 1) / max(1e-6, e2e_ms - cte_ms)}
    report["config"] = {"model": args.model, "tp": world, "gloo_gpu_rehearsal": bool(args.gloo_gpu), "batch": args.batch, "prompt": args.prompt,
                        "new_tokens": args.new, "dtype": "bf16", "graph_steps": args.graph_steps,
                        "hip_graphs": not args.no_graphs, "quantized": args.quantized,
                        "weight_layouts": None if layouts is None else {v: sum(1 for x in layouts.values() if x == v)
                                                                        for v in set(layouts.values())},
                        "data": "synthetic prompt, random-init weights"}
    if not dist.is_initialized() or dist.get_rank() == 0:
        os.makedirs(os.path.dirname(args.report) or ".", exist_ok=True)
        with open(args.report, "w") as f:
            json.dump(report, f, indent=2)
        print(json.dumps(report))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
