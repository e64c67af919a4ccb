"""Llama-3.2 (1B/3B) / Llama-3 inference CLI: trace -> generate / check accuracy / benchmark
(reference: examples/inference/llama3/llama3_runner.py + runner.py + llama3_2_inference.ipynb).

    python examples/inference/llama3_2_runner.py trace --model_path <hf dir> --traced_path out --sequence_length 2304
    python examples/inference/llama3_2_runner.py generate --traced_path out --prompt "I believe the meaning of life is"
    python examples/inference/llama3_2_runner.py check_accuracy --model_path <hf dir> --traced_path out --prompt_ids 1,2,3
    python examples/inference/llama3_2_runner.py benchmark --traced_path out
TP > 1: `torchrun --nproc-per-node N ... --tp_degree N` (one process per GPU).
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from neuronx_distributed_llama3_2_amd.inference.runner import LlamaRunner  # noqa: E402


def main(argv=None, runner_cls=LlamaRunner):
    p = argparse.ArgumentParser()
    p.add_argument("mode", choices=["trace", "generate", "check_accuracy", "benchmark"])
    p.add_argument("--model_path", default=None)
    p.add_argument("--tokenizer_path", default=None)
    p.add_argument("--traced_path", required=True)
    p.add_argument("--tp_degree", type=int, default=1)
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--max_prompt_length", type=int, default=128)
    p.add_argument("--sequence_length", type=int, default=256)
    p.add_argument("--quantized", action="store_true")
    p.add_argument("--quantization_type", default="per_channel_symmetric")
    p.add_argument("--speculation_length", type=int, default=0)
    p.add_argument("--draft_traced_path", default=None)
    p.add_argument("--prompt", action="append", default=None)
    p.add_argument("--prompt_ids", action="append", default=None, help="comma-separated token ids")
    p.add_argument("--top_k", type=int, default=1)
    p.add_argument("--do_sample", action="store_true")
    p.add_argument("--num_runs", type=int, default=20)
    a = p.parse_args(argv)
    r = runner_cls(model_path=a.model_path, tokenizer_path=a.tokenizer_path or a.model_path)
    if a.mode == "trace":
        r.trace(a.traced_path, tp_degree=a.tp_degree, batch_size=a.batch_size, max_prompt_length=a.max_prompt_length,
                sequence_length=a.sequence_length, quantized=a.quantized, quantization_type=a.quantization_type,
                speculation_length=a.speculation_length)
        print(f"traced to {a.traced_path}")
        return None
    if a.tokenizer_path is None and os.path.exists(os.path.join(a.traced_path, "tokenizer.json")):
        r.tokenizer_path = a.traced_path
    model = r.load_neuron_model(a.traced_path)
    draft = r.load_neuron_model(a.draft_traced_path) if a.draft_traced_path else None
    prompts = a.prompt or [[int(t) for t in s.split(",")] for s in (a.prompt_ids or ["1"])]
    if a.mode == "generate":
        out = r.generate_on_neuron(prompts, model, draft_model=draft, do_sample=a.do_sample, top_k=a.top_k)
        tok = r.load_tokenizer() if r.tokenizer_path else None
        for row in out:
            print(tok.decode(row, skip_special_tokens=True) if tok is not None else row.tolist())
        return out
    if a.mode == "check_accuracy":
        ok = r.check_accuracy(model, prompts)
        print(json.dumps({"accuracy_match": ok}))
        return ok
    rep = r.benchmark_sampling(model, draft, num_runs=a.num_runs,
                               report_path=os.path.join(a.traced_path, "benchmark_report.json"))
    print(json.dumps(rep, indent=2))
    return rep


if __name__ == "__main__":
    main()
