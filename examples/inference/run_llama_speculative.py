"""Speculative decoding with a small draft model (reference: examples/inference/run_llama_speculative.py).

    python examples/inference/run_llama_speculative.py --model_path <target hf> --draft_model_path <draft hf> \
        --traced_path out --draft_traced_path out_draft --speculation_length 4 --prompt_ids 1,2,3
Both models are traced with the same speculation length; generation runs greedy draft/verify/
accept rounds captured in hipGraphs (inference/speculation.py).
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from neuronx_distributed_llama3_2_amd.inference.runner import LlamaRunner  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model_path", required=True)
    p.add_argument("--draft_model_path", required=True)
    p.add_argument("--traced_path", required=True)
    p.add_argument("--draft_traced_path", required=True)
    p.add_argument("--tp_degree", type=int, default=1)
    p.add_argument("--max_prompt_length", type=int, default=128)
    p.add_argument("--sequence_length", type=int, default=256)
    p.add_argument("--speculation_length", type=int, default=4)
    p.add_argument("--prompt_ids", action="append", default=None, help="comma-separated token ids")
    a = p.parse_args(argv)
    kw = dict(tp_degree=a.tp_degree, batch_size=1, max_prompt_length=a.max_prompt_length,
              sequence_length=a.sequence_length, speculation_length=a.speculation_length)
    target = LlamaRunner(model_path=a.model_path)
    target.trace(a.traced_path, **kw)
    LlamaRunner(model_path=a.draft_model_path).trace(a.draft_traced_path, **kw)
    model = target.load_neuron_model(a.traced_path)
    draft = target.load_neuron_model(a.draft_traced_path)
    prompts = [[int(t) for t in s.split(",")] for s in (a.prompt_ids or ["1"])]
    out = target.generate_on_neuron(prompts, model, draft_model=draft)
    for row in out:
        print(row.tolist())
    return out


if __name__ == "__main__":
    main()
