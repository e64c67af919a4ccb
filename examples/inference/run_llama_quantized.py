"""int8 weight-only quantized Llama inference (reference: examples/inference/run_llama_quantized.py).

    python examples/inference/run_llama_quantized.py --model_path <hf dir> --traced_path out \
        --quantization_type per_channel_symmetric --prompt_ids 1,2,3
The decoder and lm_head linears hold int8 weights with fp32 scales; decode reads them directly in
the skinny-GEMM kernel (csrc/gemv.hip), prefill dequantises into the GEMM.
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from neuronx_distributed_llama3_2_amd.inference.runner import LlamaRunner  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model_path", default=None, help="HF directory (None: random-init weights of --config)")
    p.add_argument("--traced_path", required=True)
    p.add_argument("--tp_degree", type=int, default=1)
    p.add_argument("--max_prompt_length", type=int, default=128)
    p.add_argument("--sequence_length", type=int, default=256)
    p.add_argument("--quantization_type", default="per_channel_symmetric",
                   choices=["per_tensor_symmetric", "per_channel_symmetric"])
    p.add_argument("--prompt_ids", action="append", default=None, help="comma-separated token ids")
    a = p.parse_args(argv)
    r = LlamaRunner(model_path=a.model_path, tokenizer_path=a.model_path)
    r.trace(a.traced_path, tp_degree=a.tp_degree, batch_size=1, max_prompt_length=a.max_prompt_length,
            sequence_length=a.sequence_length, quantized=True, quantization_type=a.quantization_type)
    model = r.load_neuron_model(a.traced_path)
    prompts = [[int(t) for t in s.split(",")] for s in (a.prompt_ids or ["1"])]
    out = r.generate_on_neuron(prompts, model)
    for row in out:
        print(row.tolist())
    return out


if __name__ == "__main__":
    main()
