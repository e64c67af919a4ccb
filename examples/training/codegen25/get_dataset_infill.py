"""Build a causal-infilling (fill-in-the-middle) training token file for CodeGen2.5
(reference: examples/training/codegen25/get_dataset_infill.py — same span sampling, on token ids).

    python examples/training/codegen25/get_dataset_infill.py --input tokens.bin --output infill.bin \
        --block_size 2048 --mask_ids 51198,51197 --eom_id 51196 --sep_ids 50256,51195

Input / output: flat uint32 token files (utils/data_loader.py format, read by the native loader);
the input is cut into block_size blocks and half of them are rewritten
`prefix-with-<mask_i> ++ <|endoftext|><sep> ++ <mask_i> span_i <eom> ...`.
"""

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))

from neuronx_distributed_llama3_2_amd.utils.data_loader import write_token_file  # noqa: E402
from neuronx_distributed_llama3_2_amd.utils.training_utils import infill_token_blocks  # noqa: E402


def _ids(s):
    return [int(t) for t in s.split(",") if t]


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--input", required=True)
    p.add_argument("--output", required=True)
    p.add_argument("--block_size", type=int, default=2048)
    p.add_argument("--mask_ids", type=_ids, required=True, help="comma-separated ids of <mask_1>, <mask_2>, ...")
    p.add_argument("--eom_id", type=int, required=True)
    p.add_argument("--sep_ids", type=_ids, required=True, help="ids of '<|endoftext|><sep>'")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--fraction", type=float, default=0.5)
    a = p.parse_args(argv)
    toks = np.fromfile(a.input, dtype=np.uint32)
    n = len(toks) // a.block_size
    blocks = [toks[i * a.block_size:(i + 1) * a.block_size].tolist() for i in range(n)]
    out = infill_token_blocks(blocks, a.block_size, a.mask_ids, a.eom_id, a.sep_ids, seed=a.seed,
                              fraction=a.fraction, max_num_spans=len(a.mask_ids))
    written = write_token_file(a.output, [np.asarray(b, dtype=np.uint32) for b in out])
    print(f"wrote {written} tokens ({len(out)} blocks) to {a.output}")
    return out


if __name__ == "__main__":
    main()
