"""DBRX (16 experts, top-4, clipped QKV, LayerNorm) inference CLI (reference: examples/inference/run_dbrx.py,
dbrx/dbrx_runner.py).  Same modes and flags as llama3_2_runner.py:

    python examples/inference/run_dbrx.py trace --model_path <hf dir> --traced_path out --tp_degree 1
    python examples/inference/run_dbrx.py generate --traced_path out --prompt_ids 1,2,3
TP > 1: `torchrun --nproc-per-node N ... --tp_degree N`; experts are TP-sharded on the
intermediate dim, token generation reads only the routed experts' weights.
"""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from llama3_2_runner import main  # noqa: E402

from neuronx_distributed_llama3_2_amd.inference.moe import DbrxRunner  # noqa: E402

if __name__ == "__main__":
    main(runner_cls=DbrxRunner)
