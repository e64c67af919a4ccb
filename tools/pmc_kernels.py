"""Workload for PMC counter passes: the framework's hand-written kernels at the Llama-3-8B shapes
(flash attention fwd+bwd at TP=1 and TP=8 head counts, RMSNorm, SwiGLU, cross-entropy, AdamW)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bench_kernels as bk  # noqa: E402

torch.manual_seed(0)
bk.bench_fa(sdpa=False)
bk.bench_fa(Hq=4, Hkv=1, sdpa=False)
bk.bench_mem()
