"""Hot ops of the framework: each runs a hand-written CDNA4 HIP kernel on the GPU and a plain
PyTorch fp32 reference on the CPU (see _ext.use_native)."""

from ._ext import ext, ext_available, use_native  # noqa: F401
from .activations import swiglu, swiglu_reference  # noqa: F401
from .cross_entropy import parallel_cross_entropy_reference, vocab_parallel_cross_entropy  # noqa: F401
from .decode import argmax_rows, decode_attention, greedy_advance_, kv_cache_write, topk_sample  # noqa: F401
from .embedding import vocab_parallel_embedding  # noqa: F401
from .grouped_gemm import (grouped_linear, grouped_linear_reference, moe_dispatch, moe_permutation,  # noqa: F401
                           moe_unpermute_combine)
from .flash_attn import attention_reference, flash_attn_func, flash_attn_fwd_lse, rope_attention  # noqa: F401
from .norm import rms_norm, rms_norm_reference  # noqa: F401
from .optim import (adamw_flat_, clip_coefficient, flat_absmax, flat_sumsq, scale_flat_, sr_seed_for_step,  # noqa: F401
                    stochastic_round_bf16)
from .rope import apply_rotary_reference, inv_freq_from_config, llama3_inv_freq, rope_inplace_, rope_tables  # noqa: F401
