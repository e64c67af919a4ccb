"""Per-shard gradient parity on the HIP kernels: N ranks share the one MI355X (gloo collectives on
staged GPU tensors), bf16 compute, two accumulated micro-batches; every parameter's fp32 gradient
shard against the TP=1 gradient slice (relative max error <= 2e-2 per tensor)."""

import pytest

from shard_grad_parity import collect, compare

pytestmark = pytest.mark.gpu
_REF = {}


def _ref(preset):
    if preset not in _REF:
        _REF[preset] = collect(1, preset, False, dev_kind="cuda")
    return _REF[preset]


@pytest.mark.parametrize("preset,tp,sp,streams", [
    ("tiny8", 8, True, 1),    # one KV head per rank, the headline layout
    ("tiny8", 8, True, 2),    # + the two-stream SP halves (bench default at N > 1)
    ("tiny", 4, True, 1),     # KV heads replicated on 2 ranks (q-group order, KV-group all-reduce)
    ("tiny", 2, False, 1),    # TP without SP
])
def test_every_gradient_shard_matches_tp1_gpu(preset, tp, sp, streams):
    errs = compare(_ref(preset), collect(tp, preset, sp, streams, dev_kind="cuda"), sp)
    assert len(errs) > 10
    bad = {k: round(v, 4) for k, v in errs.items() if not v <= 2e-2}
    assert not bad, (bad, max(errs.values()))
