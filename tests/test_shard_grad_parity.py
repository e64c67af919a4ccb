"""Per-shard gradient parity of the TP / SP layers against TP=1 (tests/shard_grad_parity.py):
fp32 on CPU gloo ranks here; the same comparison on the HIP kernels is in
tests/test_shard_grad_parity_gpu.py."""

import pytest

from shard_grad_parity import collect, compare

_REF = {}


def _ref(preset):
    if preset not in _REF:
        _REF[preset] = collect(1, preset, False)
    return _REF[preset]


@pytest.mark.parametrize("preset,tp,sp,streams", [("tiny", 2, True, 1), ("tiny", 4, True, 1), ("tiny8", 8, True, 2),
                                                  ("tiny", 2, False, 1)])
def test_every_gradient_shard_matches_tp1_cpu(preset, tp, sp, streams):
    errs = compare(_ref(preset), collect(tp, preset, sp, streams), sp)
    assert len(errs) > 10
    bad = {k: v for k, v in errs.items() if not v < 1e-4}
    assert not bad, bad
