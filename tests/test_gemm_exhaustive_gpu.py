"""NXD_GEMM_TUNE=2 (exhaustive hipBLASLt search, with and without stream-K) on the in-place fp32
main_grad accumulation of the TP=8 weight-gradient shapes and the chunk-view forward / dgrad
outputs, against fp32 PyTorch (tools/check_gemm_exhaustive.py in a fresh process: the tuner reads
its mode once).  Round 3 validated candidates out of place and some picks were wrong in place."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("no_sk", ["1", "0"])
def test_exhaustive_gemm_in_place_wgrad_matches_fp32(no_sk):
    env = dict(os.environ, NXD_GEMM_TUNE="2", NXD_GEMM_NO_STREAMK=no_sk, NXD_GEMM_TUNE_MAX_ALGOS="256")
    env.pop("NXD_GEMM_TUNE_FILE", None)
    env.pop("NXD_GEMM_TABLE", None)
    r = subprocess.run([sys.executable, "tools/check_gemm_exhaustive.py", "--tokens", "4096"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=110)
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-2000:])
    assert len(recs) == 4 and all(x["ok"] for x in recs), recs
