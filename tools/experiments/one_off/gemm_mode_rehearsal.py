"""TP=4 (+SP, replicated kv heads) 4-step training on one GPU (gloo ranks) in the GEMM selection
mode of the environment (NXD_GEMM_TUNE / NXD_GEMM_NO_STREAMK), twice, plus the TP=1 baseline:
the exhaustive-search mode must give the default mode's losses (round 3: non-finite by step 2).

    NXD_GEMM_TUNE=2 NXD_GEMM_NO_STREAMK=1 python tools/gemm_mode_rehearsal.py
"""
import json
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "tests")]
from test_parallel_gpu import _train  # noqa: E402

if __name__ == "__main__":
    mode = {k: os.environ.get(k, "default") for k in ("NXD_GEMM_TUNE", "NXD_GEMM_NO_STREAMK")}
    for streams in (1, 2):
        r = _train(4, "tiny", True, streams=streams)
        print(json.dumps({**mode, "tp": 4, "streams": streams, "loss": r["loss"], "gn": r["gn"]}), flush=True)
    r = _train(1, "tiny", False)
    print(json.dumps({**mode, "tp": 1, "loss": r["loss"], "gn": r["gn"]}), flush=True)
