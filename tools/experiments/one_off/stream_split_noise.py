"""Run-to-run spread of the TP=4 (+SP, replicated kv heads) 4-step training on one GPU (gloo ranks),
with and without the two-stream SP halves: tells a numeric (deterministic) difference from a race.

    python tools/stream_split_noise.py
"""
import json
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_ROOT, os.path.join(_ROOT, "tests")]
from test_parallel_gpu import _train  # noqa: E402

if __name__ == "__main__":
    for streams in (1, 2, 1, 2, 1, 2):
        r = _train(4, "tiny", True, streams=streams)
        print(json.dumps({"streams": streams, "loss": r["loss"], "gn": r["gn"]}), flush=True)
    r = _train(1, "tiny", False)
    print(json.dumps({"tp1": True, "loss": r["loss"], "gn": r["gn"]}), flush=True)
