"""Long-sequence throughput / memory regression gate on one MI355X (reference:
test/integration/llama2_7B/test_long_seqlen.py:13-97, which asserts sequences/s and peak device memory
of Llama-2-7B truncated to 8 layers, GBS 16, MBS 1, selective recompute, at 8k / 16k / 32k).

Through bench.py (public training API, fp32-master AdamW, synthetic tokens): each sequence length must
reach at least 80 % of this tree's measured rate on one GPU (profiles/r3_long_seqlen_1gpu.jsonl:
10.42 / 4.44 / 1.68 seq/s) -- itself above the reference's whole-trn1.32xlarge thresholds of 6.60 /
2.60 / 1.00 -- and stay within 15 % of the measured peak memory (44.4 / 54.0 / 73.0 GiB).  The rate
varies by ~10 % from box to box with the same tree (round 6: 10.45-10.47 seq/s at 8k on one box,
9.44-9.47 on another, 4 runs each; profiles/r6_long_seqlen_box_variance.txt), so 90 % left no margin."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MEASURED = {8192: (10.417, 44.4), 16384: (4.438, 54.0), 32768: (1.681, 73.0)}
REFERENCE_SEQ_PER_S = {8192: 6.60, 16384: 2.60, 32768: 1.00}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seq", [8192, 16384, 32768])
def test_long_seqlen_throughput_and_memory(seq):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "1", "--model", "llama2-7b", "--layers", "8", "--gbs", "16", "--mbs", "1",
           "--seq", str(seq), "--steps", "2", "--warmup", "1", "--ckpt", "selective"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    seq_per_s = rec["value"] / seq
    rate, mem = MEASURED[seq]
    print(f"seq {seq}: {seq_per_s:.3f} seq/s (measured {rate}, trn1.32xlarge {REFERENCE_SEQ_PER_S[seq]}), "
          f"peak {rec['peak_mem_gib']} GiB (measured {mem})")
    assert seq_per_s >= 0.8 * rate and seq_per_s >= REFERENCE_SEQ_PER_S[seq], seq_per_s
    assert rec["peak_mem_gib"] <= 1.15 * mem, rec["peak_mem_gib"]
