"""Distribution of the TP=2 vs TP=1 prefill-logit difference behind the bound of
tests/test_spmd_inference_gpu.py::test_tp2_server_greedy_matches_tp1_on_gpu (rel_l2 / rel_max <= 3.5e-2):
both servers on the one GPU (TP=2 = two resident gloo ranks), random-init weights from several weight
seeds, several random prompts each; last-position prefill logits.  One JSON line per (kind, weight seed,
prompt) and a summary line per kind (max / p50 / p95).

    python tools/tp2_prefill_parity_dist.py --kinds tiny,llama3.2-1b --wseeds 3 --prompts 8
"""
import argparse
import json
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import test_spmd_inference_gpu as T  # noqa: E402
from neuronx_distributed_llama3_2_amd.inference.spmd_server import SpmdGenerationServer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="tiny,llama3.2-1b")
    ap.add_argument("--wseeds", type=int, default=3)
    ap.add_argument("--prompts", type=int, default=8)
    a = ap.parse_args()
    for kind in a.kinds.split(","):
        cfg = T._cfg(kind)
        l2s, mxs = [], []
        for ws in range(a.wseeds):
            path = os.path.join(tempfile.mkdtemp(), "full.pt")
            torch.save(T._random_full_state(cfg, kind, seed=ws), path)
            kw = dict(batch_size=2, seq_len=128, max_context_length=96, deterministic=True)
            servers = {}
            try:
                for tp in (1, 2):
                    servers[tp] = SpmdGenerationServer.from_full_state_dict(cfg.to_dict(), path, tp, kw, dtype="bfloat16")
                for pi in range(a.prompts):
                    g = torch.Generator().manual_seed(1000 * ws + pi)
                    ids = torch.randint(3, cfg.vocab_size, (2, 16 + 4 * pi), generator=g)
                    la = servers[1].pool.call("_context_encode", ids).float()
                    lb = servers[2].pool.call("_context_encode", ids).float()
                    if la.dim() == 3:
                        la, lb = la[:, -1], lb[:, -1]
                    l2 = float((la - lb).norm() / la.norm())
                    mx = float((la - lb).abs().max() / la.abs().max())
                    l2s.append(l2)
                    mxs.append(mx)
                    print(json.dumps({"kind": kind, "wseed": ws, "prompt": pi, "len": ids.shape[1],
                                      "rel_l2": round(l2, 5), "rel_max": round(mx, 5)}), flush=True)
            finally:
                for s in servers.values():
                    s.close()

        def q(v, f):
            v = sorted(v)
            return round(v[min(len(v) - 1, int(f * len(v)))], 5)
        print(json.dumps({"kind": kind, "n": len(l2s), "rel_l2_max": round(max(l2s), 5),
                          "rel_l2_p50": round(statistics.median(l2s), 5), "rel_l2_p95": q(l2s, 0.95),
                          "rel_max_max": round(max(mxs), 5), "rel_max_p50": round(statistics.median(mxs), 5),
                          "rel_max_p95": q(mxs, 0.95)}), flush=True)


if __name__ == "__main__":
    main()
