"""Long-sequence training throughput next to the reference's only published numbers.

Reference (test/integration/llama2_7B/test_long_seqlen.py:87-89, config run_llama_7b_tp_ptl.sh:
18-41): Llama-2-7B architecture truncated to 8 layers, GBS 16, MBS 1, selective activation
checkpointing, flash attention, ZeRO-1 / fp32 optimizer states, TP=32 + SP on a whole
trn1.32xlarge: 6.60 / 2.60 / 1.00 sequences/s at 8k / 16k / 32k.  Here: the same architecture,
batch and sequence lengths through bench.py on N MI355X (default 1), synthetic tokens, random
init, bf16 compute with fp32 master weights; tokens/s, seq/s and peak HBM per configuration.

    python tools/bench_long_seqlen.py [--gpus N] [--seqs 8192 16384 32768] [--steps 3 --warmup 1]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE_SEQ_PER_S = {8192: 6.60, 16384: 2.60, 32768: 1.00}   # trn1.32xlarge, TP=32
REFERENCE_MEM_BYTES = {8192: 88590512128, 16384: 109604828160, 32768: 124354230272}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--seqs", type=int, nargs="+", default=[8192, 16384, 32768])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ckpt", default="selective")
    a = ap.parse_args()
    for seq in a.seqs:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(a.gpus), "--model", "llama2-7b",
               "--layers", "8", "--gbs", "16", "--mbs", "1", "--seq", str(seq), "--steps", str(a.steps),
               "--warmup", str(a.warmup), "--ckpt", a.ckpt]
        r = subprocess.run(cmd, capture_output=True, text=True)
        recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not recs:
            print(json.dumps({"seq_len": seq, "error": r.stderr[-1500:]}), flush=True)
            return r.returncode or 1
        rec = recs[0]
        sps = rec["value"] / seq
        print(json.dumps({"config": "llama2-7b 8 layers, GBS 16, MBS 1, ckpt " + a.ckpt, "seq_len": seq,
                          "n_gpus": a.gpus, "tokens_per_s": rec["value"], "seq_per_s": round(sps, 3),
                          "ms_per_step": rec["ms_per_step"], "peak_mem_gib": rec["peak_mem_gib"], "loss": rec["loss"],
                          "reference_seq_per_s_trn1_32nc": REFERENCE_SEQ_PER_S.get(seq),
                          "reference_peak_mem_gib": round(REFERENCE_MEM_BYTES.get(seq, 0) / 2**30, 1),
                          "vs_reference": round(sps / REFERENCE_SEQ_PER_S[seq], 3) if seq in REFERENCE_SEQ_PER_S else None}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
