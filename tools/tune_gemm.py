"""Exhaustively tune recorded hipBLASLt GEMM keys (every library solution timed) and write the
table the framework ships (neuronx_distributed_llama3_2_amd/tuned/gemm_gfx950.txt).

    python tools/tune_gemm.py --keys keys.txt --out table.txt

A key is the column-major hipBLASLt problem csrc/gemm.cpp builds for D[M,N] = A[M,K] @ B[K,N]:
"opA opB m n k lda ldb ldc ldd typeAB typeCD beta_nonzero" with hipBLASLt A = B^T, m = N, n = M.
"""
import argparse
import os
import sys
import time

OP_N, OP_T = 111, 112
DT = {14: "bfloat16", 2: "float16", 0: "float32"}


def tensors_for(key, torch):
    opA, opB, m, n, k, lda, ldb, ldc, ldd, ta, tc, beta = map(int, key.split())
    N, M, K = m, n, k
    dev = "cuda"
    tab, tcd = getattr(torch, DT[ta]), getattr(torch, DT[tc])
    if opA == OP_N:
        b = torch.randn(K, lda, device=dev, dtype=tab)[:, :N]
    else:
        b = torch.randn(N, lda, device=dev, dtype=tab)[:, :K].t()
    if opB == OP_N:
        a = torch.randn(M, ldb, device=dev, dtype=tab)[:, :K]
    else:
        a = torch.randn(K, ldb, device=dev, dtype=tab)[:, :M].t()
    d = torch.zeros(M, ldd, device=dev, dtype=tcd)[:, :N]
    return a, b, d, float(beta)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.environ["NXD_GEMM_TUNE"] = "2"
    os.environ["NXD_GEMM_TUNE_FILE"] = a.out
    os.environ.pop("NXD_GEMM_TABLE", None)
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from neuronx_distributed_llama3_2_amd.ops import ext

    done = set()
    if os.path.exists(a.out):
        done = {ln.split("|")[0].strip() for ln in open(a.out) if "|" in ln}
    keys = []
    for ln in open(a.keys):
        ln = ln.strip()
        if ln and ln not in done and ln not in keys:
            keys.append(ln)
    print(f"{len(keys)} keys to tune ({len(done)} already in {a.out})", flush=True)
    for i, key in enumerate(keys):
        A, B, D, beta = tensors_for(key, torch)
        t0 = time.time()
        ext().gemm(A, B, D, None, 1.0, beta)
        torch.cuda.synchronize()
        M, K = A.shape
        N = B.shape[1]
        ms = [e[1] for e in ext().gemm_tuned_entries() if e[0] == key]
        tf = 2 * M * N * K / (ms[0] * 1e-3) / 1e12 if ms and ms[0] > 0 else 0
        print(f"[{i + 1}/{len(keys)}] {key}  M={M} N={N} K={K}  best {ms[0] if ms else -1:.4f} ms "
              f"({tf:.0f} TF)  tuned in {time.time() - t0:.1f}s", flush=True)
        del A, B, D


if __name__ == "__main__":
    main()
