#!/bin/bash
# FA bwd dS^T swizzle check: numerics tests, kernel timing, LDS bank-conflict counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fab_swz; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "flash or fa_" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_kernels.py --only fa_tp > $O/fa_tp.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_kernels.py --only fa > $O/fa.jsonl 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $O/p1 -o run -- python tools/pmc_kernels.py > $O/p1.log 2>&1
