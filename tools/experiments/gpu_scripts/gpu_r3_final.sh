#!/bin/bash
# smoke() + 1-GPU bench (driver contract) + TP=1 step profile on the current tree.
set -o pipefail
O=gpurun_out/r3final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1 || exit $?
