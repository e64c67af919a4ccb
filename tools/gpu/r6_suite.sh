#!/bin/bash
# full GPU suite as the driver runs it (plus durations), one process
O=gpurun_out/r6suite; mkdir -p $O
export TMPDIR=/tmp
START=$(date +%s)
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=30 -p no:cacheprovider > $O/suite.log 2>&1
RC=$?
echo "suite rc=$RC wall=$(( $(date +%s) - START ))s" | tee -a $O/suite.log
tail -45 $O/suite.log
exit $RC
