#!/bin/bash
# merge + o_proj launch with the split merge parallelised: tests, notebook-config decode, kernel stats
O=gpurun_out/r6l; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_inference_gpu.py tests/test_kernels_gpu.py -k "decode or attn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 6 --report $O/r_p2048_$rep.json > $O/b_$rep.log 2>&1 || { tail -30 $O/b_$rep.log; exit 1; }
  python -c "import json; r=json.load(open('$O/r_p2048_$rep.json')); print('p2048 rep $rep', r['token_generation'])"
done
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 2 --report $O/report_prof.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $S $O/kernel_stats_p2048.csv; rm -rf $O/prof
head -8 $O/kernel_stats_p2048.csv | cut -c1-160
