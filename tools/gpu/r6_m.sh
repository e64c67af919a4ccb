#!/bin/bash
# single-launch long-context attention + o_proj (SYNC): long-context test first, then the decode tests, A/B
O=gpurun_out/r6m; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_inference_gpu.py -k "long_context" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 600 $T tests/test_inference_gpu.py tests/test_kernels_gpu.py tests/test_spmd_inference_gpu.py -k "decode or attn or generate" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for sy in 1 0; do
    NXD_DECODE_ATTN_SYNC=$sy timeout -k 10 300 python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 6 --report $O/r_${sy}_$rep.json > $O/b_${sy}_$rep.log 2>&1 || { tail -30 $O/b_${sy}_$rep.log; exit 1; }
    python -c "import json; r=json.load(open('$O/r_${sy}_$rep.json')); print('sync $sy rep $rep', r['token_generation'])"
  done
done
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench_inference.py --prompt 2048 --new 256 --batch 1 --runs 2 --report $O/report_prof.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
S=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $S $O/kernel_stats_p2048.csv; rm -rf $O/prof
head -8 $O/kernel_stats_p2048.csv | cut -c1-160
