#!/bin/bash
# PMC passes of the grouped MoE kernels (fwd / dgrad 256-tile, grouped wgrad) on the Mixtral gate_up shape,
# plus the grouped-GEMM bench against the framework's loop backend.
set -o pipefail
D=gpurun_out/r3ggpmc; mkdir -p $D
export TMPDIR=/tmp
for m in 0 1 2; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $D/m${m}_p1 -o run --output-format csv -- python tools/prof_grouped.py $m 3 > $D/m${m}_p1.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $D/m${m}_p2 -o run --output-format csv -- python tools/prof_grouped.py $m 3 > $D/m${m}_p2.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/bench_grouped_gemm.py > $D/grouped_gemm_vs_framework_loop.jsonl 2>&1 || exit $?
timeout -k 10 900 python bench.py --gpus 1 --steps 4 --warmup 2 --mbs 2 > $D/bench_mbs2.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --gpus 1 --steps 4 --warmup 2 --mbs 1 > $D/bench_mbs1.log 2>&1 || exit $?
