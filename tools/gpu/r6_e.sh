#!/bin/bash
# (1) TP=2 decode tests (deterministic x batch, lost peer) + peer tests; (2) notebook-config decode;
# (3) PMC of the default dense GEMM loop (PIPE 1).
O=gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_spmd_inference_gpu.py::test_tp2_decode_lost_peer_raises tests/test_spmd_inference_gpu.py::test_tp2_decode_hipgraph_on_peer_kernels tests/test_peer_allreduce_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed|TP=" $O/tests.log | tail -20
bash tools/gpu/r6_infer.sh || exit 1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1)); rm -rf $O/p$i
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python tools/pmc_dense_gemm.py 8192 4096 4096 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
done
python tools/pmc_avg.py $O/p1 $O/p2 > $O/pmc_pipe1.txt 2>&1; rm -rf $O/p1 $O/p2
grep -A30 "dg::gemm_kernel" $O/pmc_pipe1.txt | head -32
