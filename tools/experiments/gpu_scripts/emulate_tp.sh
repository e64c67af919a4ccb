#!/bin/bash
# Per-rank compute floor of the N-GPU bench: one TP rank emulated on one GPU (tools/emulate_tp_rank.py),
# full 32-layer Llama-3-8B, then a rocprof breakdown of the last TP=8 step.
O=gpurun_out/emu; mkdir -p $O
export TMPDIR=/tmp
for tp in 8 4 2; do
  timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp $tp --steps 3 --warmup 1 > $O/tp$tp.log 2>&1 || { tail -20 $O/tp$tp.log; exit 1; }
  tail -1 $O/tp$tp.log | tee -a $O/emulate.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python tools/emulate_tp_rank.py --tp 8 --steps 1 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
T=$(find $O/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_breakdown.py $T > $O/breakdown.txt && python tools/step_breakdown.py $T --by-kernel > $O/breakdown_by_kernel.txt && rm -f $T
head -25 $O/breakdown.txt
