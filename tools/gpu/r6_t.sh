#!/bin/bash
# long-sequence gate config: direct run vs the tool / pytest way of launching bench.py (pipes, no timeout)
O=gpurun_out/r6t; mkdir -p $O
B="bench.py --gpus 1 --model llama2-7b --layers 8 --gbs 16 --mbs 1 --seq 8192 --steps 3 --warmup 1 --ckpt selective"
timeout -k 10 300 python $B > $O/direct_file.log 2>&1 || exit 1
echo "direct->file: $(grep -o '"ms_per_step": [0-9.]*' $O/direct_file.log)"
timeout -k 10 300 python $B 2>&1 | cat > $O/direct_pipe.log || exit 1
echo "direct|cat: $(grep -o '"ms_per_step": [0-9.]*' $O/direct_pipe.log)"
timeout -k 10 300 python -c "
import subprocess, sys
r = subprocess.run([sys.executable] + '$B'.split(), capture_output=True, text=True)
print([l for l in r.stdout.splitlines() if l.startswith('{')][-1][:300])
" > $O/subproc.log 2>&1 || exit 1
echo "subprocess capture: $(grep -o '"ms_per_step": [0-9.]*' $O/subproc.log)"
python $B > $O/notimeout.log 2>&1 || exit 1
echo "no timeout->file: $(grep -o '"ms_per_step": [0-9.]*' $O/notimeout.log)"
