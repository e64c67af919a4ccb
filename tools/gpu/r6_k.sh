#!/bin/bash
# FA forward tests on the final kernel; SP peer collectives' HBM-side cost (8 ranks on one GPU);
# TP=2 vs TP=1 prefill-logit difference distribution
O=gpurun_out/r6k; mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_long_attention_gpu.py tests/test_attention_dropout_gpu.py -k "flash or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python tools/bench_sp_peer_hbm.py --world 8 > $O/sp_peer_hbm.jsonl 2> $O/sp_peer_hbm.err || { tail -30 $O/sp_peer_hbm.err; exit 1; }
cat $O/sp_peer_hbm.jsonl
timeout -k 10 600 python tools/tp2_prefill_parity_dist.py --kinds tiny,llama3.2-1b --wseeds 3 --prompts 6 > $O/tp2_dist.jsonl 2> $O/tp2_dist.err || { tail -30 $O/tp2_dist.err; exit 1; }
grep '"n"' $O/tp2_dist.jsonl
