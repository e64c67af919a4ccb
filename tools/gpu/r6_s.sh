#!/bin/bash
# Llama-2-7B 8-layer 8k config (the long-sequence gate): which knob moved it from round 3's 10.42 seq/s
O=gpurun_out/r6s; mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --model llama2-7b --layers 8 --gbs 16 --mbs 1 --seq 8192 --steps 3 --warmup 1 --ckpt selective > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python -c "import json; r=[json.loads(l) for l in open('$O/$tag.log') if l.startswith('{')][-1]; print('$tag', round(r['value']/8192,3), r['ms_per_step'])"
}
run default NXD_X=0
run rms_rows0 NXD_RMS_ROWS=0
run swiglu_dual0 NXD_SWIGLU_DUAL=0 NXD_SWIGLU_DUAL_FWD=0
run slab0 NXD_FAB_DKV_SLAB=0
run tune0 NXD_GEMM_TUNE=0
run dgradwt0 NXD_DGRAD_WT=0
run wgradt0 NXD_WGRAD_T=0
run ladder0 NXD_BENCH_LADDER=0
run default2 NXD_X=0
