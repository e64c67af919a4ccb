#!/bin/bash
# TP=8 rank emulation under knob variants (same process per variant, alternating baseline).
O=gpurun_out/emuv; mkdir -p $O
run() {  # label, env..., -- extra args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u tools/emulate_tp_rank.py --tp ${TP:-8} --steps 3 --warmup 1 "$@" > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  echo "$label $(tail -1 $O/run.log)" | tee -a $O/variants.txt
}
run base X=1 --
run mbs8 X=1 -- --mbs 8
run sp_c2 NXD_SP_CHUNKS=2 --
run sp_c1 NXD_SP_CHUNKS=1 --
run wgk1 NXD_WGRAD_KERNEL=1 --
run dgwt0 NXD_DGRAD_WT=0 --
run wgt0 NXD_WGRAD_T=0 --
run base X=1 --
