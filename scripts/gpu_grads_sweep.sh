#!/bin/bash
# SoilNet bench across weight-gradient workgroup budgets (GNNQC_GRADS_WG); writes gpurun_out/gsweep/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/gsweep; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for wg in 2048 4096 8192 1024; do
  GNNQC_GRADS_WG=$wg timeout -k 10 200 python bench.py --ds soilnet --steps 48 --warmup 8 > $OUT/wg$wg.log 2>&1 || exit 3
  echo "wg=$wg $(tail -1 $OUT/wg$wg.log | python -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
done
