#!/bin/bash
# SoilNet bench across GCN node-kernel time chunks (GNNQC_NODE_TCHUNK) + kernel stats; gpurun_out/nsweep/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/nsweep; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for tc in 8 4 2 1; do
  GNNQC_NODE_TCHUNK=$tc timeout -k 10 200 python bench.py --ds soilnet --steps 48 --warmup 8 > $OUT/tc$tc.log 2>&1 || exit 3
  echo "tc=$tc $(tail -1 $OUT/tc$tc.log | python -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
done
cd /tmp && export TMPDIR=/tmp
for tc in 8 2; do
  GNNQC_NODE_TCHUNK=$tc timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof$tc -o run --output-format csv -- python3 $ROOT/bench.py --ds soilnet --steps 6 --warmup 2 --no-graph > $OUT/prof$tc.log 2>&1 || exit 4
done
echo done
