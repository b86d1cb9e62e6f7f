#!/bin/bash
# small-kernel and chain-role micro profiles (scripts/step_kernels_micro.py, scripts/chain_roles_trace.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/micro; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python scripts/step_kernels_micro.py > $OUT/kern.jsonl 2>&1 || { tail -20 $OUT/kern.jsonl; exit 3; }
grep kernel $OUT/kern.jsonl
for m in 0 1 2; do
  GNNQC_CHAIN_ROLES=$m timeout -k 10 120 python scripts/chain_roles_trace.py > $OUT/roles$m.jsonl 2>&1 || { tail -20 $OUT/roles$m.jsonl; exit 4; }
  grep roles_mode $OUT/roles$m.jsonl
done
