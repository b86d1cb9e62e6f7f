#!/bin/bash
# Same-box A/B of chain-kernel builds: the forward chain's per-stage tile-0 end times (scripts/chain_debug.py)
# for each library given (default: the in-tree build). Usage: bash scripts/chain_ab.sh [lib.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
libs=("$@"); [ ${#libs[@]} -eq 0 ] && libs=(gnnqc/_lib/libgnnqc_hip.so)
for lib in "${libs[@]}"; do
  echo "== $lib"
  GNNQC_HIP_LIB=$lib NS=6 REPS=20 timeout -k 10 100 python scripts/chain_debug.py 2>/dev/null | grep -E "trace|status" || exit 1
done
