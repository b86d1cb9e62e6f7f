#!/bin/bash
# chain launch timelines (scripts/chain_head_timeline.py) for each library given
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  GNNQC_HIP_LIB=$lib timeout -k 10 120 python scripts/chain_head_timeline.py > gpurun_out/tl_$(basename $lib .so).log 2>&1 || { tail gpurun_out/tl_$(basename $lib .so).log; exit 3; }
  tail -1 gpurun_out/tl_$(basename $lib .so).log
done
