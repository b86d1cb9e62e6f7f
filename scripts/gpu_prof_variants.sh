#!/bin/bash
# kernel traces of the graph-replayed CML step under env settings: VARIANTS="name:VAR=v,VAR2=w name2:..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for spec in $VARIANTS; do
  name=${spec%%:*}; kv=${spec#*:}
  echo "== $name ($kv)"
  (
    for a in ${kv//,/ }; do [ "$a" != "-" ] && export "$a"; done
    cd /tmp && TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_$name" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps ${STEPS:-40} --warmup 5 --no-knn-line --no-ig-line --no-soil-line \
      --no-cv-line > "$ROOT/gpurun_out/prof_$name.log" 2>&1
  ) || { tail -5 gpurun_out/prof_$name.log; exit 3; }
  python3 scripts/graph_steady_state.py gpurun_out/prof_$name > gpurun_out/ss_$name.txt && cat gpurun_out/ss_$name.txt
done
