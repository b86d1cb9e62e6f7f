#!/bin/bash
# A/B of runtime switches on the CML bench (one line per setting).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/matrix; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${CFGS:-"GNNQC_NO_SIDE_STREAM=0" "GNNQC_NO_SIDE_STREAM=1"}; do
  for g in "" "--no-graph"; do
    env $cfg timeout -k 10 200 python bench.py --steps 100 --warmup 20 $g ${BENCH_ARGS} > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }
    echo "$cfg $g $(tail -1 $OUT/b.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
