#!/bin/bash
# bench sweep over an environment knob: VAR=name VALS="a b c" bash scripts/gpu_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in $VALS; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 20 > $OUT/b_$v.log 2>&1 || { tail -5 $OUT/b_$v.log; exit 3; }
  echo "$VAR=$v $(tail -1 $OUT/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
