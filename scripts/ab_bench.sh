#!/bin/bash
# A/B of the CML bench under env settings: AB="VAR=a VAR=b ..." scripts/ab_bench.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for kv in $AB; do
  i=$((i+1))
  echo "== $kv"
  env $kv timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 24 $BENCH_ARGS > $OUT/b$i.log 2>&1 \
    || { tail -20 $OUT/b$i.log; exit 3; }
  tail -1 $OUT/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])"
done
