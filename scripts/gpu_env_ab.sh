#!/bin/bash
# Same-box A/B of environment variants (VARIANTS="name:VAR=v,VAR=v name2:..."): SoilNet step and IG
# throughput per variant, RUNS rounds interleaved. Lines in gpurun_out/env_ab.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/env_ab.txt
for r in $(seq 1 ${RUNS:-2}); do
  for v in $VARIANTS; do
    name=${v%%:*}; kv=${v#*:}; kv=${kv//,/ }
    if [ "${SOIL:-1}" = 1 ]; then
      env $kv timeout -k 10 200 python3 bench.py --ds soilnet --steps 40 --warmup 8 --no-knn-line \
          > gpurun_out/envab_soil_${name}_$r.log 2>&1 || exit 3
      echo "soil $name run $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/envab_soil_${name}_$r.log | head -1)" | tee -a $OUT
    fi
    if [ "${IG:-1}" = 1 ]; then
      env $kv timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-knn-line --no-cv-line --no-soil-line \
          > gpurun_out/envab_ig_${name}_$r.log 2>&1 || exit 3
      echo "ig $name run $r: $(grep -o '"ms_per_call": [0-9.]*' gpurun_out/envab_ig_${name}_$r.log)" | tee -a $OUT
    fi
  done
done
