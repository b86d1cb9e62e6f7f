#!/bin/bash
# Same-box A/B of the CML training step against a variant library: steady-state kernel tables of both
# (graph replays under rocprofv3), then RUNS interleaved driver-form bench runs of each.
#   VARIANT=gnnqc/_lib/<name>.so bash scripts/gpu_cml_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
V=${VARIANT:?VARIANT=<variant .so>}
VARIANTS="new:- old:GNNQC_HIP_LIB=$V" STEPS=40 bash scripts/gpu_prof_variants.sh > gpurun_out/ss_ab.log 2>&1 || exit 3
for r in $(seq 1 ${RUNS:-3}); do
  for v in new old; do
    if [ $v = old ]; then export GNNQC_HIP_LIB=$V; else unset GNNQC_HIP_LIB; fi
    timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-ig-line --no-cv-line --no-soil-line \
      --no-knn-line > gpurun_out/cab_${v}_$r.log 2>&1 || exit 3
    echo "cml $v run $r: $(grep -m1 -o '"ms_per_step": [0-9.]*' gpurun_out/cab_${v}_$r.log)" | tee -a gpurun_out/env_ab.txt
  done
done
