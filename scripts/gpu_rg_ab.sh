#!/bin/bash
# Same-box A/B of the recompute-gates backward (GNNQC_TM_RG=1 vs 0): SoilNet step and IG throughput,
# interleaved; then the RG kernel test. Lines in gpurun_out/rg_ab.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/rg_ab.txt
for r in 1 2; do
  for v in 1 0; do
    GNNQC_TM_RG=$v timeout -k 10 200 python3 bench.py --ds soilnet --steps 40 --warmup 8 --no-knn-line \
        > gpurun_out/rgab_soil_${v}_$r.log 2>&1 || exit 3
    echo "soil RG=$v run $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rgab_soil_${v}_$r.log)" | tee -a $OUT
    GNNQC_TM_RG=$v timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-knn-line --no-cv-line --no-soil-line \
        > gpurun_out/rgab_ig_${v}_$r.log 2>&1 || exit 3
    echo "ig RG=$v run $r: $(grep -o '"ms_per_call": [0-9.]*' gpurun_out/rgab_ig_${v}_$r.log)" | tee -a $OUT
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "recomputed_gates or time_major or pair_fusion or maxpool" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rgab_tests.log 2>&1; tail -2 gpurun_out/rgab_tests.log
