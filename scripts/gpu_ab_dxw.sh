#!/bin/bash
# one-off A/B: chain backward dx wave (CHAINB_DXW) - chain GPU tests, then alternating benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "chain or cml_fused or step_fusion or flag_reject" > gpurun_out/t_dxw.log 2>&1; rc=$?
tail -3 gpurun_out/t_dxw.log; [ $rc -ne 0 ] && exit $rc
AB="GNNQC_HIP_LIB=gnnqc/_lib/variants/dxw0.so GNNQC_HIP_LIB=gnnqc/_lib/libgnnqc_hip.so GNNQC_HIP_LIB=gnnqc/_lib/variants/dxw0.so GNNQC_HIP_LIB=gnnqc/_lib/libgnnqc_hip.so" \
  STEPS=400 BENCH_ARGS="--no-knn-line --no-ig-line --no-cv-line" bash scripts/ab_bench.sh
