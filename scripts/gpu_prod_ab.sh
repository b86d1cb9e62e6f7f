#!/bin/bash
# GCN forward as chain producers: GPU tests, then kernel traces with / without (GNNQC_GCN_PROD)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gcn_fused_gpu.py \
  tests/test_cml_fused_gpu.py tests/test_step_fusion_gpu.py tests/test_flag_reject_gpu.py > gpurun_out/t_prod.log 2>&1 \
  && tail -3 gpurun_out/t_prod.log \
  && VARIANTS="${VARIANTS:-prod1:- prod0:GNNQC_GCN_PROD=0}" bash scripts/gpu_prof_variants.sh
