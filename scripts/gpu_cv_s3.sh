#!/bin/bash
# Quality regression check after the bf16 state streams (GCN 5-fold CV, CML + SoilNet) and the last
# fold of the SoilNet XAI-generation baseline; writes gpurun_out/cv/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
DATASETS="cml soilnet" MODELS=gcn TAG=_s3 CV_TIMEOUT=400 bash scripts/cv_headline.sh || exit $?
FOLD_IDS=4 CV_TIMEOUT=700 bash scripts/gpu_xai_baseline.sh
