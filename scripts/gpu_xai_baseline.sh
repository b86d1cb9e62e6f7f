#!/bin/bash
# Remaining folds of the SoilNet XAI-generation baseline CV (folds 0-1 in profiles/r2_cv_soilnet_xai.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
FOLD_IDS=${FOLD_IDS:-2,3} TAG=_xai_b${FOLD_IDS//,/} DATASETS=soilnet MODELS=baseline CV_TIMEOUT=${CV_TIMEOUT:-1100} \
  bash scripts/cv_headline.sh --set pre.per_sensor=true
