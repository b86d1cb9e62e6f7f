#!/bin/bash
# Quality checks on the GPU (writes gpurun_out/cv/):
#   PART=dtype   CML 5-fold CV, GCN and baseline, bf16 vs fp32 compute (the reference trains in fp32)
#   PART=soil    SoilNet 5-fold CV, GCN vs baseline, on the generator with neighbour-only faults
#   PART=xaisoil SoilNet of the XAI generation (per-anomalous-sensor neighbourhoods), GCN vs baseline
ROOT=$(cd "$(dirname "$0")/.." && pwd)
export OUT=$ROOT/gpurun_out/cv
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
case ${PART:-dtype} in
  dtype)
    DATASETS=cml TAG=_bf16 bash "$ROOT/scripts/cv_headline.sh" && \
    DATASETS=cml TAG=_fp32 bash "$ROOT/scripts/cv_headline.sh" --set model.runtime.compute_dtype=fp32 ;;
  soil)
    DATASETS=soilnet TAG=_spatial bash "$ROOT/scripts/cv_headline.sh" ;;
  xaisoil)
    DATASETS=soilnet TAG=_xai bash "$ROOT/scripts/cv_headline.sh" --set pre.per_sensor=true ;;
esac
