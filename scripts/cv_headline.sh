#!/bin/bash
# Headline quality numbers: 5-fold CV mean ROC-AUC, GCN vs baseline, CML and SoilNet
# (CML GCN 0.941 / baseline 0.885; SoilNet GCN 0.858 / baseline 0.816).
# Synthetic data of the reference example shapes (CML: 23 links x 28 days @1 min;
# SoilNet: 40 boxes x 89 days @15 min), random-init weights, packaged model configs.
# Usage: bash scripts/cv_headline.sh [extra cli args]   (GPU box; writes gpurun_out/cv/)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-$ROOT/gpurun_out/cv}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export PYTHONPATH=$ROOT:$PYTHONPATH
CML_ARGS=${CML_ARGS:---sensors 23 --days 28 --flagged 4}
SOIL_ARGS=${SOIL_ARGS:---sensors 40 --days 89}

echo "== CML CV"; date
timeout -k 10 ${CV_TIMEOUT:-900} python3 -m gnnqc.cli cv --ds cml --synthetic $CML_ARGS --both --folds 5 \
    --out "$OUT/cv_cml.json" --log "$OUT/cv_cml.jsonl" "$@" > "$OUT/cv_cml.log" 2>&1
rc=$?; echo "cml rc=$rc"; tail -3 "$OUT/cv_cml.log"
[ $rc -ne 0 ] && exit $rc

echo "== SoilNet CV"; date
timeout -k 10 ${CV_TIMEOUT:-900} python3 -m gnnqc.cli cv --ds soilnet --synthetic $SOIL_ARGS --both --folds 5 \
    --out "$OUT/cv_soilnet.json" --log "$OUT/cv_soilnet.jsonl" "$@" > "$OUT/cv_soilnet.log" 2>&1
rc=$?; echo "soilnet rc=$rc"; tail -3 "$OUT/cv_soilnet.log"
exit $rc
