#!/bin/bash
# Headline quality numbers: 5-fold CV mean ROC-AUC, GCN vs baseline, CML and SoilNet
# (CML GCN 0.941 / baseline 0.885; SoilNet GCN 0.858 / baseline 0.816).
# Synthetic data, random-init weights, packaged model configs:
#   CML     23 links x 28 days @1 min, 4 flagged links (reference example shape, more labels)
#   SoilNet 210 sensors x 365 days @15 min (the reference's SoilNet numbers come from its
#           full multi-year set; on the 89-day example shape the GCN is under-trained,
#           see profiles/r1_soil_diag.md)
# Usage (GPU box; writes gpurun_out/cv/):
#   DATASETS="cml soilnet" MODELS="gcn baseline" bash scripts/cv_headline.sh [extra cli args]
#   FOLD_IDS=0,1,2 TAG=_a ...   (run a subset of folds; per-fold lines append to cv_<ds>_<model>.jsonl)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-$ROOT/gpurun_out/cv}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export PYTHONPATH=$ROOT:$PYTHONPATH
CML_ARGS=${CML_ARGS:---sensors 23 --days 28 --flagged 4}
SOIL_ARGS=${SOIL_ARGS:---sensors 40 --days 365}
for ds in ${DATASETS:-cml soilnet}; do
  args=$CML_ARGS; [ "$ds" = "soilnet" ] && args=$SOIL_ARGS
  for mm in ${MODELS:-gcn baseline}; do
    m=""; [ "$mm" = "baseline" ] && m="--baseline"
    echo "== $ds $mm CV"; date
    timeout -k 10 ${CV_TIMEOUT:-1000} python3 -m gnnqc.cli cv --ds $ds --synthetic $args $m --folds 5 \
        ${FOLD_IDS:+--fold-ids $FOLD_IDS} --out "$OUT/cv_${ds}_${mm}${TAG}.json" --log "$OUT/cv_${ds}_${mm}.jsonl" "$@" \
        > "$OUT/cv_${ds}_${mm}${TAG}.log" 2>&1
    rc=$?; echo "$ds $mm rc=$rc"; tail -1 "$OUT/cv_${ds}_${mm}${TAG}.log"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
