#!/bin/bash
# SoilNet GCN-vs-baseline training-curve diagnostic (first folds, longer training).
ROOT=$(cd "$(dirname "$0")/.." && pwd); cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/soil_diag; mkdir -p "$OUT"
export PYTHONPATH=$ROOT:$PYTHONPATH
EP=${EP:-30}
for mm in ${MODELS:-gcn baseline}; do
  m=""; [ "$mm" = "baseline" ] && m="--baseline"
  timeout -k 10 ${T:-500} python3 -m gnnqc.cli cv --ds soilnet --synthetic --sensors 40 --days ${DAYS:-89} --folds 5 \
      --max-folds ${FOLDS:-2} $m --set model.epochs=$EP --log "$OUT/diag.jsonl" "$@" > "$OUT/diag${m}.log" 2>&1
  rc=$?; echo "rc=$rc $m"; tail -2 "$OUT/diag${m}.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
