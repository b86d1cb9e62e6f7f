#!/bin/bash
# CML CV generator sweep (GPU box): for each "rainlike rain_fraction" pair in $COMBOS, the bench's
# 5-fold CV of the GCN and the baseline (no throughput side records); lines in gpurun_out/cvsweep.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${COMBOS:-"0.5:0.12"}; do
  rl=${c%%:*}; rf=${c##*:}
  echo "== rainlike $rl rain_fraction $rf ($(date +%T))"
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-knn-line --no-ig-line --no-soil-line \
      --cv-rainlike "$rl" --cv-rain-fraction "$rf" $EXTRA > gpurun_out/cvsweep_${rl}_${rf}.log 2>&1 || exit $?
  tail -1 gpurun_out/cvsweep_${rl}_${rf}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cv']; print(json.dumps({'rainlike': $rl, 'rain_fraction': $rf, **{k: c[k] for k in ('gcn_mean_auc','baseline_mean_auc','gcn_fold_auc','baseline_fold_auc','gcn_minus_baseline_auc','gcn_wins_folds','seconds')}}))" | tee -a gpurun_out/cvsweep.jsonl
done
