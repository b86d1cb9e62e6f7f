#!/bin/bash
# GCN backward coefficient form vs recompute: tests, micro, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gcn or chain or cml_fused or step_fusion or flag_reject or deferred" > gpurun_out/t_gcncoef.log 2>&1; rc=$?
tail -3 gpurun_out/t_gcncoef.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1; do
  GNNQC_GCN_COEF=$v timeout -k 10 120 python scripts/grads_multi_micro.py > gpurun_out/gmm_c$v.log 2>&1 || exit 3
  echo "coef=$v $(tail -1 gpurun_out/gmm_c$v.log | cut -c1-200)"
done
AB="GNNQC_GCN_COEF=0 GNNQC_GCN_COEF=1 GNNQC_GCN_COEF=0 GNNQC_GCN_COEF=1" STEPS=400 \
  BENCH_ARGS="--no-knn-line --no-ig-line --no-cv-line" bash scripts/ab_bench.sh
