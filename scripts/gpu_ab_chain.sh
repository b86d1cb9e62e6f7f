#!/bin/bash
# Same-box A/B of compile-time chain variants (scripts/build_chain_variants.py), then the GPU test
# suite on the candidate variant ($CAND).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB="$AB" BENCH_ARGS="--no-knn-line --no-ig-line" bash scripts/ab_bench.sh || exit $?
i=0
for c in $CAND; do
  i=$((i+1))
  echo "== pytest -m gpu with $c"
  GNNQC_HIP_LIB=$c timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/ab/pytest_cand$i.log 2>&1
  rc=$?; tail -2 gpurun_out/ab/pytest_cand$i.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
