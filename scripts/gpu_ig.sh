#!/bin/bash
# Integrated-gradients throughput sweep over the path-chunk size (rows per forward/backward: 640
# fits the cross-CU chain kernels, larger chunks take the per-layer kernels) + a kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/ig; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in ${ROWS:-16384 640 2048}; do
  timeout -k 10 300 python scripts/bench_ig.py --batches 3 --max-rows $r > $OUT/ig_$r.log 2>&1 \
    || { tail -20 $OUT/ig_$r.log; exit 3; }
  echo "rows=$r $(tail -1 $OUT/ig_$r.log)"
done
[ "${NOPROF:-0}" = "1" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/scripts/bench_ig.py --batches 2 --max-rows ${PROF_ROWS:-16384} > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls $OUT/prof/run_kernel_stats.csv $OUT/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 1 30
exit 0
