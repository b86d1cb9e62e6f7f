#!/bin/bash
# Round-3 measurement loop: optional focused tests -> CML bench -> rocprofv3 kernel stats of the
# graph-mode bench (the timed path) -> optional SoilNet bench.
#   TESTS="tests/x.py" K=expr STEPS=300 SOIL=1 NOPROF=1 EAGER=1 scripts/gpu_r3.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r3; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$TESTS" ]; then
  echo "== tests $TESTS"; date
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v -p no:cacheprovider \
      --timeout 120 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest.log 2>&1
  rc=$?; tail -25 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PRE" ]; then
  echo "== pre: $PRE"; date
  timeout -k 10 300 python -u $PRE > $OUT/pre.log 2>&1
  rc=$?; grep -v amdgpu.ids $OUT/pre.log | tail -40; [ $rc -ne 0 ] && exit $rc
fi
echo "== bench cml"; date
timeout -k 10 300 python bench.py --steps ${STEPS:-400} --warmup 24 $BENCH_ARGS > $OUT/bench.log 2>&1 \
  || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log
if [ "${SOIL:-0}" = "1" ]; then
  echo "== bench soilnet"; date
  timeout -k 10 300 python bench.py --ds soilnet --steps 40 --warmup 8 > $OUT/bench_soil.log 2>&1 \
    || { tail -20 $OUT/bench_soil.log; exit 3; }
  tail -1 $OUT/bench_soil.log
fi
[ "${NOPROF:-0}" = "1" ] && exit 0
echo "== rocprofv3 (graph replay)"; date
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 48 --warmup 8 $BENCH_ARGS > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls $OUT/prof/run_kernel_stats.csv $OUT/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 56 30
if [ "${SOIL:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/profs -o run --output-format csv -- \
    python3 $ROOT/bench.py --ds soilnet --steps 16 --warmup 8 > $OUT/profs.log 2>&1
  rc=$?; echo "rocprof soil rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(ls $OUT/profs/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 24 30
fi
exit 0
