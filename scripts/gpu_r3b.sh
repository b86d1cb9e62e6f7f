#!/bin/bash
# Round-3 full measurement pass: GPU tests -> CML bench -> SoilNet bench (default and with the
# producer-fused MaxPooling1D) -> IG throughput (chain-sized and per-layer chunks) -> all-reduce cost
# -> rocprofv3 kernel stats of CML and SoilNet. Every GPU step has its own time limit; the first
# failure ends the script.
#   SKIP_TESTS=1 SKIP_IG=1 SKIP_AR=1 NOPROF=1 scripts/gpu_r3b.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r3b; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { echo "== $1"; date; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step "pytest -m gpu ${TESTS:-tests}"
  # no -x: one pass lists every failure; plain test failures (rc 1) do not stop the measurements,
  # a crash, abort or time limit does
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider \
      --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head -20
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
if [ "${SMOKE:-1}" = "1" ]; then
  step "smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
  grep -v amdgpu.ids $OUT/smoke.log | tail -2
fi
step "bench cml"
timeout -k 10 300 python bench.py --steps 400 --warmup 24 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log
step "bench soilnet"
timeout -k 10 300 python bench.py --ds soilnet --steps 40 --warmup 8 > $OUT/bench_soil.log 2>&1 \
  || { tail -20 $OUT/bench_soil.log; exit 3; }
tail -1 $OUT/bench_soil.log
for v in $SOIL_VARIANTS; do
  step "bench soilnet $v"
  env $v timeout -k 10 300 python bench.py --ds soilnet --steps 40 --warmup 8 > $OUT/bench_soil_$v.log 2>&1 \
    || { tail -20 $OUT/bench_soil_$v.log; exit 3; }
  tail -1 $OUT/bench_soil_$v.log
done
if [ "${SKIP_IG:-0}" != "1" ]; then
  for r in ${IG_ROWS:-640 16384}; do
    step "ig rows=$r"
    timeout -k 10 300 python scripts/bench_ig.py --batches 6 --max-rows $r > $OUT/ig_$r.log 2>&1 \
      || { tail -20 $OUT/ig_$r.log; exit 3; }
    tail -1 $OUT/ig_$r.log
  done
fi
if [ "${SKIP_AR:-0}" != "1" ]; then
  step "ar_us"
  timeout -k 10 300 python scripts/ar_us.py > $OUT/ar_us.log 2>&1 || { tail -20 $OUT/ar_us.log; exit 3; }
  grep '^{' $OUT/ar_us.log
fi
[ "${NOPROF:-0}" = "1" ] && exit 0
cd /tmp && export TMPDIR=/tmp
if [ "${IGPROF:-0}" = "1" ]; then
  step "rocprofv3 ig"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/profig -o run --output-format csv -- \
    python3 $ROOT/scripts/bench_ig.py --batches 2 --max-rows 16384 > $OUT/profig.log 2>&1
  rc=$?; echo "rocprof ig rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(ls $OUT/profig/run_kernel_stats.csv $OUT/profig/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 3 30 > $OUT/ig_stats.txt && cat $OUT/ig_stats.txt
fi
[ "${SKIP_CML_PROF:-0}" = "1" ] || {
step "rocprofv3 cml"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 48 --warmup 8 --no-ig-line --no-knn-line > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls $OUT/prof/run_kernel_stats.csv $OUT/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 56 30 > $OUT/cml_stats.txt && cat $OUT/cml_stats.txt
}
step "rocprofv3 soilnet"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/profs -o run --output-format csv -- \
  python3 $ROOT/bench.py --ds soilnet --steps 16 --warmup 8 > $OUT/profs.log 2>&1
rc=$?; echo "rocprof soil rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls $OUT/profs/run_kernel_stats.csv $OUT/profs/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 24 30 > $OUT/soil_stats.txt && cat $OUT/soil_stats.txt
exit 0
