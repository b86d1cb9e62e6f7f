#!/bin/bash
# IG round-3 loop: IG GPU tests -> host-sync diagnostic -> IG throughput -> IG kernel profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/ig2; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_ig_gpu.py -m gpu -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; grep -E "^(FAILED|ERROR)|^E " $OUT/pytest.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 240 python scripts/diag_ig_sync.py > $OUT/diag.log 2>&1 || { tail -20 $OUT/diag.log; exit 3; }
grep -v amdgpu.ids $OUT/diag.log | head -80
timeout -k 10 300 python scripts/bench_ig.py --batches 6 --max-rows 16384 > $OUT/ig.log 2>&1 || { tail -20 $OUT/ig.log; exit 3; }
tail -1 $OUT/ig.log
timeout -k 10 300 python scripts/bench_ig.py --batches 6 --batch 256 --max-rows 32768 > $OUT/ig256.log 2>&1 || { tail -20 $OUT/ig256.log; exit 3; }
tail -1 $OUT/ig256.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $ROOT/scripts/bench_ig.py --batches 2 --max-rows 16384 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls $OUT/prof/run_kernel_stats.csv $OUT/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 $ROOT/scripts/prof_summary.py $f 3 20 > $OUT/ig_stats.txt && cat $OUT/ig_stats.txt
exit 0
