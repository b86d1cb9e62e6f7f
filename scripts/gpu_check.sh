#!/bin/bash
# One GPU-box session: kernel tests -> bench (graph / no graph) -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; anything other than a clean finish or
# ordinary test failures stops the script (no further GPU work after a fault).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== pytest -m gpu"; date
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
echo "== bench"; date
timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 10 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 10 --no-graph > $OUT/bench_nograph.log 2>&1 || { echo "bench nograph failed"; tail -20 $OUT/bench_nograph.log; exit 3; }
tail -1 $OUT/bench_nograph.log
if [ "${SKIP_PROF:-0}" = "1" ]; then exit 0; fi
echo "== rocprofv3"; date
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 3 --no-graph > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $OUT/prof.log
exit $rc
