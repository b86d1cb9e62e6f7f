#!/bin/bash
# GPU tests (all, or $TESTS) -> CML bench -> rocprofv3 kernel stats of the graph-mode bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/full; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== tests"; date
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${TESTS:-tests -m gpu} -x -q -p no:cacheprovider \
    --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert" $OUT/pytest.log | head -20; exit $rc; }
echo "== bench"; date
timeout -k 10 300 python bench.py --steps ${STEPS:-400} --warmup 24 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-400
[ "${SKIP_PROF:-0}" = "1" ] && exit 0
echo "== rocprofv3"; date
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 64 --warmup 8 > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
