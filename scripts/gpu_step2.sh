#!/bin/bash
# CML step work: focused tests -> kernel timeline -> bench -> rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/step; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== tests"; date
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests/test_cml_fused_gpu.py} -x -v -p no:cacheprovider \
    --timeout 180 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
echo "== trace"; date
timeout -k 10 120 python scripts/chain_head_trace.py > $OUT/trace.jsonl 2>&1 || { tail -5 $OUT/trace.jsonl; exit 5; }
cat $OUT/trace.jsonl | grep -v amdgpu.ids
echo "== bench"; date
timeout -k 10 300 python bench.py --steps ${STEPS:-300} --warmup 20 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log
[ "${SKIP_PROF:-0}" = "1" ] && exit 0
echo "== rocprofv3"; date
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 3 --no-graph > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
