#!/bin/bash
# Targeted GPU check: selected kernel tests (-k) then the SoilNet step bench/profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/new; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "${K:-padded or gcn_node or soilnet}" > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
[ "${SOIL:-1}" = "1" ] || exit 0
timeout -k 10 300 python bench.py --ds soilnet --steps 30 --warmup 5 > $OUT/soil_bench.log 2>&1 || { tail -20 $OUT/soil_bench.log; exit 3; }
tail -1 $OUT/soil_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --ds soilnet --steps 10 --warmup 2 --no-graph > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
