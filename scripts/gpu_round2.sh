#!/bin/bash
# GPU check of the current tree: all GPU tests, CML / SoilNet / IG benches, SoilNet kernel stats
# (writes gpurun_out/r2/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r2; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -6 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 400 --warmup 24 > $OUT/cml_bench.log 2>&1 || { tail -20 $OUT/cml_bench.log; exit 3; }
tail -1 $OUT/cml_bench.log
timeout -k 10 300 python bench.py --ds soilnet --steps 48 --warmup 8 > $OUT/soil_bench.log 2>&1 || { tail -20 $OUT/soil_bench.log; exit 3; }
tail -1 $OUT/soil_bench.log
timeout -k 10 300 python scripts/bench_ig.py --batches 8 > $OUT/ig_bench.log 2>&1 || { tail -20 $OUT/ig_bench.log; exit 3; }
tail -1 $OUT/ig_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_soil -o run --output-format csv -- python3 $ROOT/bench.py --ds soilnet --steps 10 --warmup 2 --no-graph > $OUT/prof_soil.log 2>&1
echo "rocprof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cml -o run --output-format csv -- python3 $ROOT/bench.py --steps 20 --warmup 3 --no-graph > $OUT/prof_cml.log 2>&1
echo "rocprof cml rc=$?"
