#!/bin/bash
# SoilNet GCN training-step throughput + kernel profile (diagnostic; not the headline bench).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/soil; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --ds soilnet --steps 30 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --ds soilnet --steps 30 --warmup 5 --model baseline > $OUT/bench_base.log 2>&1 || { tail -20 $OUT/bench_base.log; exit 3; }
tail -1 $OUT/bench_base.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --ds soilnet --steps 10 --warmup 2 --no-graph > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
