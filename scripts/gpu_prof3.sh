#!/bin/bash
# GCN micro timings (graph replay) + their rocprofv3 kernel stats; CML bench; rocprofv3 of the
# graph-mode bench (the measured path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/p3; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python scripts/gcn_micro.py > $OUT/gcn.jsonl 2>&1 || { tail -5 $OUT/gcn.jsonl; exit 4; }
grep -v amdgpu.ids $OUT/gcn.jsonl
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/profg -o run --output-format csv -- python3 $ROOT/bench.py --steps 50 --warmup 5 > $OUT/profg.log 2>&1
echo "rocprof graph rc=$?"
