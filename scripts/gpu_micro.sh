#!/bin/bash
# GCN micro timings + their rocprofv3 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/micro; mkdir -p $OUT
timeout -k 10 120 python scripts/gcn_micro.py > $OUT/gcn.jsonl 2>&1 || { tail -5 $OUT/gcn.jsonl; exit 4; }
grep -v amdgpu.ids $OUT/gcn.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/scripts/gcn_micro.py > $OUT/prof.log 2>&1
echo "rocprof rc=$?"
