#!/bin/bash
# IG with the HIP probability head: GPU tests, IG throughput A/B, kernel table of one IG run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ig_gpu.py > gpurun_out/t_ig.log 2>&1 && tail -1 gpurun_out/t_ig.log \
  && timeout -k 10 300 python scripts/bench_ig.py --batches 4 > gpurun_out/ig1.json 2> gpurun_out/ig1.err && cat gpurun_out/ig1.json \
  && GNNQC_IG_HEAD_HIP=0 timeout -k 10 300 python scripts/bench_ig.py --batches 4 > gpurun_out/ig0.json 2> gpurun_out/ig0.err && cat gpurun_out/ig0.json \
  && cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_ig" -o run --output-format csv \
     -- python3 "$ROOT/scripts/bench_ig.py" --batches 2 > "$ROOT/gpurun_out/prof_ig.log" 2>&1 \
  && cd "$ROOT" && python3 scripts/prof_summary.py gpurun_out/prof_ig/run_kernel_stats.csv 3 40 > gpurun_out/ig_stats.txt 2>&1 && cat gpurun_out/ig_stats.txt
