#!/bin/bash
# same-box A/B of compile-time variant libraries: bench (training step only) + chain timeline per library
# usage: bash scripts/gpu_variants_ab.sh lib1.so lib2.so ...   (STEPS, REPS env)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ab
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    GNNQC_HIP_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 24 --no-knn-line --no-ig-line \
      --no-cv-line > gpurun_out/ab/$n.$rep.log 2>&1 || { tail -20 gpurun_out/ab/$n.$rep.log; exit 3; }
    echo "$n $(tail -1 gpurun_out/ab/$n.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
  done
done
if [ -n "$TIMELINE" ]; then
  for lib in "$@"; do
    n=$(basename $lib .so)
    GNNQC_HIP_LIB=$lib timeout -k 10 120 python scripts/chain_head_timeline.py > gpurun_out/ab/tl_$n.log 2>&1 || exit 3
    echo "$n $(tail -1 gpurun_out/ab/tl_$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print([(r['loop_start_us'], r['end_us']) for r in d['bwd_blocks_tile0']])")"
  done
fi
