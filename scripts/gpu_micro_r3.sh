#!/bin/bash
# small-kernel micro profiles (scripts/step_kernels_micro.py) and the TimeLayer kernel timeline
# (scripts/chain_head_trace.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/micro; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python scripts/step_kernels_micro.py > $OUT/kern.jsonl 2>&1 || { tail -20 $OUT/kern.jsonl; exit 3; }
grep kernel $OUT/kern.jsonl
timeout -k 10 200 python scripts/chain_head_trace.py > $OUT/timeline.jsonl 2>&1 || { tail -20 $OUT/timeline.jsonl; exit 4; }
grep us $OUT/timeline.jsonl
timeout -k 10 200 python scripts/chain_phase_prof.py > $OUT/phase.jsonl 2>&1 || { tail -20 $OUT/phase.jsonl; exit 5; }
grep -v amdgpu.ids $OUT/phase.jsonl
