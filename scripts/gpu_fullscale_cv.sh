#!/bin/bash
# Full-size CML network (3,904 links x 133,920 min, 20 flagged): all 5 CV folds in bf16 on one
# MI355X (writes gpurun_out/full/cv5.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/full; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1150 python -u scripts/cml_full_scale.py --all-folds --out $OUT/cv5.json > $OUT/cv5.log 2>&1
rc=$?; grep '^{' $OUT/cv5.log | tail -3 | cut -c1-600; exit $rc
