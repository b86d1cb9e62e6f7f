#!/bin/bash
# Full-size CML network (3,904 links x 133,920 min, 20 flagged) through generation, preprocessing,
# the HBM-resident store and one CV fold in bf16 and fp32 (writes gpurun_out/full/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/full; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u scripts/cml_full_scale.py --fp32 --out $OUT/full.json > $OUT/full.log 2>&1
rc=$?; tail -5 $OUT/full.log; exit $rc
