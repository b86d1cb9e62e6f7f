#!/bin/bash
# SQ counters for the LSTM recurrence kernels on one layer shape (T=181, Din=16, H=16, M=128).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM \
  -d $OUT -o run --output-format csv -- python3 $ROOT/scripts/lstm_microbench.py --M 128 --reps 3 --only ${SHAPE:-181,16,16} > $OUT/log.txt 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/log.txt; ls $OUT
exit $rc
