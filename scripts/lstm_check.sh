#!/bin/bash
# LSTM kernel validation: GPU kernel tests, per-layer microbench (default kernels vs v1), training bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lstm_check; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/lstm_microbench.py --M 128 1024 > $OUT/micro_new.jsonl 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $OUT/bench.log 2>&1 || exit 3
GNNQC_NO_TM=1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $OUT/bench_notm.log 2>&1 || exit 3
tail -1 $OUT/bench_notm.log | cut -c1-200
tail -1 $OUT/bench.log | cut -c1-250
cat $OUT/micro_new.jsonl | grep '"M": 128'
ROOT=$(pwd)
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5) > $OUT/prof.log 2>&1
echo "prof rc=$?"
