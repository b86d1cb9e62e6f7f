#!/bin/bash
# SoilNet step: throughput, kernel stats, and HBM traffic counters (TCC FETCH_SIZE / WRITE_SIZE,
# one rocprofv3 --pmc pass each: FETCH_SIZE alone takes 3 of the 4 TCC counters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/soilpmc; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --ds soilnet --steps 30 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 3; }
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --ds soilnet --steps 10 --warmup 2 --no-graph > $OUT/prof.log 2>&1
echo "kernel trace rc=$?"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $OUT/pmc$i -o run --output-format csv -- python3 $ROOT/bench.py --ds soilnet --steps 3 --warmup 1 --no-graph > $OUT/pmc$i.log 2>&1
  echo "pmc $P rc=$?"
done
