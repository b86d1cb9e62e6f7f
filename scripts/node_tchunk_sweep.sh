set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for tc in 1 4 8; do
  GNNQC_NODE_TCHUNK=$tc timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sw_$tc -o run --output-format csv -- python bench.py --ds soilnet --steps 20 --warmup 5 --no-knn-line > gpurun_out/sw_$tc.log 2>&1
done
