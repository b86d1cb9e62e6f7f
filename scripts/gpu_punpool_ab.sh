#!/bin/bash
# producer-side un-pooling in the chain backward (GNNQC_CHAINB_PUNPOOL): chain GPU tests, kernel
# traces with / without, then driver-form bench runs alternating the two
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k chain \
  tests/test_cml_fused_gpu.py tests/test_gcn_fused_gpu.py > gpurun_out/t_punpool.log 2>&1 \
  && tail -3 gpurun_out/t_punpool.log \
  && VARIANTS="${VARIANTS:-pu1:- pu0:GNNQC_CHAINB_PUNPOOL=0}" bash scripts/gpu_prof_variants.sh \
  && for r in 1 2; do
    for v in 1 0; do
      GNNQC_CHAINB_PUNPOOL=$v timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/bench_pu${v}_$r.log 2>&1 || exit 3
      echo "pu$v run $r: $(grep -m1 '"metric"' gpurun_out/bench_pu${v}_$r.log)"
    done
  done
