#!/bin/bash
# same-box A/B of the default build against a variant library: chain GPU tests, kernel traces of both,
# then driver-form bench runs alternating the two.  VARIANT=gnnqc/_lib/variants/<name>.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
V=${VARIANT:?VARIANT=<variant .so>}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k chain \
  tests/test_cml_fused_gpu.py > gpurun_out/t_ablib.log 2>&1 \
  && tail -1 gpurun_out/t_ablib.log \
  && VARIANTS="new:- old:GNNQC_HIP_LIB=$V" bash scripts/gpu_prof_variants.sh \
  && for r in 1 2; do
    for v in new old; do
      if [ $v = old ]; then export GNNQC_HIP_LIB=$V; else unset GNNQC_HIP_LIB; fi
      timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-ig-line --no-cv-line --no-soil-line \
        > gpurun_out/bench_ab_${v}_$r.log 2>&1 || exit 3
      echo "$v run $r: $(grep -m1 -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ab_${v}_$r.log)"
    done
  done
