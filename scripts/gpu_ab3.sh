cd "${GRAFT_REPO_ROOT}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B=${B:-$PWD/gnnqc/_lib/variants/base.so}
VARIANTS="${V3:-cur:- base:GNNQC_HIP_LIB=$B}" bash scripts/gpu_prof_variants.sh > gpurun_out/ab3.txt 2>&1 || exit 3
for r in 1 2; do
  for v in ${V3N:-cur base}; do
    ( [ $v = pu0 ] && export GNNQC_CHAINB_PUNPOOL=0; [ $v = base ] && export GNNQC_HIP_LIB=$B
      timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-ig-line --no-cv-line > gpurun_out/b3_${v}_$r.log 2>&1 ) || exit 3
    echo "$v $r $(grep -m1 -o '"ms_per_step": [0-9.]*' gpurun_out/b3_${v}_$r.log)" >> gpurun_out/ab3.txt
  done
done
