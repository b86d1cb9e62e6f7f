#!/bin/bash
# GPU-box session driver: runs the named steps in order, each under its own time limit, and stops at
# the first step that fails (no further GPU work after a fault, an abort or a time limit).
#
#   bash scripts/gpu_steps.sh tests bench soil ig phase stats pmc_cml pmc_soil
#
# Outputs go to gpurun_out/<step>.log (rocprof runs under gpurun_out/prof_<step>/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
PY=python3

run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "step $name rc=$rc"; exit $rc; fi
}

prof() {  # prof <name> <seconds> <rocprofv3 args...> -- <program...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    (cd /tmp && TMPDIR=/tmp timeout -k 10 "$secs" rocprofv3 "$@") > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "step $name rc=$rc"; exit $rc; fi
}

PMC_SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"

for step in "$@"; do
    case $step in
        tests)  run tests 600 $PY -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        smoke)  run smoke 300 $PY -c "import __graft_entry__ as g; g.smoke()" ;;
        bench)  run bench 300 $PY bench.py --steps 50 --warmup 10 ;;
        bench1) run bench1 600 $PY bench.py --gpus 1 --steps 20 --warmup 5 ;;
        soil)   run soil 300 $PY bench.py --ds soilnet --steps 20 --warmup 5 --no-knn-line ;;
        cnn)    run cnn 300 $PY bench.py --time-layer cnn --steps 40 --warmup 5 ;;
        stats_cnn) prof stats_cnn 400 --kernel-trace --stats -d "$OUT/prof_stats_cnn" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --time-layer cnn --steps 40 --warmup 5 ;;
        pmc_cnn) prof pmc_cnn 120 --kernel-trace --pmc $PMC_SQ -d "$OUT/prof_pmc_cnn" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --time-layer cnn --steps 16 --warmup 2 ;;
        pmc_cnn_mem) prof pmc_cnn_mem 120 --kernel-trace --pmc FETCH_SIZE -d "$OUT/prof_pmc_cnn_mem" -o run \
                    --output-format csv -- $PY "$ROOT/bench.py" --time-layer cnn --steps 16 --warmup 2 ;;
        pmc_cnn_wr) prof pmc_cnn_wr 120 --kernel-trace --pmc WRITE_SIZE -d "$OUT/prof_pmc_cnn_wr" -o run \
                    --output-format csv -- $PY "$ROOT/bench.py" --time-layer cnn --steps 16 --warmup 2 ;;
        cvcml)  run cvcml 400 $PY bench.py --steps 8 --warmup 2 --no-knn-line --no-ig-line --no-soil-line ${CV_ARGS:-} ;;
        cvsoil) run cvsoil 600 $PY bench.py --steps 8 --warmup 2 --no-knn-line --no-ig-line ${CV_ARGS:-} ;;
        ig)     run ig 300 $PY scripts/bench_ig.py ;;
        ar)     run ar 300 $PY scripts/ar_us.py ;;
        phase)  GNNQC_HIP_LIB=gnnqc/_lib/variants/prof.so run phase 300 $PY scripts/chain_phase_prof.py ;;
        stats)  prof stats 400 --kernel-trace --stats -d "$OUT/prof_stats" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --steps 40 --warmup 5 --no-knn-line --no-ig-line --no-cv-line --no-soil-line ;;
        stats_ng) prof stats_ng 400 --kernel-trace --stats -d "$OUT/prof_stats_ng" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --steps 40 --warmup 5 --no-knn-line --no-ig-line --no-cv-line --no-soil-line --no-graph ;;
        stats_ig) prof stats_ig 400 --kernel-trace --stats -d "$OUT/prof_stats_ig" -o run --output-format csv -- \
                    $PY "$ROOT/scripts/bench_ig.py" ;;
        pmc_ig) prof pmc_ig 120 --kernel-trace --pmc $PMC_SQ -d "$OUT/prof_pmc_ig" -o run --output-format csv -- \
                    $PY "$ROOT/scripts/bench_ig.py" --batches 2 ;;
        pmc_ig_mem) prof pmc_ig_mem 120 --kernel-trace --pmc FETCH_SIZE -d "$OUT/prof_pmc_ig_mem" -o run \
                    --output-format csv -- $PY "$ROOT/scripts/bench_ig.py" --batches 2 ;;
        pmc_ig_wr) prof pmc_ig_wr 120 --kernel-trace --pmc WRITE_SIZE -d "$OUT/prof_pmc_ig_wr" -o run \
                    --output-format csv -- $PY "$ROOT/scripts/bench_ig.py" --batches 2 ;;
        stats_soil) prof stats_soil 400 --kernel-trace --stats -d "$OUT/prof_stats_soil" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --ds soilnet --steps 20 --warmup 3 --no-graph ;;
        pmc_cml) prof pmc_cml 120 --kernel-trace --pmc $PMC_SQ -d "$OUT/prof_pmc_cml" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --steps 16 --warmup 2 --no-knn-line --no-cv-line --no-ig-line --no-soil-line ;;
        pmc_cml_mem) prof pmc_cml_mem 120 --kernel-trace --pmc FETCH_SIZE -d "$OUT/prof_pmc_cml_mem" -o run \
                    --output-format csv -- $PY "$ROOT/bench.py" --steps 16 --warmup 2 --no-knn-line --no-cv-line --no-ig-line --no-soil-line ;;
        pmc_cml_wr) prof pmc_cml_wr 120 --kernel-trace --pmc WRITE_SIZE -d "$OUT/prof_pmc_cml_wr" -o run \
                    --output-format csv -- $PY "$ROOT/bench.py" --steps 16 --warmup 2 --no-knn-line --no-cv-line --no-ig-line --no-soil-line ;;
        pmc_soil) prof pmc_soil 120 --kernel-trace --pmc $PMC_SQ -d "$OUT/prof_pmc_soil" -o run --output-format csv -- \
                    $PY "$ROOT/bench.py" --ds soilnet --steps 6 --warmup 2 --no-graph ;;
        pmc_soil_mem) prof pmc_soil_mem 120 --kernel-trace --pmc FETCH_SIZE -d "$OUT/prof_pmc_soil_mem" -o run \
                    --output-format csv -- $PY "$ROOT/bench.py" --ds soilnet --steps 6 --warmup 2 --no-graph ;;
        pmc_soil_wr) prof pmc_soil_wr 120 --kernel-trace --pmc WRITE_SIZE -d "$OUT/prof_pmc_soil_wr" -o run \
                    --output-format csv -- $PY "$ROOT/bench.py" --ds soilnet --steps 6 --warmup 2 --no-graph ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== done ($(date +%T))"
