#!/bin/bash
# Profiling passes for one bench configuration, each its own rocprofv3 run (kernel trace + stats,
# then PMC sets with kernel trace only), then a summary into profiles/ (scripts/prof_summary.py).
#   TAG=r01_cfg3 ARGS="--steps 5 --warmup 2 --no-cpu-baseline" bash scripts/gpu_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r01_cfg3}
ARGS=${ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# raw traces of a long run exceed what gpurun copies back: drop them however the script ends
trap 'rm -rf $OUT/kt/*trace* $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_sq $OUT/pmc_lds' EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit 1
[[ " ${PASSES:-sq lds} " == *" sq "* ]] && { timeout -k 10 600 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_sq -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_sq.log 2>&1 || exit 1; }
[[ " ${PASSES:-sq lds} " == *" lds "* ]] && { timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_lds -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_lds.log 2>&1 || exit 1; }
# summarise on the box (raw traces of a long build exceed what gpurun copies back), keep the summary
mkdir -p gpurun_out/profiles_out
PROF_OUT=gpurun_out/profiles_out python3 scripts/prof_summary.py $OUT $TAG > gpurun_out/profiles_out/summary_$TAG.log 2>&1 || exit 1
cp $OUT/kt/kt_kernel_stats.csv gpurun_out/profiles_out/${TAG}_kernel_stats.csv
cp $OUT/kt.log gpurun_out/profiles_out/${TAG}_bench.log
echo "profile passes done: summary in gpurun_out/profiles_out"
