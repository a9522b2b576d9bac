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
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_sq -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_sq.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_lds -o p --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_lds.log 2>&1 || exit 1
echo "profile passes done: summarise locally with python3 scripts/prof_summary.py $OUT $TAG"
