#!/bin/bash
# profiling passes (separate runs: kernel trace, then PMC sets) for one bench configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
ARGS=${ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/kt.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc1 -o pmc1 --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/pmc1.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE -d gpurun_out/prof/pmc2 -o pmc2 --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/pmc2.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL -d gpurun_out/prof/pmc3 -o pmc3 --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/pmc3.log 2>&1 || exit 1
echo done
