#!/bin/bash
# One GPU call of round-6 steps (STEPS="..." bash scripts/r06_gpu_batch.sh).  Every step runs under
# its own time limit; a crash, abort, fault or time limit (rc >= 124) ends the call there.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
fatal() { [ "$1" -ge 124 ] && [ "$1" -ne 0 ]; }
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc" >> gpurun_out/steps.log
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping" >> gpurun_out/steps.log; exit $rc; fi
  return 0
}
abloop() {  # name, reps, args... : bench.py with --k1-schedule $ABS (default "0 1") alternating
  local name=$1 reps=$2; shift 2
  for i in $(seq 1 $reps); do for s in ${ABS:-0 1}; do
    timeout -k 10 300 python bench.py --k1-schedule $s "$@" --no-cpu-baseline > gpurun_out/ab.tmp 2>&1
    local rc=$?
    echo "sched$s $(tail -1 gpurun_out/ab.tmp)" >> gpurun_out/ab_$name.txt
    if [ $rc -ne 0 ]; then cp gpurun_out/ab.tmp gpurun_out/ab_${name}_fail.log; echo "step ab_$name rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
  done; done
  echo "step ab_$name rc=0" >> gpurun_out/steps.log
}
for s in ${STEPS:-decomp}; do
  case $s in
    full) run pytest_gpu 900 $PYT tests -m gpu ;;
    full1) VS_TEST_K1_SCHEDULE=1 run pytest_gpu_sched1 900 $PYT tests -m gpu ;;
    direct1) VS_TEST_K1_SCHEDULE=1 run pytest_direct_sched1 600 $PYT tests/test_gpu_int8_direct.py tests/test_gpu_baseline_shapes.py -m gpu ;;
    smoke) run smoke 300 python __graft_entry__.py --smoke ;;
    decomp) run k1_decompose 600 python scripts/k1_decompose.py --out gpurun_out/k1_decomposition.json ;;
    cfg3) run bench_cfg3 600 python bench.py ;;
    ab3) abloop cfg3 2 --steps 20 --warmup 3 ;;
    ab3n) abloop cfg3n 2 --screen native --steps 10 --warmup 3 ;;
    ab) for i in 1 2; do for lib in $ABLIBS; do
           VS_LIB_PATH=$lib timeout -k 10 300 python bench.py $ABARGS --no-cpu-baseline > gpurun_out/ab.tmp 2>&1
           rc=$?; echo "$lib $(tail -1 gpurun_out/ab.tmp)" >> gpurun_out/ab_$ABNAME.txt
           if [ $rc -ne 0 ]; then cp gpurun_out/ab.tmp gpurun_out/ab_${ABNAME}_fail.log; echo "step ab rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
         done; done; echo "step ab rc=0" >> gpurun_out/steps.log ;;
    abprod) for i in 1 2; do for lib in $ABLIBS; do
           VS_LIB_PATH=$lib timeout -k 10 300 python scripts/product_latency.py $PRODARGS > gpurun_out/ab.tmp 2>&1
           rc=$?; echo "$lib $(tail -1 gpurun_out/ab.tmp)" >> gpurun_out/abprod_$ABNAME.txt
           if [ $rc -ne 0 ]; then cp gpurun_out/ab.tmp gpurun_out/abprod_${ABNAME}_fail.log; echo "step abprod rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
         done; done; echo "step abprod rc=0" >> gpurun_out/steps.log ;;
    trace8) mkdir -p gpurun_out/trace8 && run trace8 300 rocprofv3 --kernel-trace -d gpurun_out/trace8 -o t --output-format csv -- python bench.py --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline && \
      python scripts/trace_tail.py $(ls gpurun_out/trace8/*/t_kernel_trace.csv gpurun_out/trace8/t_kernel_trace.csv 2>/dev/null | head -1) 80 "vs::|copyBuffer|nccl|rccl|Kernel" > gpurun_out/trace8_tail.txt && rm -rf gpurun_out/trace8 ;;
    trace3) mkdir -p gpurun_out/trace3 && run trace3 300 rocprofv3 --kernel-trace -d gpurun_out/trace3 -o t --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline && \
      python scripts/trace_tail.py $(ls gpurun_out/trace3/*/t_kernel_trace.csv gpurun_out/trace3/t_kernel_trace.csv 2>/dev/null | head -1) 60 "vs::|copyBuffer|Kernel" > gpurun_out/trace3_tail.txt && rm -rf gpurun_out/trace3 ;;
    ivf) run pytest_ivf 600 $PYT tests/test_gpu_ivf.py tests/test_gpu_baseline_shapes.py -m gpu -k "ivf or cfg5" ;;
    dist) run pytest_dist 600 $PYT tests/test_gpu_distributed.py tests/test_gpu_multi_device.py tests/test_gpu_int8_direct.py tests/test_gpu_int8_clustered.py -m gpu ;;
    full0) VS_TEST_K1_SCHEDULE=0 run pytest_gpu_sched0 900 $PYT tests -m gpu ;;
    ab8) abloop shard8 2 --shard-of 8 --steps 30 ;;
    shard8) run bench_shard8 300 python bench.py --shard-of 8 --steps 30 --no-cpu-baseline ;;
    cfg2) run bench_cfg2 300 python bench.py --workload cfg2 --no-cpu-baseline ;;
    cfg1) run bench_cfg1 300 python bench.py --workload cfg1 --steps 1000 --warmup 50 ;;
    shard2) run bench_shard2 300 python bench.py --shard-of 2 --steps 20 --no-cpu-baseline ;;
    shard4) run bench_shard4 300 python bench.py --shard-of 4 --steps 30 --no-cpu-baseline ;;
    cfg5skew) run bench_cfg5_skew 900 python bench.py --workload cfg5 --skew 1.1 --steps 10 --warmup 2 ;;
    prod) run product_latency_int8 300 python scripts/product_latency.py --calls 300 --screen int8 && run product_latency_native 300 python scripts/product_latency.py --calls 300 --screen native ;;
    cfg5) run bench_cfg5 900 python bench.py --workload cfg5 --steps 10 --warmup 2 ;;
    cfg4) run bench_cfg4 900 python bench.py --workload cfg4 --steps 10 --warmup 3 --no-cpu-baseline ;;
    mix10) run bench_mix10 600 python bench.py --data mixture-sorted --sigma 1.0 --warmup 8 --no-cpu-baseline ;;
    mix05) run bench_mix05 600 python bench.py --data mixture-sorted --sigma 0.5 --warmup 8 --no-cpu-baseline ;;
    profcfg2) TAG=r06_cfg2 ARGS="--workload cfg2 --steps 200 --warmup 20 --no-cpu-baseline" PASSES="sq lds" timeout -k 10 1100 bash scripts/gpu_prof.sh > gpurun_out/prof_cfg2.log 2>&1
      rc=$?; echo "step profcfg2 rc=$rc" >> gpurun_out/steps.log; if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi ;;
    profcfg3) TAG=${PTAG:-r06_final_cfg3} ARGS="--steps 20 --warmup 3 --no-cpu-baseline" PASSES=sq timeout -k 10 1100 bash scripts/gpu_prof.sh > gpurun_out/prof_cfg3.log 2>&1
      rc=$?; echo "step profcfg3 rc=$rc" >> gpurun_out/steps.log; if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi ;;
    prof3) mkdir -p gpurun_out/prof3 && run prof3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 30 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s" >> gpurun_out/steps.log; exit 2 ;;
  esac
done
