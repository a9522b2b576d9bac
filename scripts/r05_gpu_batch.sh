#!/bin/bash
# One GPU call of round-5 checks: the changed/new GPU suites (all of them run: a failing test does
# not stop the call), then the benches.  A crash, abort, fault or time limit (rc 124/134/137/139 or
# any rc > 128) ends the call there.
#   STEPS="tests cfg3 shard8 mix03 micro multi" bash scripts/r04_gpu_batch.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
TESTS=${TESTS:-"tests/test_gpu_int8_direct.py tests/test_gpu_int8_clustered.py tests/test_gpu_multi_device.py tests/test_gpu_hnsw_build.py tests/test_gpu_hnsw.py tests/test_gpu_cfg1.py tests/test_gpu_int8_screen.py tests/test_gpu_distributed.py"}
fatal() { [ "$1" -ge 124 ] && [ "$1" -ne 0 ]; }
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc" >> gpurun_out/steps.log
  if fatal $rc; then echo "fatal rc=$rc in $name: stopping" >> gpurun_out/steps.log; exit $rc; fi
  return 0
}
for s in ${STEPS:-tests cfg3 shard8 mix03 micro multi}; do
  case $s in
    tests) run pytest_new 1500 $PYT $TESTS -m gpu ;;
    full) run pytest_gpu 1500 $PYT tests -m gpu ;;
    smoke) run smoke 300 python __graft_entry__.py --smoke ;;
    cfg3) run bench_cfg3 600 python bench.py ;;
    cfg1) run bench_cfg1 300 python bench.py --workload cfg1 --steps 1000 --warmup 50 ;;
    shard8) run bench_shard8 300 python bench.py --shard-of 8 --steps 30 --no-cpu-baseline ;;
    shard2) run bench_shard2 300 python bench.py --shard-of 2 --steps 20 --no-cpu-baseline ;;
    shard4) run bench_shard4 300 python bench.py --shard-of 4 --steps 30 --no-cpu-baseline ;;
    spawn2) run bench_spawn2 600 python bench.py --gpus 2 --same-device --dist-backend gloo --rows 2000000 --steps 10 --no-cpu-baseline ;;
    mix03) run bench_mix03 600 python bench.py --data mixture-sorted --sigma 0.3 --warmup 8 --no-cpu-baseline ;;
    mix05) run bench_mix05 600 python bench.py --data mixture-sorted --sigma 0.5 --warmup 8 --no-cpu-baseline ;;
    mix10) run bench_mix10 600 python bench.py --data mixture-sorted --sigma 1.0 --warmup 8 --no-cpu-baseline ;;
    micro32) for m in 21 22 9; do for dt in 1 2; do
             timeout -k 10 120 ./abtmp/k1_micro 10000000 1536 20 $dt $m >> gpurun_out/k1_micro32.txt 2>&1
             rc=$?; if [ $rc -ne 0 ]; then echo "step micro32 rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
           done; done; echo "step micro32 rc=0" >> gpurun_out/steps.log ;;
    micro) for m in 0 2 9; do for dt in 1 2; do
             timeout -k 10 120 ./abtmp/k1_micro 10000000 1536 20 $dt $m >> gpurun_out/k1_micro.txt 2>&1
             rc=$?; if [ $rc -ne 0 ]; then echo "step micro rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
           done; done; echo "step micro rc=0" >> gpurun_out/steps.log ;;
    cfg2) run bench_cfg2 300 python bench.py --workload cfg2 --no-cpu-baseline ;;
    profmix05) mkdir -p gpurun_out/prof_mix05 && run prof_mix05 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix05 -o run --output-format csv -- python bench.py --data mixture-sorted --sigma 0.5 --screen native --steps 5 --warmup 3 --no-cpu-baseline ;;
    diagmix10m) run diag_mix03_10m 600 python scripts/diag_mixture.py --sorted --sigma 0.3 --rows 10000000 --batches 4 --check ;;
    diagmix) run diag_mix03 600 python scripts/diag_mixture.py --sorted --sigma 0.3 ;;
    multi) run multi_step 600 python scripts/multi_step_timing.py ;;
    cfg5skew) run bench_cfg5_skew 900 python bench.py --workload cfg5 --skew 1.1 --steps 10 --warmup 2 ;;
    cfg5skewpmc) mkdir -p gpurun_out/pmc5f gpurun_out/pmc5w && \
      run pmc5_fetch 900 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc5f -o p --output-format csv -- python bench.py --workload cfg5 --skew 1.1 --steps 3 --warmup 1 && \
      run pmc5_write 900 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc5w -o p --output-format csv -- python bench.py --workload cfg5 --skew 1.1 --steps 3 --warmup 1 && \
      run ivf_traffic 120 python scripts/ivf_traffic.py gpurun_out/pmc5f gpurun_out/pmc5w gpurun_out/traffic_cfg5_skew.json 1.1 50000000 && \
      rm -rf gpurun_out/pmc5f gpurun_out/pmc5w ;;
    trace8) mkdir -p gpurun_out/trace8 && run trace8 300 rocprofv3 --kernel-trace -d gpurun_out/trace8 -o t --output-format csv -- python bench.py --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline && \
      python scripts/trace_tail.py $(ls gpurun_out/trace8/*/t_kernel_trace.csv gpurun_out/trace8/t_kernel_trace.csv 2>/dev/null | head -1) 80 "vs::|copyBuffer|nccl|rccl|Kernel" > gpurun_out/trace8_tail.txt && rm -rf gpurun_out/trace8 ;;
    trace2) mkdir -p gpurun_out/trace2 && run trace2 300 rocprofv3 --kernel-trace -d gpurun_out/trace2 -o t --output-format csv -- python bench.py --workload cfg2 --steps 20 --warmup 3 --no-cpu-baseline && \
      python scripts/trace_tail.py $(ls gpurun_out/trace2/*/t_kernel_trace.csv gpurun_out/trace2/t_kernel_trace.csv 2>/dev/null | head -1) 60 "vs::|copyBuffer|Kernel" > gpurun_out/trace2_tail.txt && rm -rf gpurun_out/trace2 ;;
    product) run product_native 300 python scripts/product_latency.py && run product_int8 300 python scripts/product_latency.py --screen int8 ;;
    cfg4) run bench_cfg4 1100 python bench.py --workload cfg4 --steps 10 --warmup 3 --no-cpu-baseline ;;
    cfg5) run bench_cfg5 900 python bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline ;;
    stamps) run stamps_1250k 300 python scripts/refine_stamps.py --run --rows 1250000 && run stamps_10m 300 python scripts/refine_stamps.py --run --rows 10000000 ;;
    trace1) mkdir -p gpurun_out/trace1 && run trace1 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/trace1 -o t --output-format csv -- python bench.py --workload cfg1 --steps 200 --warmup 20 && \
      python scripts/trace_tail.py $(ls gpurun_out/trace1/*/t_kernel_trace.csv gpurun_out/trace1/t_kernel_trace.csv 2>/dev/null | head -1) 40 "vs::|copyBuffer|Kernel" > gpurun_out/trace1_tail.txt && \
      cp $(ls gpurun_out/trace1/*/t_memory_copy_trace.csv gpurun_out/trace1/t_memory_copy_trace.csv 2>/dev/null | head -1) gpurun_out/trace1_memcpy.csv; rm -rf gpurun_out/trace1 ;;
    stamps1) run stamps1_1m 300 python scripts/refine_stamps.py --run --rows 1000000 --single ;;
    stamps2) run stamps2_1250k 300 python scripts/refine_stamps.py --run --rows 1250000 --two-phase 8 ;;
    ab8) for i in 1 2; do for lib in diag/libvs_base.so photo_search_engine_amd/libvs.so; do
           VS_LIB_PATH=$lib timeout -k 10 300 python bench.py --shard-of 8 --steps 30 --no-cpu-baseline > gpurun_out/ab8.tmp 2>&1
           rc=$?; echo "$lib $(tail -1 gpurun_out/ab8.tmp)" >> gpurun_out/ab8.txt
           if [ $rc -ne 0 ]; then echo "step ab8 rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
         done; done; echo "step ab8 rc=0" >> gpurun_out/steps.log ;;
    ab3) for i in 1 2; do for lib in diag/libvs_base.so photo_search_engine_amd/libvs.so; do
           VS_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab3.tmp 2>&1
           rc=$?; echo "$lib $(tail -1 gpurun_out/ab3.tmp)" >> gpurun_out/ab3.txt
           if [ $rc -ne 0 ]; then echo "step ab3 rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
         done; done; echo "step ab3 rc=0" >> gpurun_out/steps.log ;;
    ab) for i in 1 2; do for lib in $ABLIBS; do
           VS_LIB_PATH=$lib timeout -k 10 300 python bench.py $ABARGS --no-cpu-baseline > gpurun_out/ab.tmp 2>&1
           rc=$?; echo "$lib $(tail -1 gpurun_out/ab.tmp)" >> gpurun_out/ab_$ABNAME.txt
           if [ $rc -ne 0 ]; then echo "step ab rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
         done; done; echo "step ab rc=0" >> gpurun_out/steps.log ;;
    ab2) for i in 1 2; do for lib in diag/libvs_base.so photo_search_engine_amd/libvs.so; do
           VS_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload cfg2 --no-cpu-baseline > gpurun_out/ab2.tmp 2>&1
           rc=$?; echo "$lib $(tail -1 gpurun_out/ab2.tmp)" >> gpurun_out/ab2.txt
           if [ $rc -ne 0 ]; then echo "step ab2 rc=$rc" >> gpurun_out/steps.log; exit $rc; fi
         done; done; echo "step ab2 rc=0" >> gpurun_out/steps.log ;;
    hnswins) run hnsw_insert 900 python scripts/hnsw_insert_timing.py ;;
    hnsw) run hnsw_bench 900 python scripts/hnsw_bench.py ;;
    smallscan) run small_scan 600 python scripts/small_scan_timing.py ;;
    tracemulti) mkdir -p gpurun_out/tracem && run tracemulti 600 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tracem -o t --output-format csv -- python scripts/multi_step_timing.py --reps 3 && \
      python scripts/trace_merge.py gpurun_out/tracem 140 > gpurun_out/tracem_tail.txt && rm -rf gpurun_out/tracem ;;
    trace3) mkdir -p gpurun_out/trace3 && run trace3 300 rocprofv3 --kernel-trace -d gpurun_out/trace3 -o t --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline && \
      python scripts/trace_tail.py $(ls gpurun_out/trace3/*/t_kernel_trace.csv gpurun_out/trace3/t_kernel_trace.csv 2>/dev/null | head -1) 60 "vs::|copyBuffer|Kernel" > gpurun_out/trace3_tail.txt && rm -rf gpurun_out/trace3 ;;
    prof3) mkdir -p gpurun_out/prof3 && run prof3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 30 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $s" >> gpurun_out/steps.log; exit 2 ;;
  esac
done
