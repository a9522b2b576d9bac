#!/bin/bash
# usage: bash scripts/gpu_run.sh <step>...   (on the GPU box, through gpurun)
#   smoke tests t_new shapes bench_cfg1 bench_spawn2 bench bench_i8 bench_cfg2 bench_cfg4 bench_cfg5 bench_cfg5_skew prof prof_i8 rowsweep
# Every GPU step runs under its own time limit; the first failing step ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in "$@"; do
  case $s in
    smoke) timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1 ;;
    tests) timeout -k 10 1200 $PYT tests -m gpu --durations=15 > gpurun_out/pytest_gpu.log 2>&1 ;;
    shapes) timeout -k 10 600 $PYT tests/test_gpu_baseline_shapes.py -m gpu --durations=0 > gpurun_out/shapes.log 2>&1 ;;
    quick) timeout -k 10 900 $PYT tests -m gpu -k "${K:-not baseline_shapes}" > gpurun_out/pytest_quick.log 2>&1 ;;
    t_new) timeout -k 10 900 $PYT ${TESTS_NEW:-tests/test_gpu_cfg1.py} -m gpu > gpurun_out/pytest_new.log 2>&1 ;;
    bench_cfg1) timeout -k 10 300 python bench.py --workload cfg1 --steps 1000 --warmup 50 > gpurun_out/bench_cfg1.log 2>&1 ;;
    bench_spawn2) timeout -k 10 600 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 10 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_spawn2.log 2>&1 ;;
    bench) timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 ;;
    bench_i8) timeout -k 10 600 python bench.py --screen int8 > gpurun_out/bench_i8.log 2>&1 ;;
    bench_bf16) timeout -k 10 600 python bench.py --screen bf16 > gpurun_out/bench_bf16.log 2>&1 ;;
    bench_cfg2) timeout -k 10 600 python bench.py --workload cfg2 --steps 50 > gpurun_out/bench_cfg2.log 2>&1 ;;
    bench_cfg4) timeout -k 10 900 python bench.py --workload cfg4 --steps 10 > gpurun_out/bench_cfg4.log 2>&1 ;;
    bench_cfg5) timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 2 > gpurun_out/bench_cfg5.log 2>&1 ;;
    bench_cfg5_skew) timeout -k 10 900 python bench.py --workload cfg5 --skew 1.1 --steps 10 --warmup 2 > gpurun_out/bench_cfg5_skew.log 2>&1 ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 ;;
    rowsweep) for rows in ${ROWSET:-1250000 2500000 5000000 10000000}; do timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/rowsweep_$rows.log 2>&1 || exit 1; grep '^{' gpurun_out/rowsweep_$rows.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows $rows', d['ms_per_step'], d['roofline']['kernel_ms'], d['uncertified_first_pass'])" >> gpurun_out/rowsweep.txt; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
