#!/bin/bash
# usage: bash scripts_gpu_run.sh <step>...   steps: smoke tests bench_small bench prof
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in "$@"; do
  case $s in
    smoke) timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1 ;;
    tests) timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 ;;
    bench_small) timeout -k 10 300 python bench.py --rows 1000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 ;;
    bench) timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 ;;
    bench_cfg2) timeout -k 10 600 python bench.py --workload cfg2 --steps 50 --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1 ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
