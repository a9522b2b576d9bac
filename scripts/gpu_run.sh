#!/bin/bash
# usage: bash scripts/gpu_run.sh <step>...   steps: smoke tests bench_small bench bench_cfg2 prof ablate stats pmcclk
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in "$@"; do
  case $s in
    smoke) timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1 ;;
    tests) timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 ;;
    bench_small) timeout -k 10 300 python bench.py --rows 1000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 ;;
    bench) timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 ;;
    bench_cfg5_small) timeout -k 10 600 python bench.py --workload cfg5 --rows 2000000 --steps 5 --warmup 2 > gpurun_out/bench_cfg5_small.log 2>&1 ;;
    bench_cfg5) timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 2 > gpurun_out/bench_cfg5.log 2>&1 ;;
    ivfab) for v in ${DYN:-0 1}; do VS_IVF_DYN=$v timeout -k 10 600 python bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-recall > gpurun_out/ivfab_$v.log 2>&1 || exit 1; grep '^{' gpurun_out/ivfab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dyn $v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/ivfab.txt; done ;;
    gemvab) for v in ${DYN:-0 1 0 1}; do VS_GEMV_DYN=$v timeout -k 10 300 python bench.py --workload cfg2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/gemvab_$v.log 2>&1 || exit 1; grep '^{' gpurun_out/gemvab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gemv dyn $v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/gemvab.txt; done ;;
    libab) for v in ${LIBS:-w0 w6 w8 w0 w6 w8}; do VS_LIB_PATH=$GRAFT_REPO_ROOT/abtmp/libvs_$v.so timeout -k 10 300 python bench.py --workload ${WL:-cfg2} --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/libab_$v.log 2>&1 || exit 1; grep '^{' gpurun_out/libab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lib $v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" >> gpurun_out/libab.txt; done ;;
    rfab) for v in ${LIBS:-plain rnt plain rnt}; do VS_LIB_PATH=$GRAFT_REPO_ROOT/abtmp/libvs_$v.so VS_RF_STAMPS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/rfab_$v.log 2>&1 || exit 1; echo "lib $v $(grep 'rf stamps' gpurun_out/rfab_$v.log | tail -1)" >> gpurun_out/rfab.txt; done ;;
    seedab) for v in ${SR:-0 1 0 1}; do for rows in 1250000 0; do VS_SEED_REUSE=$v timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/seedab_${v}_$rows.log 2>&1 || exit 1; grep '^{' gpurun_out/seedab_${v}_$rows.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('reuse $v rows $rows', d['ms_per_step'], d['roofline']['kernel_ms'], d['uncertified_first_pass'])" >> gpurun_out/seedab.txt; done; done ;;
    bench_cfg5_g4) VS_IVF_GRID=4 timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cfg5_g4.log 2>&1 ;;
    bench_cfg5_g16) VS_IVF_GRID=16 timeout -k 10 900 python bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cfg5_g16.log 2>&1 ;;
    bench_cfg2) timeout -k 10 600 python bench.py --workload cfg2 --steps 50 --no-cpu-baseline > gpurun_out/bench_cfg2.log 2>&1 ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 ;;
    ablate) for m in ${MODES:-0 1 2 0}; do VS_MF_ABLATE=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/ablate_$m.log 2>&1 || exit 1; tail -1 gpurun_out/ablate_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('mode $m', d['roofline']['kernel_ms'])" >> gpurun_out/ablate.txt; done ;;
    zero) for m in ${MODES:-9}; do VS_MF_ABLATE=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --zero-corpus > gpurun_out/zero_$m.log 2>&1 || exit 1; tail -1 gpurun_out/zero_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('zero mode $m', d['roofline']['kernel_ms'])" >> gpurun_out/ablate.txt; done ;;
    dist2) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --same-device --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dist2.log 2>&1 ;;
    rfprof) for v in ${LIBS:-plain qt}; do VS_LIB_PATH=$GRAFT_REPO_ROOT/abtmp/libvs_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rfprof_$v -o run --output-format csv -- python3 bench.py --rows ${ROWS:-1250000} --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rfprof_$v.log 2>&1 || exit 1; echo "lib $v $(grep -h 'k_refine\|k_screen_mfma<1, 0, 0>' gpurun_out/rfprof_$v/*/run_kernel_stats.csv gpurun_out/rfprof_$v/run_kernel_stats.csv 2>/dev/null | cut -d, -f1-4 | tr '\n' ' ')" >> gpurun_out/rfprof.txt; rm -rf gpurun_out/rfprof_$v/*/*trace* gpurun_out/rfprof_$v/*trace*; done ;;
    rowsweep) for rows in ${ROWSET:-1250000 2500000 5000000 10000000 1250000}; do timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/rowsweep_$rows.log 2>&1 || exit 1; grep '^{' gpurun_out/rowsweep_$rows.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rows $rows', d['ms_per_step'], d['roofline']['kernel_ms'])" >> gpurun_out/rowsweep.txt; done
      VS_MF_STAMPS=1 timeout -k 10 300 python bench.py --rows 1250000 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/stamps_1250k.log 2>&1 ;;
    k1ab) for rows in ${ROWSET:-1250000 10000000}; do for v in ${PCTS:-100 88 100 88}; do VS_K1_STATIC=$v timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/k1ab_${v}_$rows.log 2>&1 || exit 1; grep '^{' gpurun_out/k1ab_${v}_$rows.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('static% $v rows $rows', d['ms_per_step'], d['roofline']['kernel_ms'], d['uncertified_first_pass'])" >> gpurun_out/k1ab.txt; done; done ;;
    i8probe) for m in ${MODES:-0 9 28 9 28}; do VS_LIB_PATH=$GRAFT_REPO_ROOT/abtmp/libvs_abl.so VS_MF_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/i8p_$m -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/i8p_$m.log 2>&1 || exit 1; python3 -c "
import csv,glob,sys
for f in glob.glob('gpurun_out/i8p_$m/**/run_kernel_stats.csv', recursive=True) + glob.glob('gpurun_out/i8p_$m/run_kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_screen_mfma<1, 0, $m>' in r['Name']: print('mode $m', r['Calls'], r['AverageNs'], r['MinNs'])
" >> gpurun_out/i8probe.txt; rm -rf gpurun_out/i8p_$m/*/*trace* gpurun_out/i8p_$m/*trace*; done ;;
    rfstamps)VS_RF_STAMPS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/rfstamps.log 2>&1 ;;
    stamps) VS_MF_STAMPS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/stamps.log 2>&1 ;;
    stats) VS_MF_STATS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/stats.log 2>&1 ;;
    pmcab) for m in ${MODES:-0 9}; do
        VS_MF_ABLATE=$m timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmcab$m -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcab$m.log 2>&1 || exit 1
        VS_MF_ABLATE=$m timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU -d gpurun_out/pmcbb$m -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcbb$m.log 2>&1 || exit 1
      done ;;
    pmcclk) for m in ${MODES:-0 9}; do
        VS_MF_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmcclk$m -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcclk$m.log 2>&1 || exit 1
        VS_MF_ABLATE=$m timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmclds$m -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmclds$m.log 2>&1 || exit 1
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
