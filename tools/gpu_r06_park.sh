#!/bin/bash
# round 6: acting values parked in LDS (no scratch spills at 4 workgroups per CU) —
# acting / fused-env parity tests, same-box traces (new / HEAD), FETCH / WRITE passes of the new code
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fused_env_gpu.py tests/test_fullsize_gpu.py tests/test_seeds_gpu.py \
  tests/test_train_gpu.py tests/test_learn_gpu.py tests/test_eval_gpu.py > gpurun_out/r06_park_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_park_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/gpu_trace_ab.sh park "c2:- c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_parkold.so c3:- c3:RLMD_LIB_PATH=tools/_abh/librlmd_amd_parkold.so c4:- c4:RLMD_LIB_PATH=tools/_abh/librlmd_amd_parkold.so c2:-" > gpurun_out/r06_park_ab.log 2>&1 \
  || { tail -20 gpurun_out/r06_park_ab.log; exit 1; }
grep -E "==|act_env|fused_act|fwd_rows" gpurun_out/tab_park/summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH="bench.py --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --steps 25 --warmup 5"
OUT=gpurun_out/prof_park
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "act_env_kernel|fused_act_kernel|env_train_kernel" -f csv -d $OUT/fetch -o fetch -- python3 $BENCH > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "act_env_kernel|fused_act_kernel|env_train_kernel" -f csv -d $OUT/write -o write -- python3 $BENCH > $OUT/write.log 2>&1 || exit 1
echo ALLDONE
