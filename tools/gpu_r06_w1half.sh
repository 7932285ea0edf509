#!/bin/bash
# round 6: the actor step's fc1 blocks 16 units wide — learn parity tests, then same-box traces (new / HEAD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_learn_gpu.py \
  tests/test_target_pair_gpu.py tests/test_seeds_gpu.py > gpurun_out/r06_w1half_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_w1half_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 bash tools/gpu_trace_ab.sh w1half "c2:- c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_w1old.so c3:- c3:RLMD_LIB_PATH=tools/_abh/librlmd_amd_w1old.so c2:- c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_w1old.so" > gpurun_out/r06_w1half_ab.log 2>&1 \
  || { tail -20 gpurun_out/r06_w1half_ab.log; exit 1; }
grep -E "==|fwd_rows|qeval|critic_update|actor_update" gpurun_out/tab_w1half/summary.txt
