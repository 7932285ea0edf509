#!/bin/bash
# round 6 experiment 2: role-specialised update kernels + the critic step's loss
# without unneeded block reductions: parity tests, then same-box A/B kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_learn_gpu.py \
  tests/test_target_pair_gpu.py tests/test_seeds_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r06_exp2_tests.log 2>&1 \
  || { tail -30 gpurun_out/r06_exp2_tests.log; exit 1; }
tail -3 gpurun_out/r06_exp2_tests.log
timeout -k 10 700 bash tools/gpu_trace_ab.sh r06rs "c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_base6.so c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_lb6.so c2:- c3:RLMD_LIB_PATH=tools/_abh/librlmd_amd_base6.so c3:-" > gpurun_out/r06rs.log 2>&1 || { tail -20 gpurun_out/r06rs.log; exit 1; }
tail -45 gpurun_out/r06rs.log
