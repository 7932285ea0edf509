#!/bin/bash
# round 6 experiment 3: the role-split learner with the actor step's LDS at 68 KB:
# the GPU parity tests it touches, the default bench line, and seeds per GPU with
# the actor step at <= 128 VGPRs (aw4) against the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_learn_gpu.py \
  tests/test_target_pair_gpu.py tests/test_seeds_gpu.py tests/test_fused_env_gpu.py tests/test_train_gpu.py \
  tests/test_smoke_matrix_gpu.py > gpurun_out/r06_exp3_tests.log 2>&1 || { tail -30 gpurun_out/r06_exp3_tests.log; exit 1; }
tail -2 gpurun_out/r06_exp3_tests.log
timeout -k 10 480 python -u bench.py > gpurun_out/r06b_bench.log 2>&1 || { tail -20 gpurun_out/r06b_bench.log; exit 1; }
echo bench done
timeout -k 10 600 bash tools/gpu_seeds_ab.sh r06aw4 "base:-" "aw4:RLMD_LIB_PATH=tools/_abh/librlmd_amd_aw4.so"
