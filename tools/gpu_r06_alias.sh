#!/bin/bash
# round 6: the stored-state aliasing on the GPU — the parity tests it touches, then
# GBM_InvA SAC convergence (C2's env) with the reference's stored states.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_fused_env_gpu.py tests/test_train_gpu.py tests/test_c1_driver_gpu.py tests/test_market_driver_gpu.py \
  tests/test_fullsize_gpu.py > gpurun_out/r06_alias_tests.log 2>&1 || { tail -30 gpurun_out/r06_alias_tests.log; exit 1; }
tail -3 gpurun_out/r06_alias_tests.log
specs=""
for s in 0 1 2 3 4 5 6 7 8 9; do specs="$specs env=gbm,algo=SAC,k=8,seed=$s"; done
timeout -k 10 500 python -u tools/converge_batch.py gpurun_out/r06_gbm_alias.jsonl $specs
