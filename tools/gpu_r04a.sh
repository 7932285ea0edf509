#!/bin/bash
# round 4, first GPU pass: the learn tests (incl. the fused-actor snapshot test),
# then convergence runs on the metric's workloads and the Dice_SH_INSURED variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_learn_gpu.py \
  > gpurun_out/r04a_learn.log 2>&1 || { echo "learn tests failed"; tail -30 gpurun_out/r04a_learn.log; exit 1; }
tail -3 gpurun_out/r04a_learn.log
timeout -k 10 500 python -u tools/converge_batch.py gpurun_out/r04a_converge.jsonl \
  "env=gbm,algo=SAC,k=8,seed=0" "env=gbm,algo=SAC,k=8,seed=1" "env=gbm,algo=SAC,k=0,seed=0" \
  "env=dice_sh_a,algo=TD3,k=8,seed=0" "env=dice_sh_a,algo=TD3,loss=HUB,k=8,seed=0" "env=dice_sh_a,algo=TD3,k=0,seed=0" \
  "env=dice_sh,algo=SAC,k=8,seed=0,replay=16777216" "env=dice_sh,algo=SAC,k=32,seed=0" \
  "env=dice_sh,algo=SAC,k=8,seed=0,lanes=8192" "env=dice_sh,algo=SAC,k=8,seed=0,lanes=8192,replay=131072" \
  2>&1 | tee gpurun_out/r04a_converge.log
