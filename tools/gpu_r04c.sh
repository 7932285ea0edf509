#!/bin/bash
# round 4: bf16 learner parity, seeds per GPU, the per-handle switch tests; then
# warm-up-length experiments on the metric's workloads and a quick bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_learn_gpu.py tests/test_seeds_gpu.py tests/test_fused_env_gpu.py \
  tests/test_eval_gpu.py tests/test_fullsize_gpu.py -q -s --timeout 180 --timeout-method thread \
  > gpurun_out/r04c_tests.log 2>&1; echo "tests rc=$?"; grep -E "step 3 params|passed|failed|Error" gpurun_out/r04c_tests.log | tail -40
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 \
  > gpurun_out/r04c_bench.log 2>&1; echo "bench rc=$?"; tail -n 1 gpurun_out/r04c_bench.log | cut -c1-400
timeout -k 10 600 python -u tools/converge_batch.py gpurun_out/r04c_converge.jsonl \
  "env=dice_sh_a,algo=TD3,k=8,seed=0,warmup=100,smoothing=200" "env=dice_sh_a,algo=TD3,k=8,seed=1,warmup=100,smoothing=200" \
  "env=dice_sh_a,algo=TD3,k=8,seed=0,warmup=25,smoothing=50" "env=dice_sh_a,algo=TD3,k=1,seed=0" \
  "env=dice_sh,algo=SAC,k=8,seed=0,warmup=100,smoothing=200" "env=dice_sh,algo=SAC,k=8,seed=1,warmup=100,smoothing=200" \
  "env=gbm,algo=SAC,k=8,seed=0,warmup=100,smoothing=200" "env=gbm,algo=SAC,k=8,seed=1,warmup=100,smoothing=200" \
  "env=gbm,algo=SAC,k=8,seed=2" "env=gbm,algo=SAC,k=8,seed=3" "env=gbm,algo=SAC,k=8,seed=0,steps=40000" \
  2>&1 | tee gpurun_out/r04c_converge.log
