# widened fused steady state: fused env tests (all families, wide shapes, fused == unfused)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fused_env_gpu.py tests/test_train_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_wide.log 2>&1
echo TESTS_RC=$?
