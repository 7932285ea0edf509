# learn-path GPU check: learn / train / fused-env tests, then a short bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_learn_gpu.py tests/test_train_gpu.py tests/test_fused_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_learn.log 2>&1
rc=$?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10 > gpurun_out/bench_learn.log 2>&1 && echo BENCHOK
echo TESTS_RC=$rc
