# act_env occupancy iteration: env / train / fused-env tests, act_env stamps (C3, C2), C2 / C3 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_train_gpu.py tests/test_fused_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_env.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_env.log; exit 1; }
echo TESTS_OK
timeout -k 10 200 python tools/ts_probe.py actenv dice_sh > gpurun_out/ts_actenv_c3.log 2>&1 && \
timeout -k 10 200 python tools/ts_probe.py actenv gbm > gpurun_out/ts_actenv_c2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10 > gpurun_out/bench_learn.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_c3.log 2>&1 && echo BENCHOK
