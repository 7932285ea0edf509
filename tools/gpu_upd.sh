# fused-update iteration: learn / train tests, the critic-update stamps, a short bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_learn_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_learn.log 2>&1
echo TESTS_RC=$?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10 > gpurun_out/bench_learn.log 2>&1 && echo BENCHOK
timeout -k 10 400 python tools/ts_probe.py build > gpurun_out/tsb.log 2>&1 && timeout -k 10 300 python tools/ts_probe.py upd > gpurun_out/ts_upd.log 2>&1
cat gpurun_out/ts_upd.log
