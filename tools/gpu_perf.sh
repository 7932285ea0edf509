# Perf iteration: learn / train / full-size parity tests, headline bench (no CPU baseline / sweeps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_learn_gpu.py tests/test_train_gpu.py tests/test_fullsize_gpu.py tests/test_multistep_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/perf_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_perf.log 2>&1 || exit $?
RLMD_NO_FUSED_ENV=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_perf_unfused.log 2>&1 || exit $?
echo PERFOK
