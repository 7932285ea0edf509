# fused-update iteration: learn / train / fused-env tests, bench lines (fused actor
# on / off), kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_learn_gpu.py tests/test_train_gpu.py tests/test_fused_env_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_learn.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_learn.log; exit 1; }
echo TESTS_OK
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10 > gpurun_out/bench_learn.log 2>&1 || exit 1
RLMD_NO_FUSED_ACTOR=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10 > gpurun_out/bench_noact.log 2>&1 || exit 1
echo BENCHOK
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_learn
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o trace -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > $OUT/trace.log 2>&1
echo PROF_RC=$?
RLMD_NO_FUSED_ACTOR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_noact -o trace -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > $OUT/trace_noact.log 2>&1
echo PROF2_RC=$?
timeout -k 10 200 python tools/ts_probe.py aupd > gpurun_out/ts_aupd.log 2>&1 && timeout -k 10 200 python tools/ts_probe.py upd > gpurun_out/ts_upd.log 2>&1
echo PROBE_RC=$?
