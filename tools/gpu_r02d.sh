# eval tests + one-launch market eval profile + short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_eval
timeout -k 10 300 python -u -m pytest tests/test_eval_gpu.py tests/test_train_gpu.py -q -s --timeout 300 --timeout-method thread > gpurun_out/t_eval.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_lb.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_eval -o ev -- python3 -m pytest tests/test_eval_gpu.py -q -k one_launch_time > gpurun_out/prof_eval/log.txt 2>&1 || exit $?
echo ALLOK
