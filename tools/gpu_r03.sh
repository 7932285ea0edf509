# Round-3 GPU check: full -m gpu suite (per-test lines), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 && echo ALLOK
