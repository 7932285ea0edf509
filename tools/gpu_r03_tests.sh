# round 3: the whole -m gpu suite (one process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo TESTS_RC=$?
