# Run a subset of GPU tests (TESTS) then stop; one process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_new.log 2>&1 && echo ALLOK
