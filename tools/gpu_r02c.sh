# Round-2 closing GPU pass: the whole -m gpu suite, the default bench line, the round profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
bash tools/profile_round.sh r02 || exit $?
echo ALLOK
