# round 3 close-out on the final code: full -m gpu suite, the default bench line,
# C3 / C4 / C5 lines, and the profile round (kernel trace, FETCH / WRITE, MFMA)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit 1
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_$c.log 2>&1 || exit 1
done
timeout -k 10 700 bash tools/profile_round.sh r03 || exit 1
echo ALLOK
