# A/B: tools/_abh (HEAD build) vs working tree, same box: C2 bench lines + kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
B="--no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10"
(cd tools/_abh && timeout -k 10 300 python -u bench.py $B) > gpurun_out/ab/head.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $B > gpurun_out/ab/wt.log 2>&1 || exit 1
(cd tools/_abh && timeout -k 10 300 python -u bench.py $B) > gpurun_out/ab/head2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $B > gpurun_out/ab/wt2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab/trace_wt -o t -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > gpurun_out/ab/trace_wt.log 2>&1 || exit 1
cd tools/_abh && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/ab/trace_head" -o t -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/ab/trace_head.log" 2>&1
echo done
cd "$GRAFT_REPO_ROOT"
[ -n "$AB_TESTS" ] && { timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAILED; tail -20 gpurun_out/ab/tests.log; exit 1; }; }
