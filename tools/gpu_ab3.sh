# A/B: tools/_abh (HEAD build) vs working tree, same box, plus the working tree
# with kernel arguments forced into device memory and into host memory
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
B="--no-cpu-baseline --no-companion --k-sweep= --steps 40 --warmup 10"
run() { timeout -k 10 200 "$@"; }
(cd tools/_abh && run python -u bench.py $B) > gpurun_out/ab/head.log 2>&1 || exit 1
run python -u bench.py $B > gpurun_out/ab/wt.log 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 run python -u bench.py $B > gpurun_out/ab/wt_dev.log 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=0 run python -u bench.py $B > gpurun_out/ab/wt_host.log 2>&1 || exit 1
(cd tools/_abh && run python -u bench.py $B) > gpurun_out/ab/head2.log 2>&1 || exit 1
run python -u bench.py $B > gpurun_out/ab/wt2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ab/trace_wt -o t -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > gpurun_out/ab/trace_wt.log 2>&1 || exit 1
for f in head wt wt_dev wt_host head2 wt2; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab/$f.log') if l.startswith('{')][-1]); print('$f', round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1))"; done
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAILED; tail -20 gpurun_out/ab/tests.log; exit 1; }
fi
echo done
