#!/bin/bash
# round 6: the -m gpu suite outside the convergence file on the current code, then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r06_suite}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  --ignore=tests/test_converge_gpu.py > gpurun_out/${TAG}.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/${TAG}.log | tail -3
echo "suite rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_smoke.log
echo "smoke rc=$rc"
exit $rc
