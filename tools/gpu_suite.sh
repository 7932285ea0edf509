#!/bin/bash
# The -m gpu suite (one process, per-test timeout), then any extra step given as
# arguments (run only when the suite passed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r04}
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -n 4 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
if [ $# -gt 0 ]; then "$@"; fi
