#!/bin/bash
# round 6: the convergence test file on the GPU, per-seed records to profiles' jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r06}
export RLMD_CONVERGE_LOG=gpurun_out/${TAG}_converge.jsonl
timeout -k 10 560 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_converge_gpu.py \
  -k "consistent_with_reference and not single or c5_upper" > gpurun_out/${TAG}_converge_tests_a.log 2>&1
echo "part a rc=$?"; grep -E "PASSED|FAILED|XFAIL|XPASS|ERROR|passed|failed" gpurun_out/${TAG}_converge_tests_a.log | tail -15
timeout -k 10 560 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu tests/test_converge_gpu.py \
  -k "not (consistent_with_reference and not single) and not c5_upper" > gpurun_out/${TAG}_converge_tests_b.log 2>&1
echo "part b rc=$?"; grep -E "PASSED|FAILED|XFAIL|XPASS|ERROR|passed|failed" gpurun_out/${TAG}_converge_tests_b.log | tail -20
