#!/bin/bash
# round 4 final lines: default bench (C2 with CPU baselines), C3 and C5.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench timeout -k 10 420 python -u bench.py > gpurun_out/r04f_bench.log 2>&1
for C in c3 c5; do
  step bench_$C timeout -k 10 300 python -u bench.py --config $C > gpurun_out/r04f_bench_$C.log 2>&1
done
echo ALLDONE
