#!/bin/bash
# round 6, final code: bench lines (C2 + CPU baselines, nccl world 1, C3 / C4 / C5), the
# headline profile round (kernel trace, FETCH / WRITE, MFMA), the learner wave-state pass,
# then the -m gpu suite outside the convergence file and smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r06d}
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step lines timeout -k 10 600 bash tools/gpu_measure.sh lines $TAG
step prof timeout -k 10 520 bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1
step waits timeout -k 10 300 bash tools/probe/pmc_icache.sh $TAG > gpurun_out/${TAG}_icache.log 2>&1
[ -n "$SUITE" ] && step suite timeout -k 10 1000 bash tools/gpu_r06_suite.sh ${TAG}_suite
echo ALLDONE
