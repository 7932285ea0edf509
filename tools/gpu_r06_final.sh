#!/bin/bash
# round 6, final code: bench lines (C2 + CPU baselines, nccl world 1, C3 / C4 / C5), the
# headline profile round (kernel trace, FETCH / WRITE, MFMA) and the learner wave-state pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r06d}
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step lines timeout -k 10 600 bash tools/gpu_measure.sh lines $TAG
step prof timeout -k 10 520 bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1
step waits timeout -k 10 300 bash tools/probe/pmc_icache.sh $TAG > gpurun_out/${TAG}_icache.log 2>&1
echo ALLDONE
