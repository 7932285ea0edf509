#!/bin/bash
# round 4 profiles: the C2 profile round (trace + FETCH / WRITE + MFMA passes),
# then C3 / C5 / C4 traces with MFMA passes.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step prof timeout -k 10 600 bash tools/profile_round.sh r04 > gpurun_out/r04_prof.log 2>&1
step cfg env MFMA=1 CONFIGS="c3 c5 c4" timeout -k 10 560 bash tools/gpu_prof_configs.sh r04 \
  > gpurun_out/r04_prof_cfg.log 2>&1
echo ALLDONE
