#!/bin/bash
# round 4: the C3 / C4 / C5 bench lines, then their kernel traces + MFMA passes.
# Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for C in c3 c4 c5; do
  step bench_$C timeout -k 10 300 python -u bench.py --config $C > gpurun_out/r04_bench_$C.log 2>&1
  tail -n 1 gpurun_out/r04_bench_$C.log | cut -c1-200
done
step cfg env MFMA=1 CONFIGS="c3 c5 c4" timeout -k 10 600 bash tools/gpu_prof_configs.sh r04 > gpurun_out/r04_prof_cfg.log 2>&1
echo ALLDONE
