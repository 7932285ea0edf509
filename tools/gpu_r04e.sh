#!/bin/bash
# round 4 measurement: default bench line, the C2 profile round, C3 / C5 / C4 traces + MFMA passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/r04_bench.log 2>&1; echo "bench rc=$?"; tail -n 1 gpurun_out/r04_bench.log | cut -c1-300
timeout -k 10 700 bash tools/profile_round.sh r04 > gpurun_out/r04_prof.log 2>&1; echo "prof rc=$?"
MFMA=1 CONFIGS="c3 c5 c4" timeout -k 10 900 bash tools/gpu_prof_configs.sh r04 > gpurun_out/r04_prof_cfg.log 2>&1; echo "cfg rc=$?"
echo ALLDONE
