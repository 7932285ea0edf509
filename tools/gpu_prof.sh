# round 3: default bench line + profiles (kernel trace, FETCH/WRITE, MFMA passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 700 bash tools/profile_round.sh r03 && echo ALLOK
