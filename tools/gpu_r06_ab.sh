#!/bin/bash
# round 6 A/B: the timing probe of fwd_rows (RLMD_TIMING build), then same-box kernel traces
#   bash tools/gpu_r06_ab.sh <tag> "<gpu_trace_ab specs>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
timeout -k 10 200 python -u tools/ts_probe.py run > gpurun_out/${TAG}_ts.log 2>&1 || { tail -5 gpurun_out/${TAG}_ts.log; exit 1; }
grep -A22 "target job 0" gpurun_out/${TAG}_ts.log
grep -A6 "job windows" gpurun_out/${TAG}_ts.log
timeout -k 10 900 bash tools/gpu_trace_ab.sh $TAG "$2" > gpurun_out/${TAG}_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
grep -E "==|fwd_rows|qeval|critic_update|actor_update" gpurun_out/tab_$TAG/summary.txt
