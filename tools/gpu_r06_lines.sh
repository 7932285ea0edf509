#!/bin/bash
# round 6: deferred second fc2 stream (A/B trace), then the round's bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 bash tools/gpu_trace_ab.sh r06d2 "c2:- c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_d2.so c3:- c3:RLMD_LIB_PATH=tools/_abh/librlmd_amd_d2.so" > gpurun_out/r06d2.log 2>&1 || { tail -20 gpurun_out/r06d2.log; exit 1; }
tail -36 gpurun_out/r06d2.log
timeout -k 10 1000 bash tools/gpu_measure.sh lines r06
