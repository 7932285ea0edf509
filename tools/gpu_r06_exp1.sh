#!/bin/bash
# round 6 experiment 1: persistent acting grids (A/B kernel traces) and the
# learner's texture-addresser occupancy (one PMC pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 bash tools/gpu_trace_ab.sh r06ap "c2:- c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_ap2.so c2:RLMD_LIB_PATH=tools/_abh/librlmd_amd_ap3.so" > gpurun_out/r06ap.log 2>&1 || { tail -20 gpurun_out/r06ap.log; exit 1; }
tail -40 gpurun_out/r06ap.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_ta
mkdir -p $OUT
BENCH="bench.py --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --steps 15 --warmup 5"
timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY TA_BUFFER_WAVEFRONTS GRBM_GUI_ACTIVE SQ_WAVES --kernel-include-regex "critic_update|actor_update|fwd_rows|qeval_rows|act_env|replay_sample" -f csv -d $OUT/ta -o ta -- python3 $BENCH > $OUT/ta.log 2>&1
echo "pmc rc=$?"
for q in 1 2 0; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion --k-sweep= \
    --seeds-per-gpu= --seed-procs 1,2,3,4 --seed-proc-queues $q > gpurun_out/r06_seedprocs_q$q.log 2>&1 || { echo "seedprocs q=$q failed"; tail -5 gpurun_out/r06_seedprocs_q$q.log; exit 1; }
  echo "seedprocs q=$q done"
done
