#!/bin/bash
# Instruction-fetch counters of the learner kernels (C2 headline command), two
# separate passes (SQ wave counters; SQC instruction-cache counters):
#   bash tools/probe/pmc_icache.sh <tag>   ->  gpurun_out/pmc_ic_<tag>/
set -e
TAG=${1:-ic}
OUT=gpurun_out/pmc_ic_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH="bench.py --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --steps 10 --warmup 3"
K="fwd_rows|qeval_rows|critic_update_kernel|actor_update_kernel|act_env_kernel"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_WAVES \
  --kernel-include-regex "$K" -f csv -d $OUT/sq -o sq -- python3 $BENCH > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS \
  --kernel-include-regex "$K" -f csv -d $OUT/sqc -o sqc -- python3 $BENCH > $OUT/sqc.log 2>&1
echo done
