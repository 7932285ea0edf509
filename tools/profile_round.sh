#!/bin/bash
# One round's profiles on the GPU box (run from the repo root via gpurun):
#   1. kernel trace + stats of the default bench workload (timed region only)
#   2. separate PMC passes for the env kernel: FETCH_SIZE, WRITE_SIZE
#   3. one MFMA pass over the acting / learn kernels: SQ_VALU_MFMA_BUSY_CYCLES,
#      SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE
# Outputs under gpurun_out/prof_<tag>/; tools/pmc_summary.py turns them into
# the committed profiles/<tag>_*.  Every GPU step has its own time limit and the
# chain stops at the first failure.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH="bench.py --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --steps 25 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o trace -- python3 $BENCH > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "act_env_kernel|fused_act_kernel|env_train_kernel" -f csv -d $OUT/fetch -o fetch -- python3 $BENCH > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "act_env_kernel|fused_act_kernel|env_train_kernel" -f csv -d $OUT/write -o write -- python3 $BENCH > $OUT/write.log 2>&1
LEARN="act_env_kernel|fused_act_kernel|fwd_rows|cbwd_rows|qeval_rows|abwd_rows|gemm_kernel|adam_kernel|replay_sample|critic_update_kernel|actor_update_kernel"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$LEARN" -f csv -d $OUT/mfma -o mfma -- python3 $BENCH > $OUT/mfma.log 2>&1
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
echo done
