#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of the bench's other configs,
# C3 / C5 (TD3) and C4 (market), one pass each with its own time limit.
set -e
TAG=${1:-r04}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in ${CONFIGS:-c3 c5 c4}; do
  BENCH="bench.py --config $C --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --variants= --steps 25 --warmup 5"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_$C -o trace -- python3 $BENCH > $OUT/trace_$C.log 2>&1
  tail -n 1 $OUT/trace_$C.log | cut -c1-300
  if [ -n "${MFMA:-}" ]; then  # one MFMA-busy pass over the acting / learn kernels (its own run)
    LEARN="act_env_kernel|fused_act_kernel|fwd_rows|qeval_rows|replay_sample|critic_update_kernel|actor_update_kernel"
    timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$LEARN" \
      -f csv -d $OUT/mfma_$C -o mfma -- python3 $BENCH > $OUT/mfma_$C.log 2>&1
  fi
done
echo done
