#!/bin/bash
# A round's GPU measurements, in two calls that each fit gpurun's 20-minute limit:
#   bash tools/gpu_measure.sh lines <tag>     default bench (C2 + CPU baselines), the nccl
#                                             process group at world 1, C3 / C4 / C5 lines
#   bash tools/gpu_measure.sh profiles <tag>  C2 profile round (trace, FETCH / WRITE, MFMA),
#                                             C3 / C5 / C4 traces with MFMA passes
# then, here: python tools/pmc_summary.py <tag> c2, and copy the bench lines into profiles/.
# Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
WHAT=$1
TAG=${2:-r04}
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
if [ "$WHAT" = lines ]; then
  step bench timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1
  step nccl1 env RLMD_BENCH_FORCE_DIST=1 timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-companion --k-sweep 8 --seeds-per-gpu "" --seed-procs "" > gpurun_out/${TAG}_bench_nccl1.log 2>&1
  for C in c3 c4 c5; do
    step bench_$C timeout -k 10 300 python -u bench.py --config $C > gpurun_out/${TAG}_bench_$C.log 2>&1
  done
elif [ "$WHAT" = profiles ]; then
  step prof timeout -k 10 500 bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1
  step cfg env MFMA=1 CONFIGS="c3 c5 c4" timeout -k 10 560 bash tools/gpu_prof_configs.sh $TAG \
    > gpurun_out/${TAG}_prof_cfg.log 2>&1
else
  echo "usage: gpu_measure.sh lines|profiles <tag>"; exit 2
fi
echo ALLDONE
