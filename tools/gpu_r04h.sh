#!/bin/bash
# round 4 measurement: default bench line, the nccl process group at world 1,
# then the C2 profile round.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step bench timeout -k 10 420 python -u bench.py > gpurun_out/r04_bench.log 2>&1
tail -n 1 gpurun_out/r04_bench.log | cut -c1-300
step nccl1 env RLMD_BENCH_FORCE_DIST=1 timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 \
  --no-cpu-baseline --no-companion --k-sweep 8 --seeds-per-gpu "" > gpurun_out/r04_bench_nccl1.log 2>&1
step prof timeout -k 10 500 bash tools/profile_round.sh r04 > gpurun_out/r04_prof.log 2>&1
echo ALLDONE
