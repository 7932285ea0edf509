#!/bin/bash
# round 6 profiles: the headline profile round (kernel trace, FETCH / WRITE and MFMA
# passes), the learner's wave states and instruction cache, the texture-addresser
# pass on the role-split learner, and the per-role windows of the update kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step prof timeout -k 10 520 bash tools/profile_round.sh r06 > gpurun_out/r06_prof.log 2>&1
step icache timeout -k 10 300 bash tools/probe/pmc_icache.sh r06 > gpurun_out/r06_icache.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_ta_after
mkdir -p $OUT
step ta timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY TA_BUFFER_WAVEFRONTS GRBM_GUI_ACTIVE SQ_WAVES --kernel-include-regex "critic_update|actor_update|fwd_rows|qeval_rows|act_env|replay_sample" -f csv -d $OUT/ta -o ta -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --steps 15 --warmup 5
step ts_upd env RLMD_TS_TAG=win timeout -k 10 200 python -u tools/ts_probe.py upd > gpurun_out/r06_ts_win_upd.log 2>&1
step ts_aupd env RLMD_TS_TAG=win timeout -k 10 200 python -u tools/ts_probe.py aupd > gpurun_out/r06_ts_win_aupd.log 2>&1
echo ALLDONE
