#!/bin/bash
# Round-5 probe call: ts_probe stamps of the SAC update launches (phase and window
# builds, tools/ts_probe.py), more C4 ring-depth seeds, the headline profile round.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r05a}
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for m in upd aupd run; do
  step ts_ph_$m env RLMD_TS_TAG=_ph timeout -k 10 120 python -u tools/ts_probe.py $m > gpurun_out/${TAG}_ts_ph_$m.log 2>&1
done
for m in upd aupd; do
  step ts_win_$m env RLMD_TS_TAG=_win timeout -k 10 120 python -u tools/ts_probe.py $m > gpurun_out/${TAG}_ts_win_$m.log 2>&1
done
step ring timeout -k 10 300 python -u tools/probe/market_sweep.py gpurun_out/r05_market_sweepD.jsonl "8192:8:67108864" 3,4,5 > gpurun_out/r05_sweepD1.log 2>&1
step ring2 timeout -k 10 300 python -u tools/probe/market_sweep.py gpurun_out/r05_market_sweepD.jsonl "8192:8:16777216" 0,1,2,3,4,5 > gpurun_out/r05_sweepD2.log 2>&1
step prof timeout -k 10 500 bash tools/profile_round.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1
echo ALLDONE
