# round 3: C3 / C4 / C5 bench lines, a C3 kernel trace and the Dice_SH env stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_$c.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_c3/trace -o trace -- python3 bench.py --config c3 --no-cpu-baseline --no-companion --k-sweep= --steps 15 --warmup 5 > gpurun_out/prof_c3.log 2>&1 || exit $?
timeout -k 10 200 python tools/ts_probe.py env dice_sh > gpurun_out/ts_env_dicesh.log 2>&1
echo ALLOK
