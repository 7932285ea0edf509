# leverage-sweep tests + full-size timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_lev_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/t_lev.log 2>&1 || exit $?
for k in dice gbm dice_sh; do
  timeout -k 10 200 python -u tools/bench_lev.py --kind $k --investors 1000000 --horizon 300 --reps 2 > gpurun_out/lev_$k.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_lev
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_lev -o lev -- python3 tools/bench_lev.py --kind dice --investors 1000000 --horizon 300 --reps 2 --no-cpu-baseline > gpurun_out/prof_lev/log.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_lev.py --kind coin_flip --investors 1000000 --horizon 3000 > gpurun_out/lev_coinflip.log 2>&1 || exit $?
echo ALLOK
