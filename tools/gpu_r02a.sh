# Round-2 first GPU pass: gpu tests, default bench, short convergence curves.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
OUT=gpurun_out/converge_a.jsonl
rm -f $OUT
for env in coin dice dice_sh; do
  timeout -k 10 200 python -u tools/converge.py --env $env --lanes 65536 --k 8 --precision bf16 \
      --steps 12000 --eval-every 500 --out $OUT > gpurun_out/converge_a_$env.log 2>&1 || exit $?
done
echo ALLOK
