# the other BASELINE configs on one GPU (bench lines for the record)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-companion --k-sweep= > gpurun_out/bench_$c.log 2>&1 || exit $?
done
echo ALLOK
