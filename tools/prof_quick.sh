# Kernel-trace stats of a short default bench run -> gpurun_out/pq/ (+ bench line)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/pq
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pq -o p -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/pq.log 2>&1 && \
grep '^{' gpurun_out/pq.log | cut -c1-300 && python3 tools/prof_summary.py gpurun_out/pq/p_kernel_stats.csv 14
