# kernel trace of a short C2 bench (learn-path work): gpurun_out/prof_learn/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_learn
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o trace -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > $OUT/trace.log 2>&1
echo done
