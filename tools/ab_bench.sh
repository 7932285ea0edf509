# A/B: committed build (tools/_abh) vs working tree, same box, C2 bench lines + traces
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
B="--no-cpu-baseline --no-companion --k-sweep= --steps 30 --warmup 10"
(cd tools/_abh && timeout -k 10 300 python -u bench.py $B) > gpurun_out/ab/head.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $B > gpurun_out/ab/wt.log 2>&1 || exit 1
RLMD_NO_FUSED_ACTOR=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/ab/wt_noact.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT/tools/_abh"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/ab/trace_head" -o t -- python3 bench.py --no-cpu-baseline --no-companion --k-sweep= --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/ab/trace_head.log" 2>&1
echo done
