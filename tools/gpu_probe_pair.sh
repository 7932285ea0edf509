set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pp/t -o t -- python3 tools/ts_probe.py upd > gpurun_out/pp/upd.log 2>&1 && timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pp/a -o t -- python3 tools/ts_probe.py aupd > gpurun_out/pp/aupd.log 2>&1
