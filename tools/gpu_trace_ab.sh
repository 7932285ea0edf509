#!/bin/bash
# Kernel-level A/B on one box: a rocprofv3 kernel trace of a short bench run per
# (config, environment) pair, e.g.
#   bash tools/gpu_trace_ab.sh tag "c2:- c2:RLMD_QSPLIT=1 c3:- c3:RLMD_FSPLIT=1"
# ('-' = no extra variable).  Per run: gpurun_out/tab_<tag>/<cfg>_<n>/ holds the
# trace and stats; gpurun_out/tab_<tag>/summary.txt the per-kernel averages.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1
OUT=gpurun_out/tab_$TAG
mkdir -p $OUT
n=0
for spec in $2; do
  cfg=${spec%%:*}; ev=${spec#*:}; n=$((n + 1))
  [ "$ev" = "-" ] && ev=""
  D=$OUT/${cfg}_$n
  env $ev timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $D -o t -- python3 bench.py --config $cfg \
    --steps 20 --warmup 5 --no-cpu-baseline --no-companion --k-sweep= --seeds-per-gpu= --seed-procs= --variants= > $D.log 2>&1 \
    || { echo "run failed $spec"; tail -5 $D.log; exit 1; }
  python3 - "$D" "$spec" >> $OUT/summary.txt <<'PY'
import csv, sys, glob
d, spec = sys.argv[1], sys.argv[2]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
print("==", spec)
for r in rows[:8]:
    print(f"  {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:8.2f} us  {r['Name'][:90]}")
PY
  echo "done $spec"
done
cat $OUT/summary.txt
echo ALLDONE
