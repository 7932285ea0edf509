#!/bin/bash
# Seeds per GPU (SeedGroup) under launch-geometry / queue variants, one box:
#   bash tools/gpu_seeds_ab.sh <tag> "<name>:<env assignments or ->" ...
# Each variant runs the C2 bench with only the seeds-per-GPU block after a short
# headline (no CPU baselines, no companion, no K sweep); lines land in
# gpurun_out/seeds_<tag>/<name>.json.
set -o pipefail
tag=$1; shift
out=gpurun_out/seeds_$tag
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  [ "$envs" = "-" ] && envs=""
  echo "== $name ($envs)"
  env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-companion \
      --k-sweep '' --seed-procs '' --seeds-per-gpu "${SEEDS:-2,3,4}" > "$out/$name.json" 2> "$out/$name.err" || { echo "FAIL $name"; exit 1; }
  python - "$out/$name.json" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print("  value %.1f M" % (d["value"] / 1e6), {t: round(v["vs_one_seed"], 3) for t, v in d.get("seeds_per_gpu", {}).get("per_gpu", d.get("seeds_per_gpu", {})).items() if isinstance(v, dict) and "vs_one_seed" in v})
EOF
done
