#!/bin/bash
# Same-box A/B: bench.py with the in-tree library (A) and tools/_abh/librlmd_amd_$1.so
# (B), alternating, for each config in $CONFIGS (default "c2 c3").  JSON lines to
# gpurun_out/ab_$1.jsonl.  Stops at the first failing run.
# $1 of the form VAR=VALUE: side B is the in-tree library with that environment
# variable set (e.g. RLMD_QSPLIT=1); the tag is VAR_VALUE.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1
ENVB=""
if [[ "$1" == *=* ]]; then ENVB=$1; TAG=${1//=/_}; fi
OUT=gpurun_out/ab_${TAG}.jsonl
for cfg in ${CONFIGS:-c2 c3}; do
  for rep in 1 2 3; do
    for side in A B; do
      EXTRA=""
      if [ $side = B ]; then
        if [ -n "$ENVB" ]; then EXTRA=$ENVB; else export RLMD_LIB_PATH=$PWD/tools/_abh/librlmd_amd_${TAG}.so; fi
      else unset RLMD_LIB_PATH; fi
      env $EXTRA timeout -k 10 150 python -u bench.py --config $cfg --steps 40 --warmup 10 --no-cpu-baseline --no-companion \
        --k-sweep 8 --seeds-per-gpu "" --seed-procs "" > gpurun_out/ab_run.log 2>&1 || { echo "run failed $cfg $rep $side"; tail -5 gpurun_out/ab_run.log; exit 1; }
      python - "$cfg" "$rep" "$side" "$OUT" <<'PY'
import json, sys
cfg, rep, side, out = sys.argv[1:]
d = json.loads([l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][-1])
r = {"cfg": cfg, "rep": int(rep), "side": side, "value": d["value"], "ms_per_step": d["ms_per_step"],
     "learn_ms": d["roofline_mfma"]["avg_phase_ms"], "fused_ms": d["roofline"].get("fused_kernel_ms")}
open(out, "a").write(json.dumps(r) + "\n")
print(r, flush=True)
PY
    done
  done
done
echo ALLDONE
