#!/bin/bash
# TD3 target pairing: its tests (pairing on), then same-box A/B of C3 / C5 (A: RLMD_TARGET_PAIR=1, B: off).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RLMD_TARGET_PAIR=1 timeout -k 10 400 python -u -m pytest tests/test_target_pair_gpu.py tests/test_learn_gpu.py tests/test_fullsize_gpu.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/pair_tests.log 2>&1 || { tail -30 gpurun_out/pair_tests.log; exit 1; }
tail -2 gpurun_out/pair_tests.log
OUT=gpurun_out/ab_pair.jsonl
for cfg in c3 c5; do
  for rep in 1 2 3; do
    for side in A B; do
      if [ $side = A ]; then export RLMD_TARGET_PAIR=1; else unset RLMD_TARGET_PAIR; fi
      timeout -k 10 150 python -u bench.py --config $cfg --steps 40 --warmup 10 --no-cpu-baseline --no-companion \
        --k-sweep 8 --seeds-per-gpu "" > gpurun_out/ab_run.log 2>&1 || { echo "run failed $cfg $rep $side"; tail -5 gpurun_out/ab_run.log; exit 1; }
      python - "$cfg" "$rep" "$side" "$OUT" <<'PY'
import json, sys
cfg, rep, side, out = sys.argv[1:]
d = json.loads([l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][-1])
r = {"cfg": cfg, "rep": int(rep), "side": side, "value": d["value"], "ms_per_step": d["ms_per_step"],
     "learn_ms": d["roofline_mfma"]["avg_phase_ms"]}
open(out, "a").write(json.dumps(r) + "\n")
print(r, flush=True)
PY
    done
  done
done
echo ALLDONE
