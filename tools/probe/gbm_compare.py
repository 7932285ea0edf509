"""GBM_InvA (key 14, SAC / MSE): the reference's training and evaluation
statistics next to the build's reference-API driver, per 5,000-step window.

    python tools/probe/gbm_compare.py 'tests/golden/converge_ref_14_s?.npz' profiles/r05_gbm_single_stream.jsonl

REF_NPZ_GLOB: tests/golden/run_reference_loop.py --out files (they carry the
per-episode trial logs, rl_multiplicative.py:419-429); BUILD_JSONL:
tools/probe/gbm_single.py records.  Prints, per seed and window, the episodes
that ended, their mean length, the last episode's logtemp (the reference's
column aliases the live log_alpha tensor on CPU, so every row holds the final
value) and the evaluation leverage; then the last-third statistics of both sides and the Mann-Whitney p.
"""
import glob
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gbm_single import trial_summary  # noqa: E402


def third(v):
    v = np.asarray(v)
    return float(v[len(v) - len(v) // 3:].mean())


def main():
    from scipy.stats import mannwhitneyu

    ref, build = [], []
    for p in sorted(glob.glob(sys.argv[1])):
        with np.load(p, allow_pickle=False) as z:
            lev = z["lev"].mean(1)
            g = 100.0 * (z["reward"] - 1.0).mean(1)
            # the five fixture seeds of the convergence test carry no trial logs
            tr = trial_summary(z["trial_steps"], z["trial_logtemp"], z["trial_lev"]) if "trial_steps" in z else []
            ref.append((int(z["seed"]), third(g), third(lev), tr, lev))
    for line in open(sys.argv[2]):
        d = json.loads(line)
        if d["workload"] == "gbm_single_stream":
            build.append((d["seed"], d["growth_pct"], d["lev"], d["trial"], np.array(d["lev_curve"])))
    for name, rows in (("reference", ref), ("build", build)):
        for seed, g, lv, tr, curve in rows:
            print(f"{name} seed {seed}: last-third growth {g:.2f} %/step, lev {lv:.3f}")
            if tr:
                print("   window  episodes  mean_len  logtemp  eval_lev")
            for w, ne, ml, lt, _ in tr:
                k = min(w // 1000, len(curve)) - 1
                print(f"   {w:6d}  {ne:8d}  {ml:8.0f}  {lt if lt is None else f'{lt:7.3f}'}  {curve[k]:8.2f}")
    for i, what in ((1, "growth"), (2, "lev")):
        a, b = [r[i] for r in ref], [r[i] for r in build]
        p = mannwhitneyu(a, b, alternative="two-sided", method="exact").pvalue
        print(f"{what}: reference {np.round(sorted(a), 2)}  build {np.round(sorted(b), 2)}  Mann-Whitney p {p:.3f}")


if __name__ == "__main__":
    main()
