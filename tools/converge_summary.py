"""The convergence table of DESIGN.md §5a from a round's committed per-seed
records (tests/test_converge_gpu.py with RLMD_CONVERGE_LOG set):

    python tools/converge_summary.py profiles/r05_converge.jsonl

Per workload: the reference seeds' range (tests/golden/converge_ref_*.npz), the
build seeds' median and range, the Mann-Whitney p-values the test recorded, and
the no-learning (K = 0) control's."""
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

LABEL = {"coin": "Coin_InvA (8, SAC / MSE) — uninformative", "dice": "Dice_InvA (11, SAC / MSE) — uninformative",
         "gbm": "**GBM_InvA (14, SAC / MSE; C2's env)** — one-sided",
         "dice_sh": "Dice_SH_INSURED (17, SAC / MSE)", "dice_sh_a_mse": "**Dice_SH_InvA (18, TD3 / MSE; C3's env)**",
         "dice_sh_a_hub": "Dice_SH_InvA (18, TD3 / HUB)",
         "gbm_td3_n5": "**GBM_InvA (14, TD3 / MSE, n = 5; C5)** — bimodal",
         "market": "**SNP_InvA market (21, SAC / MSE; C4)**, 8,192 lanes on one slice stream"}


def ref_stats(stem, market):
    out = []
    for s in range(5):
        with np.load(os.path.join(ROOT, "tests", "golden", f"{stem}_s{s}.npz"), allow_pickle=False) as d:
            n = d["reward"].shape[0]
            sl = slice(n - n // 3, n)
            lev = d["risk"][sl][..., 4] if market else d["lev"][sl]
            out.append((100.0 * float((d["reward"][sl] - 1.0).mean()), float(lev.mean())))
    return out


def fmt(vals):
    v = np.asarray(vals)
    return f"{np.median(v):.3g} ({v.min():.3g} .. {v.max():.3g})"


def main(path):
    from test_converge_gpu import WORKLOADS

    recs = [json.loads(line) for line in open(path)]
    seeds = defaultdict(list)
    tests = {}
    for r in recs:
        w = r["workload"]
        if w.endswith("_test"):
            tests[(w[:-5], r.get("precision"))] = r
        elif "seed" in r and r.get("lanes") is not None and "slice_groups" in r or (
                "seed" in r and r.get("precision") and w != "market"):
            seeds[(w, r["k"], r.get("precision"))].append((r["growth_pct"], r["lev"]))
    print("| Workload (key, algo / loss) | reference growth %/step (5 seeds) | reference lev | build growth, median (range) "
          "| build lev | Mann-Whitney p (growth / lev) | K = 0 control |")
    print("|---|---|---|---|---|---|---|")
    for (w, k, prec), v in sorted(seeds.items(), key=lambda x: (list(LABEL).index(x[0][0]), x[0][2] or "")):
        if k == 0:
            continue
        ref = ref_stats(WORKLOADS[w][3], w == "market")
        t = tests.get((w, prec), {})
        p = f"{t['p_growth']:.3f} / {t['p_lev']:.3f}" if "p_growth" in t else (
            f"upper mode {tests[(w, None)]['upper_mode']} of 5 (reference 3)"
            if (w, None) in tests else "one-sided band")
        k0 = seeds.get((w, 0, "bf16"))
        kt = tests.get((w + "_k0", None))
        if kt:
            k0s = f"p {kt['p_growth']:.3f} / {kt['p_lev']:.3f}" + (" (not asserted)" if w in ("coin", "dice") else "")
        elif k0:
            k0s = f"growth {fmt([g for g, _ in k0])}, lev {fmt([x for _, x in k0])}"
        else:
            k0s = "—"
        print(f"| {LABEL.get(w, w)}{'' if prec == 'bf16' else ' ' + prec} | {min(g for g, _ in ref):.3g} .. "
              f"{max(g for g, _ in ref):.3g} | {min(x for _, x in ref):.3g} .. {max(x for _, x in ref):.3g} | "
              f"{fmt([g for g, _ in v])} | {fmt([x for _, x in v])} | {p} | {k0s} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r05_converge.jsonl"))
