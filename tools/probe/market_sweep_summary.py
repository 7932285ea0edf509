"""Summarise profiles/r05_market_sweep.jsonl (tools/probe/market_sweep.py): per
(lanes, K, ring, slice groups, precision) the seeds' last-third leverage and
growth, and a two-sided Mann-Whitney test of each group against the reference's
five market_env seeds (tests/golden/converge_ref_21_e20_s*.npz)."""
import json
import os
import sys
from collections import defaultdict

import numpy as np
from scipy.stats import mannwhitneyu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ref_seeds():
    out = []
    for s in range(5):
        with np.load(os.path.join(ROOT, "tests", "golden", f"converge_ref_21_e20_s{s}.npz"), allow_pickle=False) as d:
            n = d["reward"].shape[0]
            sl = slice(n - n // 3, n)
            out.append((100.0 * float((d["reward"][sl] - 1.0).mean()), float(d["risk"][sl][..., 4].mean())))
    return out


def main(path):
    ref = ref_seeds()
    rl, rg = [y for _, y in ref], [x for x, _ in ref]
    groups = defaultdict(list)
    for line in open(path):
        r = json.loads(line)
        key = (r["lanes"], r["k"], r["replay"], r.get("slice_groups", 0), r.get("precision", "bf16"))
        groups[key].append((r["seed"], r["growth_pct"], r["lev"], r["env_steps"], r["updates"]))
    print(f"reference (5 seeds): lev {np.round(sorted(rl), 3).tolist()}  growth {np.round(sorted(rg), 2).tolist()}")
    print("| lanes | K | ring | slices | prec | seeds | ring share of the run | lev (sorted) | growth (sorted) | MW p lev | MW p growth |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for key in sorted(groups):
        v = groups[key]
        lev = sorted(x[2] for x in v)
        gr = sorted(x[1] for x in v)
        share = min(1.0, key[2] / max(v[0][3], 1))
        pl = mannwhitneyu(lev, rl, alternative="two-sided", method="exact").pvalue
        pg = mannwhitneyu(gr, rg, alternative="two-sided", method="exact").pvalue
        print(f"| {key[0]} | {key[1]} | {key[2]} | {key[3] or 'own'} | {key[4]} | {len(v)} | {share:.3g} | "
              f"{', '.join(f'{x:.2f}' for x in lev)} | {', '.join(f'{x:.2f}' for x in gr)} | {pl:.3f} | {pg:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r05_market_sweep.jsonl"))
