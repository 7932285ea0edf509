"""Converged growth rates of the headline loop (north_star parity).

VecTrainer (65,536 lanes, SAC 256/256, K = 8 updates of B = 512 per vector
step) trains on the three gambles with analytic growth-optimal (Kelly)
leverages (lev/lev_exp.py:495-496; tools/converge.py):
  Coin_InvA        Kelly lev 0.25    growth 0.623 %/step
  Dice_InvA        Kelly lev 0.3785  growth 0.644 %/step
  Dice_SH_INSURED  Kelly lev 0.9076  growth 2.166 %/step
12,000 vector steps (96,000 updates) per run.  Every 250 vector steps the
deterministic action at the reset state (the learned constant leverage: the
envs' observations are divided by 1e18) is evaluated on 4,096 device episodes
of 100 steps.  Statistic: the mean over the last third of the evaluations.

Reference band (tests/golden/converge_ref_{8,11,17}_s{0..4}.npz: the
reference's own rl_multiplicative loop, SAC/MSE, 5e4 steps, 5 seeds, on CPU,
made by tests/golden/run_reference_loop.py).  The last-third statistics of the
five reference seeds:
  Coin_InvA        lev 0.013 .. 0.105   growth -0.178 .. 0.315 %/step
  Dice_InvA        lev -0.040 .. 0.123  growth -0.136 .. 0.303 %/step
  Dice_SH_INSURED  lev 0.863 .. 0.929   growth -4.750 .. 2.037 %/step
(the reference reaches Kelly leverage on Dice_SH_INSURED and stays near zero
leverage on Coin / Dice within its budget).

Assertion, per build seed (3 seeds x {bf16, fp32} x 3 envs): the seed's
last-third leverage and growth lie inside the reference seeds' [min, max],
widened by LEV_MARGIN = 0.05 and GROWTH_MARGIN = 0.5 %/step.  No fraction of
Kelly enters the bar.
"""
import math
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
KEYS = {"coin": 8, "dice": 11, "dice_sh": 17}
REF_SEEDS = (0, 1, 2, 3, 4)
BUILD_SEEDS = (0, 1, 2)
LEV_MARGIN = 0.05
GROWTH_MARGIN = 0.5  # %/step
STEPS, EVAL_EVERY = 12000, 250


def _final_third(recs, key):
    v = np.array([r[key] for r in recs])
    return float(v[-max(len(v) // 3, 1):].mean())


def ref_stats(golden, env):
    """Last-third mean (eval growth %/step, leverage) of each reference seed."""
    out = []
    for s in REF_SEEDS:
        d = golden(f"converge_ref_{KEYS[env]}_s{s}.npz")
        n = d["reward"].shape[0]
        sl = slice(n - n // 3, n)
        out.append((100.0 * float((d["reward"][sl] - 1.0).mean()), float(d["lev"][sl].mean())))
    return out


def ref_band(golden, env):
    st = ref_stats(golden, env)
    g = [x for x, _ in st]
    lv = [x for _, x in st]
    return (min(g) - GROWTH_MARGIN, max(g) + GROWTH_MARGIN), (min(lv) - LEV_MARGIN, max(lv) + LEV_MARGIN)


def test_kelly_optima():
    import converge

    for env, (l, g) in {"coin": (0.25, 0.6231), "dice": (0.3785, 0.6441), "dice_sh": (0.9076, 2.166)}.items():
        kl, kg = converge.kelly(env)
        assert kl == pytest.approx(l, abs=2e-4) and kg == pytest.approx(g, abs=2e-3)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("env", ["dice_sh", "coin", "dice"])
def test_build_seeds_land_in_reference_band(golden, dev, env, precision):
    import converge

    (g_lo, g_hi), (l_lo, l_hi) = ref_band(golden, env)
    got = []
    for seed in BUILD_SEEDS:
        recs = converge.run(env, 65536, 8, STEPS, precision=precision, eval_every=EVAL_EVERY, seed=seed,
                            log=lambda s: None)
        assert all(math.isfinite(r["eval_growth_pct"]) and r["nan_flag"] == 0 for r in recs)
        got.append((seed, _final_third(recs, "eval_growth_pct"), _final_third(recs, "lev")))
    print(env, precision, "build (seed, growth %/step, lev):", got, "band", (g_lo, g_hi), (l_lo, l_hi))
    for seed, g, lv in got:
        assert g_lo <= g <= g_hi, (env, precision, seed, g, (g_lo, g_hi))
        assert l_lo <= lv <= l_hi, (env, precision, seed, lv, (l_lo, l_hi))
