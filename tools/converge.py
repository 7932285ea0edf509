"""Convergence of the vectorised loop to the analytic Kelly optima.

north_star's second parity bar: the headline loop (VecTrainer, SAC, bf16,
K updates per vector step) must learn the growth-optimal leverage of the
multiplicative gambles.  The reference's own yardstick is the Kelly fraction
(lev/lev_exp.py:495-496: kelly = pu/rd - (1-pu)/ru); the growth rate of a
constant leverage l is g(l) = sum_i p_i log(1 + l r_i) for the envs'
outcome tables (envs/coin_flip_envs.py:40-93, dice_roll_envs.py:39-96,
dice_roll_sh_envs.py:39-118).

The observation of these envs is divided by MAX_VALUE = 1e18, so the policy is
effectively state-independent and its deterministic action IS the learned
constant leverage (lev = action * LEV_FACTOR).  Every `--eval-every` vector
steps this tool records
  * the deterministic action at the reset state and its leverage,
  * eval_multiplicative on the device (rlmd_eval_rollout, n_eval episodes of
    100 steps at that constant action) -> mean time-average growth per step,
  * the analytic growth g(lev) of that leverage,
and writes one JSON line per record (progress for the GPU box).

    python tools/converge.py --env coin --lanes 65536 --k 8 --steps 20000
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# outcome tables (p_i, r_i) and the action -> leverage map of each env
GAMBLES = {
    # coin_flip_envs.py:40-93: +50 % / -40 %, p = 1/2, LEV_FACTOR = 2
    "coin": dict(p=[0.5, 0.5], r=[0.5, -0.4], lev_factor=2.0, investor="A"),
    # dice_roll_envs.py:39-96: +50 % (1/6), -50 % (1/6), +5 % (2/3), LEV_FACTOR = 2
    "dice": dict(p=[1 / 6, 1 / 6, 2 / 3], r=[0.5, -0.5, 0.05], lev_factor=2.0, investor="A"),
}
# dice_roll_sh_envs.py:39-118: die + safe haven; INSURED: lev = a * I_LF, lev_sh = 1 - lev;
# R = lev * r + lev_sh * r_sh, with r_sh = -0.99 on UP / MID and +5 on DOWN
SH_I_LF = (-1 - 5) / (-0.5 - 5)
SH = dict(p=[1 / 6, 1 / 6, 2 / 3], r=[0.5, -0.5, 0.05], r_sh=[-0.99, 5.0, -0.99], lev_factor=SH_I_LF,
          investor="INSURED")
# envs of the metric's own workloads: GBM_InvA (key 14, lev = a * 5,
# gbm_envs.py:147-212) and Dice_SH_InvA (key 18, lev = a0 * 2, lev_sh = (a1 + .99) / 2,
# dice_roll_sh_envs.py:290-365); the eval risk row holds lev at column 3 and, for
# Dice_SH_InvA, lev_sh at column 6 (the reference's eval_risk_log columns)
FAMILY = {"coin": ("coin", "A"), "dice": ("dice", "A"), "dice_sh": ("dice_sh", "INSURED"), "gbm": ("gbm", "A"),
          "dice_sh_a": ("dice_sh", "A"), "market": ("market", "A")}
# C4 (key 21, SNP_InvA, D1): main.py's market schedule -- 1e3 training days per
# episode, 250 test days, shuffled in 5 / 3-day intervals, a 5-20 day gap
# (rl_market.py:56-60, eval_episodes.py:402-611); no analytic optimum


def market_kw():
    with np.load(os.path.join(ROOT, "tests", "golden", "stooq_snp.npz"), allow_pickle=False) as z:
        prices = np.ascontiguousarray(z[z.files[0]], dtype=np.float64).reshape(-1, 1)
    return dict(prices=prices, obs_days=1, time_length=1000, shuffle_days=5, sample_days=1000 + 250 + 1 + 20 - 1)
# GBM log-return N(mu - sigma^2 / 2, sigma) (gbm_envs.py:43-63): expected log growth
# lev * (mu - sigma^2 / 2) per step, monotone in lev (the optimum is the 4.95 corner,
# tempered by the lev_max termination)
GBM_MU, GBM_SIGMA = 0.0540025395205692, 0.1897916175617430


def growth(env, lev, lev_sh=None):
    """Expected log growth per step of a constant leverage (natural log)."""
    if env == "gbm":
        return float(lev * (GBM_MU - GBM_SIGMA ** 2 / 2))
    if env == "dice_sh_a":
        p, r, rs = np.array(SH["p"]), np.array(SH["r"]), np.array(SH["r_sh"])
        R = np.maximum(lev * r + (lev_sh if lev_sh is not None else 0.0) * rs, -0.99)
        return float(np.sum(p * np.log1p(R)))
    if env == "dice_sh":
        p, r, rs = np.array(SH["p"]), np.array(SH["r"]), np.array(SH["r_sh"])
        R = lev * r + (1.0 - lev) * rs
    else:
        g = GAMBLES[env]
        p, R = np.array(g["p"]), lev * np.array(g["r"])
    R = np.maximum(R, -0.99 if env == "dice_sh" else -0.9)  # env MIN_RETURN clips
    return float(np.sum(p * np.log1p(R)))


def kelly(env):
    """Growth-optimal leverage (golden-section search of g) and its growth %/step.
    GBM: the max-leverage corner; Dice_SH_InvA: a grid over (lev, lev_sh)."""
    if env == "gbm":
        return 4.95, 100.0 * math.expm1(growth("gbm", 4.95))
    if env == "dice_sh_a":
        best = max((growth(env, l, h), l, h) for l in np.linspace(-1.98, 1.98, 397)
                   for h in np.linspace(0.0, 0.99, 100))
        return best[1], 100.0 * math.expm1(best[0])
    lf = SH["lev_factor"] if env == "dice_sh" else GAMBLES[env]["lev_factor"]
    lo, hi = 0.0, 0.99 * lf
    for _ in range(200):
        m1, m2 = lo + (hi - lo) * 0.382, lo + (hi - lo) * 0.618
        if growth(env, m1) < growth(env, m2):
            lo = m1
        else:
            hi = m2
    l = 0.5 * (lo + hi)
    return l, 100.0 * math.expm1(growth(env, l))


def run(env, lanes, k, steps, precision="bf16", warmup=1000, smoothing=2000, eval_every=500, n_eval=4096,
        seed=0, replay=1 << 20, algo="SAC", out=None, log=print, device="cuda:0", loss="MSE", schedule="updates", multi_steps=1,
        slice_groups=0, stored_state="reference"):
    """warmup / smoothing: the reference's lengths (main.py gym_envs warm-up 1e3,
    smoothing_window_mul 2e3), mapped to vector steps by trainer.schedule_steps.
    stored_state: the replay rows' s (VecTrainer.set_stored_state; "reference" =
    the reference loop's aliased post-step state)."""
    import torch

    from rlmd_amd.trainer import VecTrainer, schedule_steps

    fam, inv = FAMILY[env]
    kw = market_kw() if env == "market" else {}
    tr = VecTrainer(env=fam, investor=inv, n_lanes=lanes, n_gambles=1, algo=algo, loss=loss, k_updates=k,
                    replay_capacity=replay, seed=seed, warmup_steps=schedule_steps(warmup, k, schedule),
                    smoothing_window=schedule_steps(smoothing, k, schedule), precision=precision, device=device,
                    init_seed=seed, multi_steps=multi_steps, slice_groups=slice_groups, stored_state=stored_state, **kw)
    l_star, g_star = kelly(env) if env != "market" else (None, None)
    # the reset state (identical for every lane; market lanes start on their own slices)
    reset_obs = tr.env.reset()[:1].float().clone() if env != "market" else tr.obs[:1].float().clone()
    tr2 = None
    recs = []
    t0 = time.perf_counter()
    for step in range(1, steps + 1):
        tr.step()
        if step % eval_every == 0 or step == steps:
            a = tr.agent.act(reset_obs, mode=1)[0].cpu().numpy()
            if env == "market":
                # eval_risk_log = [gap, reward, wealth, step return, mean lev, ...]
                # (eval_episodes.py:542-543, market_envs.py:196): the leverage is column 4
                # (the reference's summary prints column 3, the last step's return, as
                # "lev")
                # episode i starts from lane (i mod N)'s position plus a gap (one
                # evaluation launch summarises at most 1,024 episodes)
                ev = tr.evaluate_market(n_eval=min(n_eval, 1024), test_days=250)
                lev = float(np.mean(ev["risk_log"][:, 4]))
            else:
                ev = tr.evaluate(n_eval=n_eval, max_steps=100, with_stats=False)
                # the reference's statistic: the eval risk rows' leverage column
                # (eval_episodes.py:267-274 -> eval_risk_log[..., 3]; lev_sh at 6)
                lev = float(np.mean(ev["risk"][:, 3]))
            grow = 100.0 * float(np.mean(ev["reward"] - 1.0))
            lev_sh = float(np.mean(ev["risk"][:, 6])) if env == "dice_sh_a" else None
            rec = {"env": env, "algo": algo, "loss": loss, "precision": precision, "lanes": lanes, "k": k,
                   "replay": replay, "multi_steps": multi_steps, "stored_state": stored_state, "step": step, "updates": step * k, "env_steps": step * lanes,
                   "action": [float(x) for x in a], "lev": lev, "lev_sh": lev_sh,
                   "eval_growth_pct": grow, "eval_steps": float(np.mean(ev["steps"])),
                   "analytic_growth_pct": None if env == "market" else 100.0 * math.expm1(growth(env, lev, lev_sh)),
                   "kelly_lev": l_star, "kelly_growth_pct": g_star, "wall_s": time.perf_counter() - t0,
                   "nan_flag": tr.agent.scalars()["nan_flag"], "log_alpha": tr.agent.scalars()["log_alpha"]}
            recs.append(rec)
            log(json.dumps(rec))
            if out is not None:
                out.write(json.dumps(rec) + "\n")
                out.flush()
    return recs


def market_single(seed, steps=100000, n_eval=20):
    """C4's single-stream control: the build's reference-API market driver
    (rlmd_amd.main.run -> scripts/rl_market.market_env: one env, one update per
    env step, the device Agent_sac) on the reference's settings (key 21, SAC /
    MSE, `steps` steps, evaluations of n_eval episodes x 250 test days, np.random
    and torch seeded with `seed`).  Returns the per-evaluation growth %/step and
    leverage (eval_risk_log column 4), averaged over the episodes."""
    import tempfile

    import torch

    from rlmd_amd.config import INPUTS
    from rlmd_amd.main import run as main_run

    prices = market_kw()["prices"]
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            os.makedirs("market_data")
            np.save("market_data/stooq_snp.npy", prices)
            np.random.seed(seed)
            torch.manual_seed(seed)
            inputs = dict(INPUTS, n_trials_mkt=1, n_cumsteps_mkt=float(steps), n_eval_mkt=n_eval,
                          market_dir="./market_data/", test_agent=True)
            ((_, _, ev, _, ev_risk),), = main_run([21], ["SAC"], ["MSE"], [1], inputs=inputs, log=None)[21]
        finally:
            os.chdir(cwd)
    return 100.0 * (ev[0, :, :, 1] - 1.0).mean(1), ev_risk[0, :, :, 4].mean(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="coin", choices=sorted(FAMILY))
    ap.add_argument("--lanes", type=int, default=65536)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--smoothing", type=int, default=2000)
    ap.add_argument("--eval-every", type=int, default=500)
    ap.add_argument("--n-eval", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--replay", type=int, default=1 << 20)
    ap.add_argument("--algo", default="SAC", choices=["SAC", "TD3"])
    ap.add_argument("--loss", default="MSE")
    ap.add_argument("--schedule", default="updates", choices=["updates", "vector"])
    ap.add_argument("--multi-steps", type=int, default=1)
    ap.add_argument("--out", default=None, help="append JSON lines here")
    a = ap.parse_args()
    out = open(a.out, "a") if a.out else None
    run(a.env, a.lanes, a.k, a.steps, a.precision, a.warmup, a.smoothing, a.eval_every, a.n_eval, a.seed,
        a.replay, a.algo, out, loss=a.loss, schedule=a.schedule, multi_steps=a.multi_steps)


if __name__ == "__main__":
    main()
