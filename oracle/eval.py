"""Evaluation episodes and their summary — TEST INFRASTRUCTURE (see oracle/__init__.py).

Restates tools/eval_episodes.py:176-399 (eval_multiplicative): each episode
starts from the env's reset state, holds the policy's action for the whole
episode (utils.action_window first when warmup < cum_steps <= smoothing_window,
which makes it float64), steps until done or max_eval_steps, and keeps the last
reward, the step count and the last risk vector; the summary is the reference's
own NumPy expressions (:289-330).  Pinned by tests/golden/eval.npz, produced by
running the reference's eval_multiplicative itself.
"""
import math

import numpy as np

from . import envs as oe


def window_action(action_f32, cum, warmup, smoothing):
    a = np.asarray(action_f32, dtype=np.float32)
    if cum <= smoothing and cum > warmup:
        w = (math.sin(math.pi * (cum / smoothing - 0.5)) + 1) / 2
        return np.clip(a.astype(np.float64), w * -0.99, w * 0.99)
    return a


def rollout(family, investor, n, action_f32, cum, warmup, smoothing, n_eval, max_steps, draws):
    """draws [n_eval, max_steps, D] -> (last reward [n_eval], steps, last risk [n_eval, R])."""
    a = window_action(action_f32, cum, warmup, smoothing)
    env = oe.OracleVecEnv(family, investor, n_eval, n)
    env.reset()
    acts = np.repeat(a[None, :], n_eval, 0)
    reward, steps = np.zeros(n_eval), np.zeros(n_eval, np.int64)
    risk = np.zeros((n_eval, env.R))
    live = np.ones(n_eval, bool)
    with np.errstate(all="ignore"):  # finished lanes keep stepping (ignored)
        for k in range(max_steps):
            _, r, d, rk = env.step(acts, draws[:, k])
            reward[live], risk[live], steps[live] = r[live], rk[live], k + 1
            live &= ~d[:, 0]
            if not live.any():
                break
    return reward, steps, risk


def market_rollout(algo, actor, prices, investor, obs_days, test_days, starts, cum, warmup, smoothing,
                   shuffle_days=1, seed=0, max_action=0.99, policy=None):
    """eval_market (tools/eval_episodes.py:402-611): episode i runs a Market_Inv?_D1/Dx
    env of time_length test_days + obs_days - 1 over the extract starting at price
    row starts[i] (gap + eval_start_idx), shuffled in blocks of shuffle_days (the
    Philox block permutations of oracle.envs); every step the deterministic policy
    (tanh(mu) * max_action, algo_sac.py:220-236 / algo_td3.py:225-238) acts on the
    f32 cast of the state (:507), action_window'd when cum <= smoothing (:509-517).
    actor: {param name: tensor} of the actor net (policy: a callable state f32 ->
    mu replacing its forward, e.g. a restatement of the bf16 kernel).  Returns (last reward, steps,
    last risk) per episode, as eval_log[..., 1], eval_log[..., 2], eval_risk_log[..., 1:]."""
    import torch

    from .learn import mlp

    n_eval = len(starts)
    tl = test_days + obs_days - 1
    env = oe.OracleVecEnv(oe.MARKET, investor, n_eval, prices.shape[1], seed=seed, prices=prices,
                          obs_days=obs_days, time_length=tl, shuffle_days=shuffle_days,
                          sample_days=tl + 1)
    state = env.reset(start_at=np.asarray(starts))
    head = "pi" if algo == "SAC" else "mu"
    reward, steps = np.zeros(n_eval), np.zeros(n_eval, np.int64)
    risk = np.zeros((n_eval, env.R))
    live = np.ones(n_eval, bool)
    n_steps = tl if obs_days == 1 else tl - obs_days + 1
    with np.errstate(all="ignore"), torch.no_grad():
        for k in range(n_steps):
            x = torch.from_numpy(state.astype(np.float32))
            mu = policy(x) if policy is not None else mlp(actor, x, head)[1]
            a = (torch.tanh(mu) * max_action).numpy()
            a = window_action(a, cum, warmup, smoothing)
            state, r, d, rk = env.step(a)
            reward[live], risk[live], steps[live] = r[live], rk[live], k + 1
            live &= ~d[:, 0]
            if not live.any():
                break
    return reward, steps, risk


def market_summary(reward, steps, risk_log):
    """The 14 statistics of eval_market (eval_episodes.py:545-585); risk_log is
    eval_risk_log's row [gap, risk...], so V$ is risk[0] and the 'lev' column risk[2]."""
    return summary(reward, steps, risk_log, oe.INV_A)[1:15]


def summary(reward, steps, risk, investor):
    """The 15 statistics of eval_episodes.py:289-330, then mean stop-loss / retention."""
    mean_reward = np.mean(reward)
    med_reward = np.percentile(reward, q=50, method="median_unbiased")
    reward_95 = np.percentile(reward, q=5, method="median_unbiased")
    mad_reward = np.mean(np.abs(reward - mean_reward))
    std_reward = np.std(reward, ddof=0)
    val = risk[:, 1]
    mean_val = np.mean(val)
    med_val = np.percentile(val, q=50, method="median_unbiased")
    val_95 = np.percentile(val, q=5, method="median_unbiased")
    mad_val = np.mean(np.abs(val - mean_val))
    mean_lev = np.mean(risk[:, 3])
    step = np.asarray(steps, dtype=np.float64)
    mean_step = np.mean(step)
    med_step = np.percentile(step, q=50, method="median_unbiased")
    step_95 = np.percentile(step, q=5, method="median_unbiased")
    mad_step = np.mean(np.abs(step - mean_step))
    std_step = np.std(step, ddof=0)
    stop = np.mean(risk[:, 4]) if investor in (oe.INV_B, oe.INV_C) else np.nan
    ret = np.mean(risk[:, 5]) if investor == oe.INV_C else np.nan
    return np.array([mean_lev * 100, (mean_reward - 1) * 100, (med_reward - 1) * 100, (reward_95 - 1) * 100,
                     mad_reward * 100, std_reward * 100, mean_val, med_val, val_95, mad_val, mean_step, med_step,
                     step_95, mad_step, std_step, stop, ret])
