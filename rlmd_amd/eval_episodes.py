"""Evaluation episodes of the single-agent drivers, on the device.

``eval_multiplicative`` keeps tools/eval_episodes.py:176-399's signature and
log layout: n_eval episodes of <= max_eval_steps on a fresh env, each with ONE
constant action (the deterministic policy at the episode's reset state, the
action window applied as at cum_steps, :231-243), logging per episode
[time, reward, steps, loss[11], logtemp, loss_params[4], cum_steps] and the
last risk row (:263-273).  All episodes run as lanes of one rlmd_eval_rollout
launch; the event's wall time is split evenly over them.  The reference's
printed summary statistics come from rlmd_eval_stats (NumPy-exact).

``eval_market`` keeps tools/eval_episodes.py:402-611's signature and log
layout for the single-stream market driver (rlmd_amd.scripts.rl_market): the
gaps are drawn on the host as the reference draws them (one
``np.random.randint(gap_min, gap_max + 1, n_eval)``, offset by
eval_start_idx), then every episode runs as one lane of rlmd_eval_market
(trainer.market_evaluate: test slice of test_days + obs_days - 1 steps from
row gap_i, shuffled in blocks of test_shuffle_days, the deterministic policy
acting every day, the action window as at cum_steps), logging
[time, reward, steps, loss[11], logtemp, loss_params[4], cum_steps] and
[gap, risk...] per episode (:528-543).  The evaluation env is created once per
(price table, shape) and reused; each event's resets advance its Philox
episode counters, so every event draws fresh shuffles.

``agent_shadow_mean`` is tools/utils.py:441-471 on the device
(rlmd_shadow_means on the 16-entry statistics row).
"""
import time

import numpy as np
import torch

from . import _abi
from ._abi import check, ptr, stream_ptr
from .envs import ENV_CLASSES, VecEnv, private_seed

# Evaluation envs, reused across the events of one driver run (building one
# allocates device lanes).  Bounded, and cleared by the drivers when they return
# (clear_eval_envs), so a run over many env keys does not keep every key's envs
# and device price tables alive.
_EVAL_ENVS = {}
_MARKET_EVAL_ENVS = {}
_MAX_CACHED = 4


def _cache_put(cache, key, value):
    while len(cache) >= _MAX_CACHED:
        cache.pop(next(iter(cache)))
    cache[key] = value


def clear_eval_envs():
    """Drop the cached evaluation envs (the drivers call this when they return)."""
    _EVAL_ENVS.clear()
    _MARKET_EVAL_ENVS.clear()


def env_class_name(env_id):
    """main.py gym_envs name of an inputs["env_id"] (name + "_n" + n_gambles)."""
    name = str(env_id)
    return name.rsplit("_n", 1)[0] if name.rsplit("_n", 1)[-1].isdigit() else name


def _eval_env(inputs, n_gambles, n_eval, device):
    cls = ENV_CLASSES[env_class_name(inputs["env_id"])]
    key = (cls.family, cls.investor, n_gambles, n_eval, str(device))
    env = _EVAL_ENVS.get(key)
    if env is None:
        seed = int(inputs["eval_seed"]) if "eval_seed" in inputs else private_seed()
        env = VecEnv(cls.family, cls.investor, n_eval, n_gambles, seed=seed, device=device)
        _cache_put(_EVAL_ENVS, key, env)
    return env


def agent_shadow_mean(inputs, loss, device=None):
    """[shadow1, shadow2] of tools/utils.py:441-471 (loss[0:2] where the tail index
    is >= 1), computed by rlmd_shadow_means."""
    dev = torch.device(device or "cuda:0")
    row = torch.tensor(np.asarray(list(loss[:11]) + [0.0] * 5, dtype=np.float32), device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    check(_abi.lib().rlmd_shadow_means(ptr(row), 1, 16, float(inputs["shadow_low_mul"]),
                                       float(inputs["shadow_high_mul"]), ptr(out), 2, stream_ptr()))
    s = out.cpu().numpy().astype(np.float64)
    return [float(s[0]), float(s[1])]


def eval_multiplicative(n_gambles, agent, inputs, eval_log, eval_risk_log, multi_step, cum_steps, round, eval_run,
                        loss, logtemp, loss_params, device=None):
    dev = torch.device(device or agent.dev.device)
    n_eval = int(inputs["n_eval"])
    env = _eval_env(inputs, n_gambles, n_eval, dev)
    t0 = time.perf_counter()
    obs = env.reset().float()
    actions = agent.dev.act(obs, mode=1)
    reward = torch.empty(n_eval, dtype=torch.float64, device=dev)
    steps = torch.empty(n_eval, dtype=torch.int32, device=dev)
    risk = torch.empty(n_eval, env.risk_dim, dtype=torch.float64, device=dev)
    check(_abi.lib().rlmd_eval_rollout(env.h, ptr(actions), int(inputs["max_eval_steps"]), int(cum_steps),
                                       int(inputs["random"]), int(inputs["smoothing_window"]), None, ptr(reward),
                                       ptr(steps), ptr(risk), stream_ptr()))
    r, st, rk = reward.cpu().numpy(), steps.cpu().numpy(), risk.cpu().numpy()
    dt = time.perf_counter() - t0
    e = eval_log[round, eval_run]
    e[:, 0] = dt / n_eval
    e[:, 1] = r
    e[:, 2] = st
    e[:, 3:14] = np.asarray(loss, dtype=np.float64)
    e[:, 14] = logtemp
    e[:, 15:19] = np.asarray(loss_params, dtype=np.float64)
    e[:, 19] = cum_steps
    eval_risk_log[round, eval_run] = rk
    return {"reward": r, "steps": st, "risk": rk}


def _market_eval_env(market_data, investor, obs_days, test_length, n_eval, shuffle, action_days, device):
    from .envs import VecEnv

    key = (id(market_data), investor, obs_days, test_length, n_eval, shuffle, action_days, str(device))
    hit = _MARKET_EVAL_ENVS.get(key)
    if hit is not None and hit[0] is market_data:
        return hit[1]
    seed = private_seed()
    env = VecEnv("market", investor, n_eval, market_data.shape[1], seed=seed, prices=market_data,
                 obs_days=obs_days, time_length=test_length, action_days=action_days, shuffle_days=shuffle,
                 sample_days=test_length * action_days + 1, device=device)
    _cache_put(_MARKET_EVAL_ENVS, key, (market_data, env))
    return env


def market_investor(env_id):
    """'A' / 'B' / 'C' of a market env_id such as SNP_InvB_D1_T1 (the
    reference's inputs["env_id"][-10:-6] is 'InvB')."""
    return str(env_id).split("_Inv")[1][0]


def eval_market(market_data, obs_days, eval_start_idx, agent, inputs, eval_log, eval_risk_log, multi_step, cum_steps,
                round, eval_run, loss, logtemp, loss_params, device=None):
    from .trainer import market_evaluate

    market_data = np.asarray(market_data, dtype=np.float64)
    n_eval = int(inputs["n_eval"])
    action_days = int(inputs["action_days"])
    test_length = int(inputs["test_days"] + obs_days - 1)
    gap = np.random.randint(int(inputs["gap_days_min"]), int(inputs["gap_days_max"]) + 1, size=n_eval)
    gap += eval_start_idx
    dev = torch.device(device or agent.dev.device)
    inv = market_investor(inputs["env_id"])
    env = _market_eval_env(market_data, inv, obs_days, test_length, n_eval, int(inputs["test_shuffle_days"]),
                           action_days, dev)
    t0 = time.perf_counter()
    res = market_evaluate(agent.dev, market_data, inv, obs_days, int(inputs["test_days"]), gap, int(cum_steps),
                          int(inputs["random"]), int(inputs["smoothing_window"]),
                          shuffle_days=int(inputs["test_shuffle_days"]), action_days=action_days, device=dev, env=env)
    dt = time.perf_counter() - t0
    e = eval_log[round, eval_run]
    e[:, 0] = dt / n_eval
    e[:, 1] = res["reward"]
    e[:, 2] = res["steps"]
    e[:, 3:14] = np.asarray(loss, dtype=np.float64)
    e[:, 14] = logtemp
    e[:, 15:19] = np.asarray(loss_params, dtype=np.float64)
    e[:, 19] = cum_steps
    eval_risk_log[round, eval_run, :, 0] = gap
    eval_risk_log[round, eval_run, :, 1:] = res["risk"]
    return dict(res, gap=gap)

