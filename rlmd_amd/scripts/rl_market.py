"""Single-stream training driver for the market envs (keys 21-26).

The build's counterpart of scripts/rl_market.py:42-491 over the
reference-named facade classes (``Market_Inv{A,B,C}_{D1,Dx}`` from
rlmd_amd.envs, ``Agent_sac`` / ``Agent_td3`` from rlmd_amd.agent), so a
reference ``gym_envs`` / ``inputs`` pair and price table run unchanged:

  * per episode: ``time_slice`` (random start row; sample_length reserves the
    test window and the largest gap, :54-62), ``shuffle_data`` in blocks of
    train_shuffle_days, the first observation (``observed_market_state``) and
    ``env.reset(obs)`` (:199-214; host NumPy, rlmd_amd.env_resources);
  * per step: the warm-up action is the raw ``env.action_space.sample()`` (no
    absolute value on markets, :220-224), then ``agent.select_next_action``;
    the float64 action window while cum_steps <= smoothing_window (:226-234);
    the next observation and ``env.step(action, obs)`` on the device
    (envs/market_envs.py:133-202, :611-682); ``store_transistion`` with
    learn_done; ``learn()`` every grad_step steps with the NaN guard
    (:250-272);
  * evaluation every eval_freq steps from eval_start_idx = start_idx + step
    with loss[6:8] = agent_shadow_mean first (:281-301), on the device
    (rlmd_amd.eval_episodes.eval_market);
  * per-episode trial rows and the last risk vector (:303-311), the
    trailing-score checkpoint (:313-320), ``continue`` (:172-183), and the four
    .npy logs under utils.save_directory truncated to the longest trial
    (:459-478).

Test hooks (not in the reference signature): ``env`` replaces the env built
from gym_envs, ``agent_factory(inputs)`` the Agent_sac / Agent_td3 choice.
"""
import os
import time

import numpy as np

from .. import env_resources, eval_episodes, logs
from ..agent import Agent_sac, Agent_td3
from ..envs import ENV_CLASSES
from .rl_multiplicative import action_window, critic_learning


def make_env(gym_envs, key, n_assets, train_length, obs_days, device=None, seed=None):
    """Market_<Inv>_D1 / _Dx (rl_market.py:70-83: the env_id's last four letters)."""
    cls = ENV_CLASSES["Market_" + gym_envs[str(key)][0][-4:] + ("_D1" if obs_days == 1 else "_Dx")]
    kw = {} if device is None else {"device": device}
    return cls(n_assets, train_length, obs_days, seed=seed, **kw)


def market_env(gym_envs, inputs, market_data, obs_days, env=None, agent_factory=None, log=print, device=None):
    try:
        return _market_env(gym_envs, inputs, market_data, obs_days, env, agent_factory, log, device)
    finally:
        eval_episodes.clear_eval_envs()  # the evaluation envs live for one driver run


def _market_env(gym_envs, inputs, market_data, obs_days, env, agent_factory, log, device):
    market_data = np.asarray(market_data, dtype=np.float64)
    n_assets = market_data.shape[1]
    action_days = int(inputs["action_days"])
    train_length = int(inputs["train_days"] + obs_days - 1)
    test_length = int(inputs["test_days"] + obs_days - 1)
    gap_max = int(inputs["gap_days_max"])
    sample_length = int(action_days * (train_length + test_length) + obs_days + gap_max - 1)
    inputs = {"env_id": gym_envs[str(inputs["ENV_KEY"])][0] + f"_D{obs_days}_T{action_days}", **inputs}
    if env is None:
        env = make_env(gym_envs, inputs["ENV_KEY"], n_assets, train_length, obs_days, device=device)
    inputs = {
        "input_dims": env.observation_space.shape, "num_actions": env.action_space.shape[0],
        "max_action": env.action_space.high.max(), "min_action": env.action_space.low.min(),
        "random": gym_envs[str(inputs["ENV_KEY"])][3], "dynamics": "MKT", "n_trials": inputs["n_trials_mkt"],
        "n_cumsteps": inputs["n_cumsteps_mkt"], "trial": 0, "eval_freq": inputs["eval_freq_mkt"],
        "n_eval": inputs["n_eval_mkt"], "smoothing_window": inputs["smoothing_window_mkt"],
        "actor_percentile": inputs["actor_percentile_mkt"], "critic_percentile": inputs["critic_percentile_mkt"],
        "algo": "TD3", "s_dist": "N", "mini_batch_size": 1, "loss_fn": "MSE", "multi_steps": 1, **inputs,
    }
    risk_dim = logs.market_log_dim(inputs["env_id"], n_assets)
    factory = agent_factory or (lambda inp: Agent_td3(inp) if inp["algo"] == "TD3" else Agent_sac(inp))
    n_cum, n_trials = int(inputs["n_cumsteps"]), int(inputs["n_trials"])
    n_evals, n_eval = int(inputs["n_cumsteps"] / inputs["eval_freq"]), int(inputs["n_eval"])
    shape = dict(n_assets=n_assets, action_days=action_days, train_length=train_length, sample_length=sample_length,
                 obs_days=obs_days)
    out = []
    for algo in inputs["algo_name"]:
        inputs["s_dist"] = inputs["sample_dist"][algo]
        bsz = int(inputs["batch_size"][algo])
        actor_batch = int(bsz / inputs["actor_percentile"] * 100)
        critic_batch = int(bsz / inputs["critic_percentile"] * 100)
        inputs["mini_batch_size"] = max(actor_batch, critic_batch)
        for loss_fn in inputs["critic_loss"]:
            for mstep in inputs["bootstraps"]:
                inputs["loss_fn"], inputs["algo"], inputs["multi_steps"] = loss_fn, algo, mstep
                trial_log = np.zeros((n_trials, n_cum, 19), dtype=np.float32)
                eval_log = np.zeros((n_trials, n_evals, n_eval, 20), dtype=np.float32)
                directory = logs.save_directory(inputs, results=True)
                trial_risk_log = np.zeros((n_trials, n_cum, risk_dim), dtype=np.float32)
                eval_risk_log = np.zeros((n_trials, n_evals, n_eval, risk_dim + 1), dtype=np.float32)
                logtemp, prev_prefix = None, None
                for rnd in range(n_trials):
                    inputs["trial"] = rnd + 1
                    cont = rnd > 0 and inputs["continue"]
                    if cont:
                        inputs["initial_logtemp"] = logtemp
                    agent = factory(inputs)
                    if cont:
                        # as in rl_multiplicative: the previous trial's checkpoints (the
                        # reference's load_models() looks under the new trial's name)
                        agent.load_models(prefix=prev_prefix)
                    rows = _run_trial(env, agent, inputs, market_data, shape, mstep, rnd, eval_log, eval_risk_log,
                                      log)
                    count = len(rows["score"])
                    trial_log[rnd, :count, 0], trial_log[rnd, :count, 1] = rows["time"], rows["score"]
                    trial_log[rnd, :count, 2], trial_log[rnd, :count, 3:14] = rows["steps"], rows["loss"]
                    trial_log[rnd, :count, 14], trial_log[rnd, :count, 15:] = rows["logtemp"], rows["params"]
                    trial_risk_log[rnd, :count, :] = rows["risk"]
                    logtemp = rows["logtemp"][-1]
                    prev_prefix = getattr(agent, "file_prefix", None)
                counts = [int(np.min(np.where(trial_log[t, :, 0] == 0)[0])) if (trial_log[t, :, 0] == 0).any()
                          else n_cum for t in range(n_trials)]
                m = max(counts)
                trial_log, trial_risk_log = trial_log[:, :m], trial_risk_log[:, :m]
                os.makedirs(os.path.dirname(directory), exist_ok=True)
                np.save(directory + "_trial.npy", trial_log)
                np.save(directory + "_eval.npy", eval_log)
                np.save(directory + "_trial_risk.npy", trial_risk_log)
                np.save(directory + "_eval_risk.npy", eval_risk_log)
                out.append((directory, trial_log, eval_log, trial_risk_log, eval_risk_log))
    return out


def _run_trial(env, agent, inputs, market_data, shape, mstep, rnd, eval_log, eval_risk_log, log):
    rows = {k: [] for k in ("time", "score", "steps", "loss", "logtemp", "params", "risk")}
    cum_steps, eval_run, episode = 0, 0, 1
    best_score = env.reward_range[0]
    n_cum, eval_freq = int(inputs["n_cumsteps"]), int(inputs["eval_freq"])
    warmup, window = int(inputs["random"]), int(inputs["smoothing_window"])
    grad_step = int(inputs["grad_step"][inputs["algo"]])
    ad, d = shape["action_days"], shape["obs_days"]
    loss, logtemp, loss_params = [np.nan] * 11, np.nan, [np.nan] * 4
    while cum_steps < n_cum:
        start_time = time.perf_counter()
        market_slice, start_idx = env_resources.time_slice(market_data, shape["train_length"], ad,
                                                           shape["sample_length"])
        extract = env_resources.shuffle_data(market_slice, inputs["train_shuffle_days"])
        time_step = 0
        state = env.reset(env_resources.observed_market_state(extract, time_step, ad, d))
        done, step, score = False, 0, 0
        end_time = start_time
        risk = None
        while not done:
            time_step += 1
            if cum_steps >= warmup:
                action = agent.select_next_action(state)
            else:
                action = env.action_space.sample()  # raw sample on markets (rl_market.py:224)
            if cum_steps <= window:
                action = action_window(action, inputs["max_action"], inputs["min_action"], cum_steps, window, warmup)
            obs = env_resources.observed_market_state(extract, time_step, ad, d)
            next_state, reward, env_done, risk = env.step(action, obs)
            done, learn_done = env_done[0], env_done[1]
            agent.store_transistion(state, action, reward, next_state, learn_done)
            if cum_steps % grad_step == 0:
                loss, logtemp, loss_params = agent.learn()
                critic_learning(cum_steps, inputs["mini_batch_size"], loss)
            state = next_state
            score = reward
            step += 1
            cum_steps += 1
            end_time = time.perf_counter()
            if cum_steps % eval_freq == 0:
                loss = list(loss)
                loss[6:8] = eval_episodes.agent_shadow_mean(inputs, loss)
                eval_episodes.eval_market(market_data, d, start_idx + step, agent, inputs, eval_log, eval_risk_log,
                                          mstep, cum_steps, rnd, eval_run, loss, logtemp, loss_params)
                eval_run += 1
            if cum_steps >= n_cum:
                break
        loss = list(loss)
        loss[6:8] = eval_episodes.agent_shadow_mean(inputs, loss)
        rows["time"].append(end_time - start_time)
        rows["score"].append(score)
        rows["steps"].append(step)
        rows["loss"].append(list(loss))
        rows["logtemp"].append(logtemp)
        rows["params"].append(list(loss_params))
        rows["risk"].append(np.asarray(risk, dtype=np.float64).ravel())
        trail_score = np.mean(rows["score"][-int(inputs["trail"]):])
        if trail_score > best_score:
            best_score = trail_score
            agent.save_models()
        if log is not None and (episode % 10 == 0 or cum_steps >= n_cum):
            log(f"E{inputs['ENV_KEY']}_m{mstep}_d{d}_t{ad} {inputs['algo']}-{inputs['s_dist']}-{inputs['loss_fn']}-"
                f"{rnd + 1} ep {episode} cst/st {cum_steps}/{step} T {start_idx + time_step}: "
                f"l% {100 * float(np.ravel(risk)[3]):1.0f}, g% {100 * (reward - 1):1.1f}, "
                f"C {np.nanmean(loss[0:2]):1.2f}")
        episode += 1
    return rows
