"""Single-stream training driver for the multiplicative envs (config C1).

The build's counterpart of scripts/rl_multiplicative.py:41-457: the same
schedule over the reference-named facade classes (``Coin_InvA`` ... from
rlmd_amd.envs, ``Agent_sac`` / ``Agent_td3`` from rlmd_amd.agent), so a
reference ``gym_envs`` / ``inputs`` pair runs unchanged:

  * warm-up: ``env.action_space.sample()`` (absolute value except GBM) for the
    first gym_envs[key][3] steps, then ``agent.select_next_action`` (:192-201);
  * the action window (float64 clip) while cum_steps <= smoothing_window
    (:203-211, tools/utils.py:345-373);
  * env.step -> store_transistion(state, action, reward, next_state,
    learn_done) -> learn() every grad_step steps, with the NaN guard of
    tests/test_live_learning.py:119-255 (terminates the run: SystemExit);
  * evaluation every eval_freq steps with loss[6:8] = agent_shadow_mean first
    (:252-270), on the device (rlmd_amd.eval_episodes);
  * per-episode trial rows [time, score, steps, loss[11], logtemp,
    loss_params[4]] and the last risk vector (:275-283, :400-414);
  * a checkpoint (save_models) at every new high of the trailing mean of the
    last inputs["trail"] episode scores (:285-293); with inputs["continue"],
    trial r > 0 starts from the previous trial's log temperature and models
    (:172-183);
  * the four .npy logs under utils.save_directory, trial logs truncated to the
    longest trial (:436-450).

Test hooks (not in the reference signature): ``env`` replaces the env built
from gym_envs, ``agent_factory(inputs)`` the Agent_sac / Agent_td3 choice.
"""
import os
import time

import numpy as np

from .. import logs
from ..agent import Agent_sac, Agent_td3
from ..config import env_dynamics
from ..envs import ENV_CLASSES
from ..eval_episodes import agent_shadow_mean, clear_eval_envs, eval_multiplicative


def smoothing_func(ratio):
    """tools/utils.py:330-342."""
    return (np.sin(np.pi * (ratio - 1 / 2)) + 1) / 2


def action_window(action, max_action, min_action, cum_step, max_step, warmup):
    """tools/utils.py:345-373: clip post-warm-up actions to a widening window
    (np.float64 bounds, so the result is float64)."""
    if cum_step > warmup:
        width = smoothing_func(cum_step / max_step)
        return np.clip(action, width * min_action, width * max_action)
    return action


class NaNLearning(SystemExit):
    """The reference prints and exit()s when a critic statistic is NaN
    (tests/test_live_learning.py:255); the driver raises this SystemExit."""


def critic_learning(cum_step, batch_size, loss):
    """tests/test_live_learning.py:119-255's guard on loss[0:6] + loss[8:10]."""
    if cum_step > batch_size:
        critic = np.array(list(loss[0:6]) + list(loss[8:10]), dtype=np.float32)
        if np.any(np.isnan(critic)):
            print(f"Script terminated due to the presence of NaN's within critic losses. Cumulative Step: "
                  f"{cum_step}, critic statistics {critic}")
            raise NaNLearning(1)


def make_env(gym_envs, key, n_gambles, device=None, seed=None):
    name = gym_envs[str(key)][0]
    cls = ENV_CLASSES[name]
    kw = {} if device is None else {"device": device}
    return cls(seed=seed, **kw) if name.startswith("Dice_SH") else cls(n_gambles, seed=seed, **kw)


def multiplicative_env(gym_envs, inputs, n_gambles, env=None, agent_factory=None, log=print, device=None):
    try:
        return _multiplicative_env(gym_envs, inputs, n_gambles, env, agent_factory, log, device)
    finally:
        clear_eval_envs()  # the evaluation envs live for one driver run


def _multiplicative_env(gym_envs, inputs, n_gambles, env, agent_factory, log, device):
    inputs = {"env_id": gym_envs[str(inputs["ENV_KEY"])][0] + "_n" + str(n_gambles), **inputs}
    _, sh_key, _ = env_dynamics(gym_envs)
    if env is None:
        env = make_env(gym_envs, inputs["ENV_KEY"], n_gambles, device=device)
    inputs = {
        "input_dims": env.observation_space.shape, "num_actions": env.action_space.shape[0],
        "max_action": env.action_space.high.max(), "min_action": env.action_space.low.min(),
        "random": gym_envs[str(inputs["ENV_KEY"])][3], "dynamics": "M", "n_trials": inputs["n_trials_mul"],
        "n_cumsteps": inputs["n_cumsteps_mul"], "trial": 0, "eval_freq": inputs["eval_freq_mul"],
        "n_eval": inputs["n_eval_mul"], "max_eval_steps": inputs["max_eval_steps_mul"],
        "smoothing_window": inputs["smoothing_window_mul"], "actor_percentile": inputs["actor_percentile_mul"],
        "critic_percentile": inputs["critic_percentile_mul"], "algo": "TD3", "s_dist": "N", "mini_batch_size": 1,
        "loss_fn": "MSE", "multi_steps": 1, "env_gym": gym_envs[str(inputs["ENV_KEY"])][0], **inputs,
    }
    risk_dim = logs.multi_log_dim(inputs["env_id"], n_gambles)
    factory = agent_factory or (lambda inp: Agent_td3(inp) if inp["algo"] == "TD3" else Agent_sac(inp))
    n_cum, n_trials = int(inputs["n_cumsteps"]), int(inputs["n_trials"])
    n_evals, n_eval = int(inputs["n_cumsteps"] / inputs["eval_freq"]), int(inputs["n_eval"])
    warmup, window = int(inputs["random"]), int(inputs["smoothing_window"])
    gbm = "GBM" in inputs["env_id"]
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
                trial_risk_log = np.zeros((n_trials, n_cum, risk_dim), dtype=np.float32)
                eval_risk_log = np.zeros((n_trials, n_evals, n_eval, risk_dim), dtype=np.float32)
                directory = logs.save_directory(inputs, results=True)
                logtemp, prev_prefix = None, None
                for rnd in range(n_trials):
                    inputs["trial"] = rnd + 1
                    cont = rnd > 0 and inputs["continue"]
                    if cont:
                        inputs["initial_logtemp"] = logtemp
                    agent = factory(inputs)
                    if cont:
                        # the reference calls agent.load_models() on the NEW agent, whose
                        # file stem already carries this trial's number (utils.py:213-215),
                        # so it raises FileNotFoundError; the intent (main.py:212) is the
                        # previous trial's parameters, loaded here
                        agent.load_models(prefix=prev_prefix)
                    rows = _run_trial(env, agent, inputs, n_gambles, mstep, rnd, eval_log, eval_risk_log,
                                      warmup, window, gbm, sh_key, log)
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


def _run_trial(env, agent, inputs, n_gambles, mstep, rnd, eval_log, eval_risk_log, warmup, window, gbm, sh_key,
               log):
    rows = {k: [] for k in ("time", "score", "steps", "loss", "logtemp", "params", "risk")}
    cum_steps, eval_run, episode = 0, 0, 1
    best_score = env.reward_range[0]
    n_cum, eval_freq = int(inputs["n_cumsteps"]), int(inputs["eval_freq"])
    grad_step = int(inputs["grad_step"][inputs["algo"]])
    loss, logtemp, loss_params = [np.nan] * 11, np.nan, [np.nan] * 4
    while cum_steps < n_cum:
        start_time = time.perf_counter()
        state = env.reset()
        done, step, score = False, 0, 0
        end_time = start_time
        risk = None
        while not done:
            if cum_steps >= warmup:
                action = agent.select_next_action(state)
            else:
                action = env.action_space.sample()
                action = action if gbm else np.abs(action)
            if cum_steps <= window:
                action = action_window(action, inputs["max_action"], inputs["min_action"], cum_steps, window, warmup)
            next_state, reward, env_done, risk = env.step(action)
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
                loss[6:8] = agent_shadow_mean(inputs, loss)
                eval_multiplicative(n_gambles, agent, inputs, eval_log, eval_risk_log, mstep, cum_steps, rnd,
                                    eval_run, loss, logtemp, loss_params)
                eval_run += 1
            if cum_steps >= n_cum:
                break
        loss = list(loss)
        loss[6:8] = agent_shadow_mean(inputs, loss)
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
        if log is not None and (episode % 100 == 0 or cum_steps >= n_cum):
            log(f"E{inputs['ENV_KEY']}_m{mstep}_n{n_gambles} {inputs['algo']}-{inputs['s_dist']}-{inputs['loss_fn']}-"
                f"{rnd + 1} ep {episode} cst/st {cum_steps}/{step}: l% {100 * float(np.ravel(risk)[3]):1.0f}, "
                f"g% {100 * (reward - 1):1.1f}, C {np.nanmean(loss[0:2]):1.2f}")
        episode += 1
    return rows
