"""The market path of the reference's host entry points (GPU).

1. The reference-API single env: ``Market_Inv?_{D1,Dx}(n_assets, time_length,
   obs_days)`` with ``reset(assets)`` / ``step(action, next_assets)`` handed the
   observations of observed_market_state, on the device kernel, against the
   reference's own episodes (tests/golden/market_env.npz, stooq_usei, 3
   assets): rtol 1e-12.
2. F6-market (tests/golden/market_trace.npz, make_golden.market_trace): the
   reference's own scripts/rl_market.market_env (SNP_InvB on stooq_snp, TD3,
   HUB, obs_days 1 and 5, 2,500 steps: warm-up, smoothing window, policy)
   recorded step by step, replayed through rlmd_amd.scripts.rl_market with
     * each episode's start row and shuffled extract handed back where the
       driver calls time_slice / shuffle_data (the reference's np.random
       stream is not reproduced),
     * the warm-up samples replayed from env.action_space.sample,
     * an agent that returns the reference's policy outputs and learn() values,
     * eval_market replaced by a recorder of its arguments,
   so everything in between is the build's: the raw warm-up actions, the f64
   action window, the observations, the device env step, the episode
   bookkeeping, the shadow means of loss[6:8] (device), the trailing-score
   checkpoints and the trial logs.  Tolerances as in test_c1_driver_gpu.
3. The live loop: a real device Agent_td3, eval_market on the device, main.run
   dispatching market key 21 from a price directory.
"""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.mark.parametrize("name", [f"Market_Inv{i}_{d}" for i in "ABC" for d in ("D1", "Dx")])
def test_reference_api_market_env_matches_reference_episode(golden, dev, name):
    from rlmd_amd import envs
    from rlmd_amd.env_resources import observed_market_state

    g = golden("market_env.npz")
    ext, d, tl = g[name + "/extract"], int(g[name + "/obs_days"]), int(g[name + "/time_length"])
    env = envs.ENV_CLASSES[name](ext.shape[1], tl, d, device=dev, seed=1)
    state = env.reset(observed_market_state(ext, 0, 1, d))
    acts = g[name + "/actions"]
    for t in range(acts.shape[0]):
        np.testing.assert_allclose(state, g[name + "/state"][t], rtol=RTOL)
        ns, r, dn, risk = env.step(acts[t], observed_market_state(ext, t + 1, 1, d))
        np.testing.assert_allclose(ns, g[name + "/next_state"][t], rtol=RTOL)
        np.testing.assert_allclose(r, g[name + "/reward"][t], rtol=RTOL)
        assert dn == list(g[name + "/done"][t])
        np.testing.assert_allclose(risk, g[name + "/risk"][t], rtol=RTOL, equal_nan=True)
        if t > 0:
            assert ns is state  # one next_state array, overwritten in place (market_envs.py:111, 202)
        state = ns
    assert dn[0]  # the episode ends where the reference's did
    with pytest.raises(ValueError):
        env.step(acts[0], np.zeros(ext.shape[1] * d + 1))


def _mkt_inputs(f, **kw):
    from rlmd_amd.config import INPUTS, input_initialisation

    n_steps, _, key, _, train_days = (int(x) for x in f["params"])
    algo, loss_fn = (str(x) for x in f["spec"])
    inputs = dict(INPUTS)
    inputs.update({"n_trials_mkt": 1, "n_cumsteps_mkt": float(n_steps), "eval_freq_mkt": 1e3, "n_eval_mkt": 4,
                   "train_days": float(train_days)})
    inputs.update(kw)
    inputs = input_initialisation(inputs, [key], [algo], [loss_fn], [1])
    inputs["test_agent"] = True
    inputs["ENV_KEY"] = key
    return inputs


class _ReplayMarket:
    """The build's reference-API market env with the reference run's warm-up
    samples replayed; records what the driver hands it."""

    def __init__(self, f, dev, train_length, obs_days):
        from rlmd_amd.envs import ENV_CLASSES

        self._env = ENV_CLASSES["Market_InvB_" + ("D1" if obs_days == 1 else "Dx")](1, train_length, obs_days,
                                                                                   device=dev, seed=0)
        self.observation_space, self.reward_range = self._env.observation_space, self._env.reward_range
        self.f, self.t, self.seen, self.obs, self.resets = f, 0, [], [], []
        env = self

        class _Space:
            shape, high, low = self._env.action_space.shape, self._env.action_space.high, self._env.action_space.low

            def sample(self_inner):
                return env.f["action"][env.t].astype(np.float64)

        self.action_space = _Space()

    def reset(self, assets):
        self.resets.append(np.asarray(assets, np.float64).copy())
        return self._env.reset(assets)

    def step(self, action, next_assets):
        self.seen.append(np.asarray(action).copy())
        self.obs.append(np.asarray(next_assets, np.float64).copy())
        self.t += 1
        return self._env.step(action, next_assets)


class _ScriptedAgent:
    def __init__(self, f, env):
        self.f, self.env = f, env
        self.i_pol = self.i_learn = 0
        self.saves, self.stored = [], []

    def select_next_action(self, state):
        a = self.f["policy"][self.i_pol].astype(np.float32)
        self.i_pol += 1
        return a

    def store_transistion(self, s, a, r, s2, d):
        # copied at call time (replay.py:164-167)
        self.stored.append((np.asarray(s, np.float64).copy(), float(r), bool(d), np.asarray(s2, np.float64).copy()))

    def learn(self):
        i = self.i_learn
        self.i_learn += 1
        return list(self.f["learn_loss"][i]), self.f["learn_logtemp"][i], list(self.f["learn_params"][i])

    def save_models(self):
        self.saves.append(len(self.stored))


@pytest.mark.parametrize("obs_days", [1, 5])
def test_market_driver_replays_reference_loop(golden, dev, tmp_path, monkeypatch, obs_days):
    from rlmd_amd import env_resources, eval_episodes
    from rlmd_amd.config import GYM_ENVS
    from rlmd_amd.scripts import rl_market

    z = golden("market_trace.npz")
    f = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(f"d{obs_days}/")}
    n = int(f["params"][0])
    monkeypatch.chdir(tmp_path)
    inputs = _mkt_inputs(f)
    train_length = int(inputs["train_days"]) + obs_days - 1
    test_length = int(inputs["test_days"]) + obs_days - 1
    sample_length = train_length + test_length + obs_days + int(inputs["gap_days_max"]) - 1  # rl_market.py:58-60
    prices = golden("stooq_snp.npz")["prices"]
    ep = {"i": 0}
    slices = []

    def time_slice(p, extract_days, action_days, sample_days):
        slices.append((p is prices or np.array_equal(p, prices), extract_days, action_days, sample_days))
        return None, int(f["start_idx"][ep["i"]])

    def shuffle_data(sl, interval_days):
        assert interval_days == int(inputs["train_shuffle_days"])
        e = f["extract"][ep["i"]]
        ep["i"] += 1
        return e

    evals = []

    def eval_market(md, od, start, agent, inp, eval_log, eval_risk_log, mstep, cum_steps, rnd, eval_run, loss,
                    logtemp, params):
        evals.append((od, start, cum_steps, eval_run, np.asarray(loss, np.float64), float(logtemp),
                      np.asarray(params, np.float64)))

    monkeypatch.setattr(env_resources, "time_slice", time_slice)
    monkeypatch.setattr(env_resources, "shuffle_data", shuffle_data)
    monkeypatch.setattr(eval_episodes, "eval_market", eval_market)
    env = _ReplayMarket(f, dev, train_length, obs_days)
    holder = {}

    def factory(inp):
        holder["agent"] = _ScriptedAgent(f, env)
        return holder["agent"]

    (directory, trial, _, trial_risk, _), = rl_market.market_env(GYM_ENVS, inputs, prices, obs_days, env=env,
                                                                 agent_factory=factory, log=None)
    ag = holder["agent"]
    assert env.t == n and len(ag.stored) == n
    assert ep["i"] == len(f["start_idx"]) and all(s == (True, train_length, 1, sample_length) for s in slices)
    # first observations, per-step observations and actions as the reference handed them over
    np.testing.assert_array_equal(np.stack(env.resets), f["reset_obs"])
    np.testing.assert_array_equal(np.stack(env.obs), f["obs"])
    seen = np.stack([np.asarray(a, np.float64).reshape(-1) for a in env.seen])
    np.testing.assert_array_equal(seen, f["action"])  # raw warm-up samples, f64 window, f32 policy
    np.testing.assert_array_equal(np.array([np.asarray(a).dtype == np.float64 for a in env.seen]), f["action_dtype"])
    # the device env's outputs
    # what store_transistion received: the market env mutates one next_state array
    # (market_envs.py:111, 172-174, 202) and rl_market.py:240-273 stores state after
    # state = next_state, so from an episode's second step the stored state is the
    # post-step state; the facade's in-place buffer reproduces it
    st = np.stack([s for s, _, _, _ in ag.stored])
    np.testing.assert_allclose(st, f["stored_state"], rtol=RTOL, atol=0)
    np.testing.assert_allclose(np.stack([s2 for _, _, _, s2 in ag.stored]), f["stored_next_state"], rtol=RTOL, atol=0)
    assert np.all(f["stored_state"] == f["stored_next_state"], 1).sum() > n // 2
    np.testing.assert_allclose(np.array([r for _, r, _, _ in ag.stored]), f["reward"], rtol=RTOL, atol=0)
    np.testing.assert_array_equal(np.array([d for _, _, d, _ in ag.stored]), f["done"][:, 1])
    assert ag.i_learn == len(f["learn_loss"]) and ag.i_pol == len(f["policy"])
    assert ag.saves == f["save_step"].tolist()
    # evaluations: from start_idx + step, at the reference's cum_steps, shadow means filled on the device
    assert [e[1] for e in evals] == f["eval_start_idx"].tolist()
    assert [e[2] for e in evals] == f["eval_cum_steps"].tolist() and [e[3] for e in evals] == list(range(len(evals)))
    for e, rl, rp in zip(evals, f["eval_loss"], f["eval_params"]):
        keep = [c for c in range(11) if c not in (6, 7)]
        np.testing.assert_array_equal(e[4][keep], rl[keep])
        np.testing.assert_array_equal(np.isnan(e[4][6:8]), np.isnan(rl[6:8]))
        np.testing.assert_allclose(e[4][6:8][~np.isnan(rl[6:8])], rl[6:8][~np.isnan(rl[6:8])], rtol=2e-6)
        np.testing.assert_array_equal(e[6], rp)
    # trial logs: score / steps / loss columns as float32 (shadow means 2e-6), logtemp
    # and risk as test_c1_driver_gpu explains (the reference's CPU aliases)
    ref, ref_risk = f["trial"], f["trial_risk"]
    assert trial.shape == ref.shape and trial_risk.shape == ref_risk.shape
    cols = [1, 2] + [c for c in range(3, 19) if c not in (9, 10, 14)]
    np.testing.assert_array_equal(trial[0, :, cols], ref[0, :, cols])
    sh, rs = trial[0, :, 9:11].astype(np.float64), ref[0, :, 9:11].astype(np.float64)
    np.testing.assert_array_equal(np.isnan(sh), np.isnan(rs))
    np.testing.assert_allclose(sh[~np.isnan(sh)], rs[~np.isnan(rs)], rtol=2e-6)
    np.testing.assert_array_equal(np.isnan(trial[0, :, 14]), np.isnan(ref[0, :, 14]))
    ends = np.cumsum(ref[0, :, 2]).astype(np.int64) - 1
    np.testing.assert_allclose(trial_risk[0], f["risk"][ends].astype(np.float32), rtol=1e-6, atol=0, equal_nan=True)
    assert directory.startswith(f"./results/test_market/data/SNP_InvB_D{obs_days}_T1/")
    for suffix in ("_trial.npy", "_eval.npy", "_trial_risk.npy", "_eval_risk.npy"):
        assert os.path.exists(directory + suffix)


def test_market_driver_live_td3_through_main(golden, dev, tmp_path, monkeypatch):
    """main.run on market key 21 (SNP_InvA) with past_days [1, 3]: the price
    table from inputs['market_dir'], a real device Agent_td3, eval_market on the
    device every 1e3 steps (gaps 5..20 past start_idx + step, test slices
    shuffled in blocks of 3), NaN placeholders until the buffer exceeds B, the
    four log files per obs_days."""
    from rlmd_amd.config import INPUTS
    from rlmd_amd.main import run

    monkeypatch.chdir(tmp_path)
    mdir = tmp_path / "market_data"
    mdir.mkdir()
    np.save(mdir / "stooq_snp.npy", golden("stooq_snp.npz")["prices"])
    np.random.seed(5)
    inputs = dict(INPUTS, n_trials_mkt=1, n_cumsteps_mkt=2000, n_eval_mkt=16, train_days=150, past_days=[1, 3],
                  market_dir="./market_data/", test_agent=True)  # relative, as learning_tests requires
    out = run([21], ["TD3"], ["MSE"], [1], inputs=inputs, log=None)
    assert len(out[21]) == 2
    for d, ((directory, trial, ev, trial_risk, ev_risk),) in zip((1, 3), out[21]):
        assert directory.startswith(f"./results/test_market/data/SNP_InvA_D{d}_T1/")
        n_ep = int((trial[0, :, 0] != 0).sum())
        assert trial[0, :n_ep, 2].sum() == 2000
        early = np.cumsum(trial[0, :n_ep, 2]) <= 200  # before the first real TD3 update (B = 200)
        assert np.all(np.isnan(trial[0, :n_ep][early, 3])) and np.all(np.isfinite(trial[0, :n_ep][~early, 3]))
        assert ev.shape == (1, 2, 16, 20) and ev_risk.shape == (1, 2, 16, 5)
        assert np.all(ev[0, :, :, 19] == np.array([1000, 2000])[:, None])
        assert np.all((ev[0, :, :, 2] >= 1) & (ev[0, :, :, 2] <= 250)) and np.isfinite(ev[0, :, :, 1]).all()
        gaps = ev_risk[0, :, :, 0]
        assert np.all(gaps >= 5) and np.all(gaps == np.round(gaps))
        for suffix in ("_trial.npy", "_eval.npy", "_trial_risk.npy", "_eval_risk.npy"):
            assert os.path.exists(directory + suffix)
    assert glob.glob("results/test_market/models/SNP_InvA_D1_T1/*_actor.pt")
