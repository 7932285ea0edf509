"""Config C1 through the reference-named facade (GPU).

F6 (tests/golden/c1_trace.npz, make_golden.c1_trace) is the reference's own
scripts/rl_multiplicative.py loop (Coin_InvA, SAC, MSE, 2,500 steps: warm-up,
smoothing window and policy phases), recorded step by step, including what
store_transistion received (the aliased post-step state from an episode's
second step); F6-GBM (c1_gbm_trace.npz) is the same on GBM_InvA (key 14, C2's
env).  The replay test drives rlmd_amd.scripts.rl_multiplicative with
  * an env that is the device Coin_InvA / GBM_InvA fed the reference's draws, and
  * an agent that returns the reference's own policy outputs and learn() values,
so everything in between is the build's: the warm-up |sample| rule, the
float64 action window, the env step on the device, the episode bookkeeping,
the shadow means of loss[6:8] (device), the trailing-50 checkpoint schedule
and the trial logs.  Tolerances: env outputs rtol 1e-12 (f64 env path), actions
bit-exact (the window is f64 host arithmetic), trial log score / steps / loss
columns equal as float32 except the shadow-mean columns (rtol 2e-6, the f32
gamma-function restatement; NaN positions exact).

The live test runs the driver with the real device Agent_sac.
"""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _c1_inputs(n_steps, n_trials=1, key=8, **kw):
    from rlmd_amd.config import INPUTS, input_initialisation

    inputs = dict(INPUTS)
    inputs.update({"n_trials_mul": n_trials, "n_cumsteps_mul": float(n_steps)})
    inputs.update(kw)
    inputs = input_initialisation(inputs, [key], ["SAC"], ["MSE"], [1])
    inputs["test_agent"] = True
    inputs["ENV_KEY"] = key
    return inputs


class _ReplayEnv:
    """The device env of the trace (Coin_InvA / GBM_InvA) with the reference's
    draws injected in order and its warm-up samples replayed.  Steps go through
    the facade's own step (``_step`` with injected draws), so the driver gets
    the facade's in-place next_state buffer, as it would from env.step."""

    def __init__(self, f, dev, name):
        from rlmd_amd.envs import ENV_CLASSES

        self._env = ENV_CLASSES[name](1, device=dev, seed=0)
        self.observation_space = self._env.observation_space
        self.reward_range = self._env.reward_range
        self.f = f
        self.t = 0
        self.seen = []
        env = self

        class _Space:
            shape = self._env.action_space.shape
            high = self._env.action_space.high
            low = self._env.action_space.low

            def sample(self_inner):
                return env.f["action"][env.t].astype(np.float64)

        self.action_space = _Space()

    def reset(self):
        return self._env.reset()

    def step(self, action):
        a = np.asarray(action)
        self.seen.append(a.copy())
        draw = torch.tensor(self.f["draw"][self.t].reshape(1, -1), dtype=torch.float64)
        self.t += 1
        return self._env._step(a, draw)


class _ScriptedAgent:
    """Returns the reference run's policy outputs and learn() values in order."""

    def __init__(self, f, dev, inputs):
        self.f, self.inputs = f, inputs
        self.i_pol = self.i_learn = self.n_store = 0
        self.saves, self.stored = [], []
        agent = self

        class _Dev:
            device = dev

            def act(self_inner, obs, mode=1):
                a = agent.f["policy"][max(agent.i_pol - 1, 0)].astype(np.float32)
                return torch.as_tensor(np.tile(a, (obs.shape[0], 1)), device=dev)

        self.dev = _Dev()

    def select_next_action(self, state):
        a = self.f["policy"][self.i_pol].astype(np.float32)
        self.i_pol += 1
        return a

    def store_transistion(self, s, a, r, s2, d):
        # copied at call time, as the reference's ReplayBuffer.store_exp does (replay.py:164-167)
        self.stored.append((np.asarray(s, np.float64).copy(), float(r), bool(d), np.asarray(s2, np.float64).copy()))
        self.n_store += 1

    def learn(self):
        i = self.i_learn
        self.i_learn += 1
        return list(self.f["learn_loss"][i]), self.f["learn_logtemp"][i], list(self.f["learn_params"][i])

    def save_models(self):
        self.saves.append(self.n_store)


@pytest.mark.parametrize("fixture", ["c1_trace.npz", "c1_gbm_trace.npz"])
def test_c1_driver_replays_reference_loop(golden, dev, tmp_path, monkeypatch, fixture):
    """F6 (Coin_InvA, key 8) and F6-GBM (GBM_InvA, key 14, C2's env)."""
    from rlmd_amd.config import GYM_ENVS
    from rlmd_amd.scripts.rl_multiplicative import multiplicative_env

    f = golden(fixture)
    n = int(f["n_steps"])
    key = int(f["key"])
    name = GYM_ENVS[str(key)][0]
    monkeypatch.chdir(tmp_path)
    env = _ReplayEnv(f, dev, name)
    holder = {}

    def factory(inputs):
        holder["agent"] = _ScriptedAgent(f, dev, inputs)
        return holder["agent"]

    inputs = _c1_inputs(n, n_eval_mul=16, key=key)
    (directory, trial, _, trial_risk, _), = multiplicative_env(GYM_ENVS, inputs, 1, env=env, agent_factory=factory,
                                                               log=None)
    ag = holder["agent"]
    assert env.t == n and ag.n_store == n
    seen = np.stack([np.asarray(a, np.float64).reshape(-1) for a in env.seen])
    np.testing.assert_array_equal(seen, f["action"].reshape(n, -1))  # warm-up |sample|, f64 window, policy
    np.testing.assert_array_equal(np.array([np.asarray(a).dtype == np.float64 for a in env.seen]), f["action_dtype"])
    # what store_transistion received: the reference's env mutates one next_state
    # array and its loop stores state after state = next_state, so from an
    # episode's second step the stored state IS the post-step state
    # (rl_multiplicative.py:213-245, gbm_envs.py:184-186); the facade's in-place
    # buffer reproduces it through the build's driver
    st = np.stack([s for s, _, _, _ in ag.stored])
    np.testing.assert_allclose(st, f["stored_state"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(np.stack([s2 for _, _, _, s2 in ag.stored]), f["stored_next_state"], rtol=1e-12, atol=0)
    aliased = np.all(f["stored_state"] == f["stored_next_state"], 1)
    assert aliased.sum() > n // 2 and not np.array_equal(f["stored_state"], f["state"])  # the fixture shows it
    np.testing.assert_allclose(np.array([r for _, r, _, _ in ag.stored]), f["reward"], rtol=1e-12, atol=0)
    np.testing.assert_array_equal(np.array([d for _, _, d, _ in ag.stored]), f["done"][:, 1])
    assert ag.i_learn == len(f["learn_loss"])
    assert ag.saves == f["save_step"].tolist()
    ref, ref_risk = f["trial"], f["trial_risk"]
    assert trial.shape == ref.shape and trial_risk.shape == ref_risk.shape
    cols = [1, 2] + [c for c in range(3, 19) if c not in (9, 10, 14)]
    np.testing.assert_array_equal(trial[0, :, cols], ref[0, :, cols])
    # logtemp (col 14): learn() returns log_alpha.detach().cpu().numpy() (algo_sac.py:
    # 394, 500, 589), which on a CPU device is a VIEW of the parameter, so the
    # reference's CPU log holds the final log temperature in every row (our fixture
    # run); on its default cuda device it is a copy, one value per episode.  The
    # build logs per-episode values: the last learn() of each episode.
    ends = np.cumsum(ref[0, :, 2]).astype(np.int64) - 1
    np.testing.assert_array_equal(trial[0, :, 14], f["learn_logtemp"][ends].astype(np.float32))
    assert np.all(ref[0, :, 14] == np.float32(f["learn_logtemp"][-1]))
    sh, rs = trial[0, :, 9:11].astype(np.float64), ref[0, :, 9:11].astype(np.float64)
    np.testing.assert_array_equal(np.isnan(sh), np.isnan(rs))
    np.testing.assert_allclose(sh[~np.isnan(sh)], rs[~np.isnan(rs)], rtol=2e-6)
    # risk rows: the reference appends env.step's risk array, one buffer the env
    # reuses (self.risk, coin_flip_envs.py:209-212), so every row of its saved
    # trial_risk log is the LAST step's risk vector; the build logs each episode's
    # own final risk vector, the values the reference's rows held when appended
    np.testing.assert_allclose(trial_risk[0], f["risk"][ends].astype(np.float32), rtol=1e-6, atol=0)
    assert np.all(ref_risk[0] == f["risk"][-1].astype(np.float32))
    assert directory.startswith(f"./results/test_multiplicative/data/{name}_n1/")
    for suffix in ("_trial.npy", "_eval.npy", "_trial_risk.npy", "_eval_risk.npy"):
        assert os.path.exists(directory + suffix)


def test_c1_driver_live_sac_and_continue(dev, tmp_path, monkeypatch):
    """The C1 loop with the real device Agent_sac: 2 trials with `continue`
    (the second loads the first's checkpoints and log temperature), evaluation
    at every 1e3 steps, NaN-placeholder learn() until mem_idx > B, then finite
    critic statistics (the NaN guard would raise)."""
    from rlmd_amd.config import GYM_ENVS
    from rlmd_amd.scripts.rl_multiplicative import multiplicative_env

    monkeypatch.chdir(tmp_path)
    np.random.seed(3)
    inputs = _c1_inputs(2000, n_trials=2, n_eval_mul=20, **{"continue": True})
    (directory, trial, ev, trial_risk, ev_risk), = multiplicative_env(GYM_ENVS, inputs, 1, log=None)
    assert trial.shape[0] == 2 and trial.shape[2] == 19 and trial_risk.shape[2] == 4
    assert ev.shape == (2, 2, 20, 20) and ev_risk.shape == (2, 2, 20, 4)
    for t in range(2):
        steps = trial[t, :, 2]
        n_ep = int((trial[t, :, 0] != 0).sum())
        assert steps[:n_ep].sum() == 2000
        cum = np.cumsum(steps[:n_ep])
        early = cum <= 512  # episodes that ended before the first real update
        assert np.all(np.isnan(trial[t, :n_ep][early, 3])) and np.all(np.isfinite(trial[t, :n_ep][~early, 3]))
        assert np.all(ev[t, :, :, 19] == np.array([1000, 2000])[:, None])
        assert np.all(np.isfinite(ev[t, :, :, 1])) and np.all(ev[t, :, :, 2] >= 1)
    ckpt = glob.glob("results/test_multiplicative/models/Coin_InvA_n1/*_actor.pt")
    assert ckpt, "no trailing-score checkpoint written"
    for p in ckpt:
        sd = torch.load(p, weights_only=True)
        assert set(sd) == {"fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "pi.weight", "pi.bias",
                           "log_scale.weight", "log_scale.bias"}


def test_agent_save_load_round_trip(dev, tmp_path):
    """save_models / load_models (algo_sac.py:617-632): torch state dicts with the
    reference's layer names, read back with weights_only=True into a fresh agent,
    which then acts identically."""
    from rlmd_amd.agent import Agent_sac, Agent_td3
    from rlmd_amd.config import INPUTS

    for cls, algo in ((Agent_sac, "SAC"), (Agent_td3, "TD3")):
        inputs = dict(INPUTS, input_dims=(5,), num_actions=1, max_action=0.99, algo=algo, loss_fn="MSE",
                      mini_batch_size=64, s_dist="N", n_cumsteps=1000, actor_percentile=50, critic_percentile=50)
        inputs["batch_size"] = {"SAC": 32, "TD3": 32}
        a1, a2 = cls(inputs), cls(inputs)
        a1.file_prefix = a2.file_prefix = str(tmp_path / f"model_{algo}")
        a1.save_models()
        for net in ("actor", "critic_1", "critic_2"):
            sd = torch.load(f"{a1.file_prefix}_{net}.pt", weights_only=True)
            assert all(v.dtype == torch.float32 and v.device.type == "cpu" for v in sd.values())
        a2.load_models()
        for net in ("actor", "critic_1", "critic_2"):
            for (k1, v1), (k2, v2) in zip(a1.dev.state_dict(net).items(), a2.dev.state_dict(net).items()):
                assert k1 == k2
                assert torch.equal(v1, v2)
        s = np.full(5, 1e-14)
        np.testing.assert_array_equal(a1.eval_next_action(s), a2.eval_next_action(s))
