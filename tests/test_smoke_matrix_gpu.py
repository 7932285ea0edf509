"""The reference's smoke matrix (tests/test_script_agent.py:190-322) through the
build's single-stream drivers, at reduced scale.

The reference runs keys [8, 13, 15] (n_gambles [1, 5]), [17, 19] and market
[21] (past_days [1, 5]) with SAC and TD3, critic losses MSE (+ HUB/MAE/HSC as
its TEST_CRITICS_EXTRA) and multi_steps [1, 5], and passes when every run
completes.  Here each key is one test that runs the whole algo x loss x
multi-step product inside one driver call (the drivers loop over them as the
reference's do: rl_multiplicative.py:154-183, rl_market.py:167-196), 600
steps per trial (the reference's 3e3, reduced), and checks per run:
  * the four log files and their shapes (trial [1, episodes, 19], eval
    [1, 2, n_eval, 20], risk widths of utils.multi_log_dim / market_log_dim);
  * the steps of the logged episodes add up to n_cumsteps;
  * NaN loss placeholders while the buffer holds <= B transitions
    (algo_sac.py:380-396) and finite critic statistics afterwards;
  * finite evaluation rewards with 1..max_eval_steps steps.
The per-step learner is the device agent (librlmd_amd.so) in every run.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALGOS = ["SAC", "TD3"]
LOSSES = ["MSE", "HUB", "MAE", "HSC"]
MSTEPS = [1, 5]
N_CUM, EVAL_FREQ, N_EVAL = 600, 300, 10
BATCH = {"SAC": 512, "TD3": 200}  # mini-batch sizes at the 50 % percentiles (rl_multiplicative.py:108-113)


def _inputs(tmp_path, **over):
    from rlmd_amd.config import INPUTS, input_initialisation

    inp = dict(INPUTS, n_trials_mul=1, n_cumsteps_mul=N_CUM, eval_freq_mul=EVAL_FREQ, n_eval_mul=N_EVAL,
               n_trials_mkt=1, n_cumsteps_mkt=N_CUM, eval_freq_mkt=EVAL_FREQ, n_eval_mkt=N_EVAL, **over)
    inp = input_initialisation(inp, [], ALGOS, LOSSES, MSTEPS)
    inp["test_agent"] = True
    return inp


def _check_runs(out, risk_width, max_eval_steps):
    assert len(out) == len(ALGOS) * len(LOSSES) * len(MSTEPS)
    for (directory, trial, ev, trial_risk, ev_risk), (algo, loss, ms) in zip(
            out, [(a, l, m) for a in ALGOS for l in LOSSES for m in MSTEPS]):
        tag = f"{algo}-{loss}-m{ms}"
        assert f"_{algo}-" in directory and f"_{loss}-" in directory and f"_M{ms}_" in directory, (tag, directory)
        for suffix in ("_trial.npy", "_eval.npy", "_trial_risk.npy", "_eval_risk.npy"):
            assert os.path.exists(directory + suffix), (tag, suffix)
        n_ep = int((trial[0, :, 0] != 0).sum())
        assert trial.shape[0] == 1 and trial.shape[2] == 19 and trial_risk.shape[2] == risk_width, (tag, trial.shape)
        assert ev.shape == (1, N_CUM // EVAL_FREQ, N_EVAL, 20), (tag, ev.shape)
        assert trial[0, :n_ep, 2].sum() == N_CUM, tag
        # placeholders while mem_idx <= B, learning afterwards: the critic
        # statistics loss[0:6] of each episode's last learn() call
        ends = np.cumsum(trial[0, :n_ep, 2])
        stats = trial[0, :n_ep, 3:9]
        early, late = ends <= BATCH[algo], ends > BATCH[algo]
        assert np.all(np.isnan(stats[early])), tag
        assert late.any() and np.all(np.isfinite(stats[late])), tag
        assert np.isfinite(ev[0, :, :, 1]).all() and np.all((ev[0, :, :, 2] >= 1) & (ev[0, :, :, 2] <= max_eval_steps)), tag
        assert np.all(ev[0, :, :, 19] == (np.arange(1, N_CUM // EVAL_FREQ + 1) * EVAL_FREQ)[:, None]), tag


@pytest.mark.parametrize("key,n_gambles", [(8, 1), (8, 5), (13, 1), (15, 1), (17, 1), (19, 1)])
def test_multiplicative_smoke_matrix(dev, tmp_path, monkeypatch, key, n_gambles):
    from rlmd_amd import logs
    from rlmd_amd.config import GYM_ENVS
    from rlmd_amd.scripts.rl_multiplicative import multiplicative_env

    monkeypatch.chdir(tmp_path)
    np.random.seed(key)
    inputs = _inputs(tmp_path)
    inputs["ENV_KEY"] = key
    out = multiplicative_env(GYM_ENVS, inputs, n_gambles=n_gambles, log=None)
    env_id = GYM_ENVS[str(key)][0] + "_n" + str(n_gambles)
    _check_runs(out, logs.multi_log_dim(env_id, n_gambles), int(inputs["max_eval_steps_mul"]))


@pytest.mark.parametrize("past_days", [1, 5])
def test_market_smoke_matrix(golden, dev, tmp_path, monkeypatch, past_days):
    from rlmd_amd import logs
    from rlmd_amd.config import GYM_ENVS
    from rlmd_amd.scripts.rl_market import market_env

    monkeypatch.chdir(tmp_path)
    np.random.seed(21 + past_days)
    data = golden("stooq_snp.npz")["prices"]
    inputs = _inputs(tmp_path)
    inputs["ENV_KEY"] = 21
    out = market_env(GYM_ENVS, inputs, market_data=data, obs_days=past_days, log=None)
    env_id = GYM_ENVS["21"][0] + f"_D{past_days}_T1"
    # market eval risk rows carry the start index in front (eval_episodes.py:542-543)
    _check_runs(out, logs.market_log_dim(env_id, data.shape[1]), int(inputs["test_days"]))
    for (_, _, _, _, ev_risk) in out:
        assert ev_risk.shape[-1] == logs.market_log_dim(env_id, data.shape[1]) + 1
