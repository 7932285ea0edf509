"""Entry point with main.py's shape (main.py:262-330): pick env keys, algorithms,
critic losses and multi-step counts, fold them into the inputs dict and run the
matching driver per key.

    python -m rlmd_amd.main --envs 8 --algo SAC --critic MSE --steps 50000 --trials 1

Multiplicative keys (8-16, over n_gambles) and the safe-haven keys (17-20)
run rlmd_amd.scripts.rl_multiplicative.multiplicative_env; the market keys
(21-26) load their price table (load_market_data) and run
rlmd_amd.scripts.rl_market.market_env once per inputs["past_days"] entry
(main.py:322-327).  Each is one env stream with the reference's schedule and
the learner on the device.  The vectorised loop of the same envs (tens of
thousands of lanes per launch) is rlmd_amd.experiment / bench.py.
"""
import argparse
import os
import time

import numpy as np

from .config import GYM_ENVS, INPUTS, env_dynamics, env_tests, input_initialisation, learning_tests

MARKET_FILES = ["stooq_snp.npy", "stooq_usei.npy", "stooq_minor.npy", "stooq_medium.npy", "stooq_major.npy",
                "stooq_dji.npy", "stooq_full.npy"]


def market_env_keys(gym_envs):
    """tools/utils.py:134-135: the last key (the _InvC row) of each market."""
    market_key = env_dynamics(gym_envs)[2]
    return [k for k in (int(k) for k, v in gym_envs.items() if v[0][-5:] == "_InvC") if k >= market_key]


def load_market_data(key, gym_envs, inputs):
    """tools/utils.py:140-167: inputs["market_dir"] + the key's stooq_*.npy
    (plain array files, loaded without pickle)."""
    for last, name in zip(market_env_keys(gym_envs), MARKET_FILES):
        if key <= last:
            path = os.path.join(inputs["market_dir"], name)
            if not os.path.exists(path):
                raise FileNotFoundError(f"{path}: the reference's tools/market_data/{name} (set inputs['market_dir'])")
            return np.load(path, allow_pickle=False)
    raise KeyError(f"ENV_KEY {key} is past the market keys")


def run(envs, algo=("SAC",), critic=("MSE",), multi_steps=(1,), inputs=None, gym_envs=None, log=print):
    gym_envs = gym_envs or GYM_ENVS
    inputs = input_initialisation(dict(inputs or INPUTS), list(envs), list(algo), list(critic), list(multi_steps))
    # main.py:277-280: the input checks before any run (AssertionError on bad inputs)
    learning_tests(inputs)
    env_tests(gym_envs, inputs)
    multi_key, sh_key, market_key = env_dynamics(gym_envs)
    from .scripts.rl_market import market_env
    from .scripts.rl_multiplicative import multiplicative_env

    out = {}
    for key in envs:
        t0 = time.perf_counter()
        inputs["ENV_KEY"] = key
        if multi_key <= key < sh_key:
            out[key] = [multiplicative_env(gym_envs, inputs, n_gambles=g, log=log) for g in inputs["n_gambles"]]
        elif sh_key <= key < market_key:
            out[key] = [multiplicative_env(gym_envs, inputs, n_gambles=1, log=log)]
        elif market_key <= key <= market_env_keys(gym_envs)[-1]:
            data = load_market_data(key, gym_envs, inputs)
            out[key] = [market_env(gym_envs, inputs, market_data=data, obs_days=d, log=log)
                        for d in inputs["past_days"]]
        else:
            raise NotImplementedError(f"ENV_KEY {key}: not one of the keys {multi_key}-"
                                      f"{market_env_keys(gym_envs)[-1]} this build runs")
        if log is not None:
            log(f"ENV_KEY {key} done in {time.perf_counter() - t0:1.0f} s")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[8])
    ap.add_argument("--algo", nargs="+", default=["SAC"])
    ap.add_argument("--critic", nargs="+", default=["MSE"])
    ap.add_argument("--multi-steps", type=int, nargs="+", default=[1])
    ap.add_argument("--steps", type=float, default=INPUTS["n_cumsteps_mul"])
    ap.add_argument("--trials", type=int, default=INPUTS["n_trials_mul"])
    ap.add_argument("--past-days", type=int, nargs="+", default=INPUTS["past_days"])
    ap.add_argument("--market-dir", default=INPUTS["market_dir"])
    ap.add_argument("--test-agent", action="store_true")
    a = ap.parse_args()
    inputs = dict(INPUTS, n_cumsteps_mul=a.steps, n_trials_mul=a.trials, n_cumsteps_mkt=a.steps,
                  n_trials_mkt=a.trials, past_days=a.past_days, market_dir=a.market_dir)
    if a.test_agent:
        inputs["test_agent"] = True
    run(a.envs, a.algo, a.critic, a.multi_steps, inputs=inputs)


if __name__ == "__main__":
    main()
