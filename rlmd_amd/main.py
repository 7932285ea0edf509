"""Entry point with main.py's shape (main.py:262-330): pick env keys, algorithms,
critic losses and multi-step counts, fold them into the inputs dict and run the
matching driver per key.

    python -m rlmd_amd.main --envs 8 --algo SAC --critic MSE --steps 50000 --trials 1

Multiplicative keys (8-16, over n_gambles) and the safe-haven keys (17-20)
run rlmd_amd.scripts.rl_multiplicative.multiplicative_env (one env stream,
the reference's schedule, learner on the device).  The vectorised loop of the
same envs (tens of thousands of lanes per launch) is rlmd_amd.experiment /
bench.py.
"""
import argparse
import time

from .config import GYM_ENVS, INPUTS, env_dynamics, input_initialisation


def run(envs, algo=("SAC",), critic=("MSE",), multi_steps=(1,), inputs=None, gym_envs=None, log=print):
    gym_envs = gym_envs or GYM_ENVS
    inputs = input_initialisation(dict(inputs or INPUTS), list(envs), list(algo), list(critic), list(multi_steps))
    multi_key, sh_key, market_key = env_dynamics(gym_envs)
    from .scripts.rl_multiplicative import multiplicative_env

    out = {}
    for key in envs:
        t0 = time.perf_counter()
        inputs["ENV_KEY"] = key
        if multi_key <= key < sh_key:
            out[key] = [multiplicative_env(gym_envs, inputs, n_gambles=g, log=log) for g in inputs["n_gambles"]]
        elif sh_key <= key < market_key:
            out[key] = [multiplicative_env(gym_envs, inputs, n_gambles=1, log=log)]
        else:
            raise NotImplementedError(f"ENV_KEY {key}: only the multiplicative keys {multi_key}-{market_key - 1} "
                                      "have a single-stream driver; market envs run vectorised (rlmd_amd.experiment)")
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
    ap.add_argument("--test-agent", action="store_true")
    a = ap.parse_args()
    inputs = dict(INPUTS, n_cumsteps_mul=a.steps, n_trials_mul=a.trials)
    if a.test_agent:
        inputs["test_agent"] = True
    run(a.envs, a.algo, a.critic, a.multi_steps, inputs=inputs)


if __name__ == "__main__":
    main()
