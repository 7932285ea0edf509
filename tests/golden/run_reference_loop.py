"""Run the reference's own multiplicative training loop (config C1 shape) on CPU
and keep its evaluation curve as a fixture: the calibration of what the
reference *converges to* on Coin / Dice / Dice_SH_INSURED, against which
tests/test_converge_gpu.py holds the vectorised MI355X loop.

Build container only (imports /root/reference through the §8c shims of
_refshim.py; the reference never travels).  Calls
scripts/rl_multiplicative.multiplicative_env (rl_multiplicative.py:41-457)
with main.py's gym_envs table and inputs dict (main.py:41-259) widened by
utils.input_initialisation (tools/utils.py:80-106), one trial, SAC, MSE,
seeded np.random + torch, with --algo (SAC | TD3), --loss (any of
main.py:137's critic losses) and --multi-steps (n-step returns, C5).  From the saved logs it keeps, per evaluation
(every eval_freq = 1e3 steps, 100 episodes of <= 100 steps at one constant
deterministic action): the mean leverage (eval_risk_log[..., 3],
eval_episodes.py:296-297), the final rewards (eval_log[..., 1]) and the whole
eval risk row (for Dice_SH_InvA column 6 is the safe-haven leverage,
dice_roll_sh_envs.py:355-362).

    python tests/golden/run_reference_loop.py --key 8 --steps 50000 --seed 0
writes tests/golden/converge_ref_<key>_s<seed>.npz (SAC / MSE) or
tests/golden/converge_ref_<key>_<algo>_<loss>[_n<multi_steps>]_s<seed>.npz otherwise.
"""
import argparse
import glob
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refshim  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", type=int, default=8, help="main.py gym_envs key (8 Coin_InvA, 11 Dice_InvA, "
                                                     "17 Dice_SH_INSURED)")
    ap.add_argument("--steps", type=int, default=50000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--algo", default="SAC", choices=["SAC", "TD3"])
    ap.add_argument("--loss", default="MSE")
    ap.add_argument("--multi-steps", type=int, default=1, help="n-step returns (C5: 5)")
    ap.add_argument("--n-eval", type=int, default=0, help="evaluation episodes (0: main.py's)")
    ap.add_argument("--out", default="", help="output path (default: the fixture name under tests/golden)")
    a = ap.parse_args()
    market = 21 <= a.key <= 26
    _refshim.install()
    import torch

    torch.set_num_threads(a.threads)
    import main as ref_main  # noqa: E402  (module level only defines the tables)
    from tools import utils

    inputs = dict(ref_main.inputs)
    inputs.update({"n_trials_mul": 1, "n_cumsteps_mul": float(a.steps), "n_trials_mkt": 1,
                   "n_cumsteps_mkt": float(a.steps), "gpu": "cpu", "buffer_gpu": False})
    if a.n_eval:
        inputs.update({"n_eval_mul": float(a.n_eval), "n_eval_mkt": float(a.n_eval)})
    inputs = utils.input_initialisation(inputs, [a.key], [a.algo], [a.loss], [a.multi_steps])
    inputs["test_agent"] = True
    inputs["ENV_KEY"] = a.key
    import envs.dice_roll_sh_envs as sh_mod

    class _ArrayFix:
        """dice_roll_sh_envs' np with NumPy 1.22's array() of a list holding a
        size-1 ndarray (Dice_SH_INSURED risk list); np.random stays
        the real (seeded) generator."""

        def __getattr__(self, name):
            return getattr(np, name)

        def array(self, obj, *args, **kw):
            if isinstance(obj, list):
                obj = [o.reshape(()) if isinstance(o, np.ndarray) and o.size == 1 else o for o in obj]
            return np.array(obj, *args, **kw)

    sh_mod.np = _ArrayFix()
    tag = "" if (a.algo, a.loss) == ("SAC", "MSE") else f"_{a.algo}_{a.loss}"
    tag += f"_n{a.multi_steps}" if a.multi_steps != 1 else ""
    tag += f"_e{a.n_eval}" if a.n_eval else ""
    out = a.out or os.path.join(HERE, f"converge_ref_{a.key}{tag}_s{a.seed}.npz")
    np.random.seed(a.seed)
    torch.manual_seed(a.seed)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            if market:  # main.py:322-327 with the key's price file (SNP: stooq_snp, EI: stooq_usei)
                from scripts.rl_market import market_env

                name = "stooq_snp.npy" if a.key <= 23 else "stooq_usei.npy"
                data = np.load(os.path.join(_refshim.REF, "tools", "market_data", name), allow_pickle=False)
                market_env(ref_main.gym_envs, inputs, market_data=data, obs_days=1)
            else:
                from scripts.rl_multiplicative import multiplicative_env

                multiplicative_env(ref_main.gym_envs, inputs, n_gambles=1)
            ev = np.load(glob.glob("results/**/*_eval.npy", recursive=True)[0])
            er = np.load(glob.glob("results/**/*_eval_risk.npy", recursive=True)[0])
            # per training episode (rl_multiplicative.py:419-429): length, logtemp, last risk row
            tr = np.load(glob.glob("results/**/*_trial.npy", recursive=True)[0])
            trr = np.load(glob.glob("results/**/*_trial_risk.npy", recursive=True)[0])
        finally:
            os.chdir(cwd)
    np.savez_compressed(out, key=a.key, seed=a.seed, steps=a.steps, env=ref_main.gym_envs[str(a.key)][0],
                        cum_steps=ev[0, :, 0, 19], reward=ev[0, :, :, 1], eval_steps=ev[0, :, :, 2],
                        lev=er[0, :, :, 3], risk=er[0].astype(np.float32), algo=a.algo, loss=a.loss,
                        multi_steps=a.multi_steps, **({"trial_steps": tr[0, :, 2], "trial_logtemp": tr[0, :, 14],
                                                       "trial_lev": trr[0, :, 3]} if a.out else {}))
    print("wrote", out, "final mean lev", er[0, -5:, :, 3].mean(), "final mean reward", ev[0, -5:, :, 1].mean())


if __name__ == "__main__":
    main()
