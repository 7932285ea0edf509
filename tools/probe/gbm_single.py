"""GBM_InvA (key 14, SAC / MSE) through the build's reference-API driver
(rlmd_amd.main.run -> the multiplicative loop of scripts/rl_multiplicative.py:
one env, one update per env step, the device Agent_sac), on main.py's settings
(5e4 steps, evaluations of 100 episodes every 1e3 steps), against the
reference's five seeds.  The control for the N = 1 / K = 1 vectorised result
(DESIGN.md §5a): if this driver lands in the reference's band and the
vectorised single lane does not, the difference is in the vectorised loop's
glue, not in the learner.

    RLMD_CONVERGE_LOG=gpurun_out/gbm_single.jsonl python tools/probe/gbm_single.py 0-4 [--steps=50000] [--prestep]
"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def one(seed, steps):
    import numpy as np
    import torch

    from rlmd_amd.config import INPUTS
    from rlmd_amd.main import run as main_run

    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            np.random.seed(seed)
            torch.manual_seed(seed)
            inputs = dict(INPUTS, n_trials_mul=1, n_cumsteps_mul=float(steps), test_agent=True)
            ((_, tr, ev, trr, ev_risk),), = main_run([14], ["SAC"], ["MSE"], [1], inputs=inputs, log=None)[14]
        finally:
            os.chdir(cwd)
    g = 100.0 * (ev[0, :, :, 1] - 1.0).mean(1)
    lev = ev_risk[0, :, :, 3].mean(1)
    return g, lev, trial_summary(tr[0, :, 2], tr[0, :, 14], trr[0, :, 3])


def trial_summary(steps, logtemp, lev, every=5000):
    """Per window of `every` training steps: episodes ended, their mean length,
    the last episode's logtemp and its last action's leverage (the trial logs of
    rl_multiplicative.py:419-429), for the build's driver and the reference's."""
    import numpy as np

    n = int(np.argmax(steps == 0)) if (steps == 0).any() else len(steps)
    steps, logtemp, lev = steps[:n], logtemp[:n], lev[:n]
    end = np.cumsum(steps)
    out = []
    for w0 in range(0, int(end[-1]), every):
        m = (end > w0) & (end <= w0 + every)
        if not m.any():
            out.append([w0 + every, 0, 0.0, None, None])
            continue
        j = int(np.nonzero(m)[0][-1])
        out.append([w0 + every, int(m.sum()), float(steps[m].mean()), round(float(logtemp[j]), 3), round(float(lev[j]), 3)])
    return out


def main():
    import numpy as np

    import test_converge_gpu as t

    args = sys.argv[1:]
    if "--prestep" in args:
        # the round-5 build's semantics: a fresh next_state array per step, so the
        # driver stores the true pre-step state.  The facade's default since round 6
        # is the reference's: one next_state array mutated in place by every step
        # (gbm_envs.py:125, 184-186, 212), which the loop stores after
        # `state = next_state` (rl_multiplicative.py:213-245).
        from rlmd_amd import envs as envs_mod

        base_step = envs_mod._SingleEnv.step

        def fresh_step(self, action):
            ns, r, d, risk = base_step(self, action)
            return np.array(ns, copy=True), r, d, risk

        envs_mod._SingleEnv.step = fresh_step
    steps = 50000
    for a in [a for a in args if a.startswith("--steps=")]:
        steps = int(a.split("=")[1])
    lo, hi = (int(v) for v in [a for a in args if not a.startswith("--")][0].split("-"))
    ref = t.ref_stats(lambda n: np.load(os.path.join(ROOT, "tests", "golden", n), allow_pickle=False), "gbm")
    got = []
    for seed in range(lo, hi + 1):
        g, lev, trial = one(seed, steps)
        n = len(g)
        sl = slice(n - n // 3, n)
        got.append((float(g[sl].mean()), float(lev[sl].mean())))
        t.record("gbm_single_stream", seed=seed, steps=steps, growth_pct=got[-1][0], lev=got[-1][1],
                 lev_curve=[round(float(x), 3) for x in lev], trial=trial)
        print(f"gbm single stream seed {seed}: growth {got[-1][0]:.3f} lev {got[-1][1]:.4f} "
              f"curve {' '.join(f'{x:.2f}' for x in lev[::5])}", flush=True)
        for row in trial:
            print("   ", row, flush=True)
    pg, pl = t.mw_p(got, ref)
    print(f"gbm single stream: Mann-Whitney p growth {pg:.3f} lev {pl:.3f}; lev median "
          f"{np.median([x for _, x in got]):.3f}", flush=True)
    t.record("gbm_single_stream_test", steps=steps, p_growth=pg, p_lev=pl, n=len(got))


if __name__ == "__main__":
    main()
