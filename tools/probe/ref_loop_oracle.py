"""The reference's own multiplicative loop (env, replay, sampling, evaluation:
scripts/rl_multiplicative.py) with only the learner's arithmetic swapped for the
oracle's restatement (oracle/learn.py OracleLearner).  Build container only, as
tests/golden/run_reference_loop.py (it imports /root/reference through the same
shims; nothing here travels to the GPU box).

Agent_sac.learn (algo_sac.py:369-595) is replaced by: sample the mini-batch
with the reference's own ReplayBuffer.sample_exp, draw the two policy-noise
tensors from torch's generator, run OracleLearner.learn, and copy the oracle's
actor and log temperature back into the reference agent, whose
select_next_action / eval_next_action the loop then uses.  If this loop lands
where the reference does and the build does not, the build's long-run
difference is not in the restated update; if it climbs like the build, the
restatement (and the device learner pinned to it) differs from the reference
in something the 4-step learn fixtures do not see.

    python tools/probe/ref_loop_oracle.py --seed 0 --out gpurun_out/reforacle/s0.npz
"""
import argparse
import glob
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)
import _refshim  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", type=int, default=14)
    ap.add_argument("--steps", type=int, default=50000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--philox-env", action="store_true",
                    help="GBM returns from the build's Philox normals (oracle/philox.py) instead of np.random")
    a = ap.parse_args()
    _refshim.install()
    import torch

    torch.set_num_threads(1)
    import algos.algo_sac as asac
    import main as ref_main
    from tools import utils

    from oracle.learn import OracleLearner, flatten, layout, views

    def learn(self):
        if self.memory.mem_idx <= self.batch_size:
            return [np.nan] * 11, self.log_alpha.detach().cpu().numpy().copy(), [np.nan] * 4
        s, act, r, s2, done, _ = self.memory.sample_exp()
        B, A = self.batch_size, int(self.num_actions)
        if not hasattr(self, "_oracle"):
            S = int(np.ravel(self.input_dims)[0])
            h1, h2 = self.actor.fc1.out_features, self.actor.fc2.out_features
            lay, n = layout("SAC", S, A, h1, h2)
            sd = {nm: {pn: p.detach().numpy() for pn, p in getattr(self, nm).named_parameters()}
                  for nm in ("actor", "critic_1", "critic_2")}
            td = {"actor": sd["actor"], **{nm: {pn: p.detach().numpy() for pn, p in
                                                getattr(self, "target_" + nm).named_parameters()}
                                           for nm in ("critic_1", "critic_2")}}
            self._oracle = OracleLearner("SAC", S, A, h1, h2, B, int(self.optimise_count), self.loss_type,
                                         flatten(sd, lay, n), flatten(td, lay, n),
                                         logtemp=float(self.log_alpha.detach()))
        eps_next = torch.randn(B, A)
        eps_cur = torch.randn(B, A)
        loss, logtemp, lp = self._oracle.learn(s, act, r, s2, done, eps_next, eps_cur)
        P = views(self._oracle.P, self._oracle.lay)["actor"]
        with torch.no_grad():
            for pn, p in self.actor.named_parameters():
                p.copy_(P[pn])
            self.log_alpha.fill_(logtemp)
        return [np.float32(x) for x in loss], np.array(logtemp, dtype=np.float32), lp

    asac.Agent_sac.learn = learn
    if a.philox_env:
        import envs.gbm_envs as gbm_mod

        from oracle import philox as px

        ctr = [0]

        class _PhiloxRandom:
            def normal(self, loc=0.0, scale=1.0, size=None):
                n = int(np.prod(size)) if size is not None else 1
                z = np.asarray(px.normal_draws(a.seed, np.zeros(1, dtype=np.uint64), ctr[0], px.TAG_ENV_DRAW, n)).ravel()[:n]
                ctr[0] += 1
                out = loc + scale * z
                return out.reshape(size) if size is not None else float(out[0])

            def __getattr__(self, name):
                return getattr(np.random, name)

        class _Np:
            random = _PhiloxRandom()

            def __getattr__(self, name):
                return getattr(np, name)

        gbm_mod.np = _Np()

    inputs = dict(ref_main.inputs)
    inputs.update({"n_trials_mul": 1, "n_cumsteps_mul": float(a.steps), "gpu": "cpu", "buffer_gpu": False})
    inputs = utils.input_initialisation(inputs, [a.key], ["SAC"], ["MSE"], [1])
    inputs["test_agent"] = True
    inputs["ENV_KEY"] = a.key
    np.random.seed(a.seed)
    torch.manual_seed(a.seed)
    out = os.path.abspath(a.out)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            from scripts.rl_multiplicative import multiplicative_env

            multiplicative_env(ref_main.gym_envs, inputs, n_gambles=1)
            ev = np.load(glob.glob("results/**/*_eval.npy", recursive=True)[0])
            er = np.load(glob.glob("results/**/*_eval_risk.npy", recursive=True)[0])
            tr = np.load(glob.glob("results/**/*_trial.npy", recursive=True)[0])
        finally:
            os.chdir(cwd)
    np.savez_compressed(out, key=a.key, seed=a.seed, steps=a.steps, reward=ev[0, :, :, 1], lev=er[0, :, :, 3],
                        trial_steps=tr[0, :, 2], trial_logtemp=tr[0, :, 14], trial_lev=np.zeros_like(tr[0, :, 2]))
    print("wrote", out, "final mean lev", er[0, -5:, :, 3].mean())


if __name__ == "__main__":
    main()
