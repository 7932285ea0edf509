"""Per-update A/B of the oracle's restated SAC update against the reference's
own Agent_sac.learn, along the reference's own GBM_InvA trajectory.  Build
container only (imports /root/reference through tests/golden/_refshim.py).

The reference loop (scripts/rl_multiplicative.py) runs unchanged, but every
learn() is wrapped: the mini-batch indices and the two policy-noise tensors
are drawn first, the oracle is loaded with the reference agent's complete
state (parameters, targets, the Adam moments and step counts of the actor,
critic and temperature optimisers, log alpha, Cauchy scales), both take the
same update, and the parameter / log-alpha differences are recorded relative
to the size of the update itself.  The 4-step learn fixtures pin the update
from one initialisation; this pins it in every regime the reference visits
(tanh saturation, clamped log scales, small temperatures).

    python tools/probe/learn_resync_ab.py --seed 0 --steps 30000 --out gpurun_out/resync_s0.jsonl
"""
import argparse
import json
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
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--every", type=int, default=500)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    _refshim.install()
    import torch
    from torch.distributions import Normal

    torch.set_num_threads(1)
    import algos.algo_sac as asac
    import main as ref_main
    import tools.replay as rp
    from tools import utils

    from oracle.learn import OracleLearner, flatten, layout, views

    orig_learn = asac.Agent_sac.learn
    nets = ("actor", "critic_1", "critic_2")
    acc = {"n": 0, "actor": [], "critic": [], "alpha": [], "sat": [], "ls_clamp": []}
    fout = open(a.out, "w")

    def named(agent, nm):
        return {pn: p.detach().numpy().copy() for pn, p in getattr(agent, nm).named_parameters()}

    def adam_flat(agent, lay, n):
        m, v, t = np.zeros(n, np.float32), np.zeros(n, np.float32), {}
        for nm in nets:
            opt = getattr(agent, nm).optimiser
            for (pn, shp, o), p in zip(lay[nm], getattr(agent, nm).parameters()):
                st = opt.state.get(p, {})
                sz = int(np.prod(shp))
                if st:
                    m[o:o + sz] = st["exp_avg"].numpy().ravel()
                    v[o:o + sz] = st["exp_avg_sq"].numpy().ravel()
                    t[nm] = int(st["step"])
                else:
                    t[nm] = 0
        return m, v, t

    def learn(self):
        if self.memory.mem_idx <= self.batch_size:
            return orig_learn(self)
        B, A = self.batch_size, int(self.num_actions)
        S = int(np.ravel(self.input_dims)[0])
        h1, h2 = self.actor.fc1.out_features, self.actor.fc2.out_features
        lay, n = layout("SAC", S, A, h1, h2)
        max_mem = min(self.memory.mem_idx, self.memory.mem_size)
        idx = np.random.choice(max_mem, size=B, replace=False)
        eps_next, eps_cur = torch.randn(B, A), torch.randn(B, A)
        # the oracle, loaded with the reference agent's whole state
        P0 = flatten({nm: named(self, nm) for nm in nets}, lay, n)
        T0 = flatten({"actor": named(self, "actor"), "critic_1": named(self, "target_critic_1"),
                      "critic_2": named(self, "target_critic_2")}, lay, n)
        m, v, t = adam_flat(self, lay, n)
        la0 = float(self.log_alpha.detach())
        o = OracleLearner("SAC", S, A, h1, h2, B, int(self.optimise_count), self.loss_type, P0, T0,
                          logtemp=la0)
        o.load_state(P0, T0, m, v, [float(self.cauchy_scale_1), float(self.cauchy_scale_2)], la0)
        o.opt_a.t, o.opt_c.t = t["actor"], t["critic_1"]
        o.cntr = self.learn_step_cntr
        ts = self.temp_optimiser.state.get(self.log_alpha, {})
        if ts:
            o.opt_t.m = ts["exp_avg"].detach().clone().view(1)
            o.opt_t.v = ts["exp_avg_sq"].detach().clone().view(1)
            o.opt_t.t = int(ts["step"])
        mem = self.memory
        o.learn(mem.state_memory[idx], mem.action_memory[idx], mem.reward_memory[idx], mem.next_state_memory[idx],
                mem.terminal_memory[idx], eps_next, eps_cur)
        # the reference's own update on the same indices and noise
        q = [eps_next, eps_cur]
        saved_np, saved_rs = rp.np, Normal.rsample

        class _Rand:
            def choice(self, *args, **kw):
                return idx

        class _Np:
            random = _Rand()

            def __getattr__(self, name):
                return getattr(np, name)

        def _rsample(dist, sample_shape=torch.Size()):
            return dist.loc + q.pop(0) * dist.scale

        rp.np, Normal.rsample = _Np(), _rsample
        try:
            out = orig_learn(self)
        finally:
            rp.np, Normal.rsample = saved_np, saved_rs
        P1 = flatten({nm: named(self, nm) for nm in nets}, lay, n)
        Po = o.P.numpy()
        c0 = lay["critic_1"][0][2]
        for part, sl in (("actor", slice(0, c0)), ("critic", slice(c0, n))):
            step = np.abs(P1[sl] - P0[sl]).max()
            acc[part].append(float(np.abs(Po[sl] - P1[sl]).max() / max(step, 1e-30)))
        la1 = float(self.log_alpha.detach())
        acc["alpha"].append(abs(float(o.log_alpha) - la1) / max(abs(la1 - la0), 1e-30))
        # regime markers: deterministic action saturation and clamped log scales
        with torch.no_grad():
            s = torch.as_tensor(mem.state_memory[idx[:64]], dtype=torch.float32)
            mu, scale = self.actor.forward(s)
            acc["sat"].append(float((torch.tanh(mu).abs() > 0.999).float().mean()))
            acc["ls_clamp"].append(float(((scale.log() <= -20 + 1e-6) | (scale.log() >= 2 - 1e-6)).float().mean()))
        acc["n"] += 1
        if acc["n"] % a.every == 0:
            rec = {"update": acc["n"], "logtemp": la1,
                   **{k: {"median": float(np.median(acc[k])), "max": float(np.max(acc[k]))}
                      for k in ("actor", "critic", "alpha")},
                   "sat": float(np.mean(acc["sat"])), "ls_clamp": float(np.mean(acc["ls_clamp"]))}
            fout.write(json.dumps(rec) + "\n")
            fout.flush()
            print(json.dumps(rec), flush=True)
            for k in ("actor", "critic", "alpha", "sat", "ls_clamp"):
                acc[k] = []
        return out

    asac.Agent_sac.learn = learn
    inputs = dict(ref_main.inputs)
    inputs.update({"n_trials_mul": 1, "n_cumsteps_mul": float(a.steps), "gpu": "cpu", "buffer_gpu": False})
    inputs = utils.input_initialisation(inputs, [a.key], ["SAC"], ["MSE"], [1])
    inputs["test_agent"] = True
    inputs["ENV_KEY"] = a.key
    np.random.seed(a.seed)
    torch.manual_seed(a.seed)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            from scripts.rl_multiplicative import multiplicative_env

            multiplicative_env(ref_main.gym_envs, inputs, n_gambles=1)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
