"""The device learner against the oracle along the build's own GBM_InvA
trajectory (GPU box; the companion of tools/probe/learn_resync_ab.py, which
pins the oracle to the reference along the reference's trajectory).

The build's reference-API driver (rlmd_amd.main.run([14]), fp32 device agent)
runs as in tools/probe/gbm_single.py, but every `--every`-th learn() takes its
mini-batch from the device replay and its two noise tensors from torch, loads
the oracle with the device agent's state (parameters, targets, Adam moments
and step counts, Cauchy scales, log alpha) and applies the same update on
both.  Recorded per check: the largest parameter difference as a fraction of
the learning rate, the share of elements within 2e-6, the loss statistics'
relative difference, and the regime (deterministic-action saturation, log
alpha).  The temperature's own Adam moments are not exposed by the device, so
log alpha is not compared.

    python tools/probe/gbm_resync_gpu.py --seed 0 --steps 30000 --every 500 --out gpurun_out/resync_gpu_s0.jsonl
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--every", type=int, default=500)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import torch

    from oracle import learn as ol
    from rlmd_amd import agent as ag_mod
    from rlmd_amd.config import INPUTS
    from rlmd_amd.main import run as main_run

    orig = ag_mod.Agent_sac.learn
    cnt = {"n": 0}
    fout = open(a.out, "w")

    def learn(self):
        if self.memory.mem_idx <= self.batch_size:
            return orig(self)
        cnt["n"] += 1
        if cnt["n"] % a.every:
            return orig(self)
        dev = self.dev
        B, A, S, k = self.batch_size, dev.A, dev.S, self.optimise_count
        h1, h2 = dev.cfg.h1, dev.cfg.h2
        sc = dev.scalars()
        torch.cuda.synchronize()
        P0, T0 = dev.params.cpu().clone(), dev.target.cpu().clone()
        m0, v0 = dev.adam_m.cpu().clone(), dev.adam_v.cpu().clone()
        s, act, r, s2, d, _ = self._mini_batch()
        s, act, r, s2, d = (x.cpu() for x in (s, act, r, s2, d))
        ea, eb = torch.randn(B, A), torch.randn(B, A)
        o = ol.OracleLearner("SAC", S, A, h1, h2, B, k, "MSE", P0.numpy(), T0.numpy(), logtemp=sc["log_alpha"])
        o.load_state(P0, T0, m0, v0, sc["cauchy"], sc["log_alpha"])
        o.cntr = sc["learn_step_cntr"]
        o.opt_a.t = o.opt_c.t = sc["learn_step_cntr"]
        loss_o, _, _ = o.learn(s.numpy(), act.numpy(), r.numpy(), s2.numpy(), d.numpy(), ea, eb)
        st = dev.learn_batch(s, act, r, s2, d, ea, eb).double().cpu().numpy()
        P1 = dev.params.cpu().numpy()
        diff = np.abs(P1 - o.P.numpy())
        lay = o.lay
        c0 = lay["critic_1"][0][2]
        with torch.no_grad():
            pa = ol.views(torch.as_tensor(P1), lay)["actor"]
            h, mu = ol.mlp(pa, s[:64], "pi")
            ls = torch.nn.functional.linear(h, pa["log_scale.weight"], pa["log_scale.bias"])
        lo = np.asarray(loss_o, dtype=np.float64)
        rel = np.nanmax(np.abs(st[:11] - lo) / np.maximum(np.abs(lo), 1e-6)) if np.isfinite(lo).any() else None
        rec = {"update": cnt["n"], "log_alpha": sc["log_alpha"],
               "actor_max_over_lr": float(diff[:c0].max() / 3e-4), "critic_max_over_lr": float(diff[c0:].max() / 3e-4),
               "within_2e-6": float(np.mean(diff <= 2e-6)), "loss_rel": None if rel is None else float(rel),
               "actor_loss": [float(st[10]), float(lo[10])],
               "sat": float((torch.tanh(mu).abs() > 0.999).float().mean()), "mu": float(mu.mean()),
               "log_scale": float(ls.clamp(-20, 2).mean())}
        fout.write(json.dumps(rec) + "\n")
        fout.flush()
        print(json.dumps(rec), flush=True)
        return [float(x) for x in st[:11]], np.float32(st[11]), [float(x) for x in st[12:16]]

    ag_mod.Agent_sac.learn = learn
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            np.random.seed(a.seed)
            torch.manual_seed(a.seed)
            inputs = dict(INPUTS, n_trials_mul=1, n_cumsteps_mul=float(a.steps), test_agent=True)
            main_run([14], ["SAC"], ["MSE"], [1], inputs=inputs, log=None)
        finally:
            os.chdir(cwd)


if __name__ == "__main__":
    main()
