"""The device's SAC exploration noise as a distribution (GPU box).  An fp32
agent whose actor is all zeros has mu = 0 and log scale 0, so its stochastic
action is tanh(eps) * max_action with eps the device's Philox Box-Muller draw
(rlmd_policy.h policy_draw); atanh recovers eps.  Prints the moments and the
tail frequencies against N(0, 1) with their z-scores.

    python tools/probe/policy_noise_stats.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from scipy.stats import norm

    from rlmd_amd.agent import DeviceAgent

    S, A, N = 5, 1, 65536
    ag = DeviceAgent("SAC", S, A, 256, 256, 512, 256, precision="fp32", seed=12345)
    with torch.no_grad():
        ag.params.zero_()
    ag.params_written()
    obs = torch.zeros(N, S, device="cuda:0")
    xs = []
    for c in range(1, 41):
        a = ag.act(obs, mode=0, noise_ctr=c).double().cpu().numpy().ravel()
        xs.append(np.arctanh(np.clip(a / 0.99, -1 + 1e-7, 1 - 1e-7)))
    x = np.concatenate(xs)
    n = x.size
    print(f"n {n} mean {x.mean():.5f} std {x.std():.5f} kurtosis {((x - x.mean()) ** 4).mean() / x.var() ** 2:.4f}")
    for t in (-3.5, -3.0, -2.5, -2.0, -1.0, 1.0, 2.0, 2.5, 3.0, 3.5):
        p = (x < t).mean() if t < 0 else (x > t).mean()
        e = norm.cdf(t) if t < 0 else norm.sf(t)
        print(f"{t:+.1f}: {p:.6f} expected {e:.6f}  z = {(p - e) / np.sqrt(e * (1 - e) / n):+.1f}")


if __name__ == "__main__":
    main()
