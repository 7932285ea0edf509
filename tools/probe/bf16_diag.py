"""Diagnose bf16 device-vs-oracle parameter differences (GPU box): which layers,
and the oracle's gradient at the worst elements."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import learn as ol
from rlmd_amd.agent import DeviceAgent, reference_init
from tests.test_oracle_learn import NETS, TNETS

algo, S, A, h1, h2, B, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
init = reference_init(algo, S, A, h1, h2, seed=5)
lay, n = ol.layout(algo, S, A, h1, h2)
p = ol.flatten({nm: dict(zip([x[0] for x in lay[nm]], [t.numpy() for t in init[nm]])) for nm in NETS}, lay, n)
t = ol.flatten({nm: dict(zip([x[0] for x in lay[nm]], [t.numpy() for t in init[tn]])) for nm, tn in zip(NETS, TNETS)}, lay, n)
ora = ol.OracleLearner(algo, S, A, h1, h2, B, k, "MSE", p, t, precision="bf16")
ag = DeviceAgent(algo, S, A, h1, h2, B, k, loss="MSE", precision="bf16", init=init)
rng = np.random.default_rng(105)
for step in range(2):
    s = torch.from_numpy(rng.normal(0, 1, (B, S)).astype(np.float32))
    a = torch.from_numpy(rng.uniform(-0.99, 0.99, (B, A)).astype(np.float32))
    r = torch.from_numpy(rng.uniform(0.5, 1.5, B).astype(np.float32))
    s2 = torch.from_numpy(rng.normal(0, 1, (B, S)).astype(np.float32))
    d = torch.from_numpy(rng.random(B) < 0.1)
    ea = torch.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
    eb = torch.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
    st = ag.learn_batch(s, a, r, s2, d, ea, eb if algo == "SAC" else None).double().cpu().numpy()
    lo, _, _ = ora.learn(s.numpy(), a.numpy(), r.numpy(), s2.numpy(), d.numpy(), ea.numpy(), eb.numpy() if algo == "SAC" else None)
    print("step", step, "stats dev", st[:11], "\n  ora", np.asarray(lo))
    dp = np.abs(ag.params.cpu().numpy() - ora.P.numpy())
    for net, entries in lay.items():
        for pn, shp, o in entries:
            m = int(np.prod(shp))
            sl = dp[o:o + m]
            if sl.max() > 2e-6:
                print(f"  {net}.{pn}: {np.sum(sl > 2e-6)} / {m} > 2e-6, max {sl.max():.3g}")
    if step == 1:
        g = ora.last_grad.numpy()
        worst = np.argsort(-dp[:len(g)])[:10]
        print("  worst actor elements (idx, diff, oracle grad):", [(int(i), float(dp[i]), float(g[i])) for i in worst])
        print("  |grad| quantiles", np.quantile(np.abs(g), [0.001, 0.01, 0.5]))
