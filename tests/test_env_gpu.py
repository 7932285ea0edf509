"""HIP env kernels vs the CPU oracle (pinned to the reference) — GPU only.

Bar: done / learn_done flags bit-exact; f64 state / reward / risk to 1e-12
relative (libm ulps between the device and glibc exp/log/cos).
"""
import numpy as np
import pytest
import torch

from oracle import envs as oe
from tests.test_oracle_golden import env_keys, parse_env_key

pytestmark = pytest.mark.gpu
RTOL = 1e-12
# Philox-mode GBM: z comes from Box–Muller with device vs glibc log/cos (1 ulp);
# r = LOG_MEAN + VOL*z cancels near r = 0, so the error is absolute: 1e-16 in
# return units = 1e-34 in MAX_VALUE-normalised state units.
ATOL_STATE, ATOL_RISK = 1e-30, 1e-12


def _venv(fam, inv, n_lanes, n, **kw):
    from rlmd_amd.envs import VecEnv

    return VecEnv(fam, inv, n_lanes, n, **kw)


def test_golden_traces_injected_draws(golden, dev):
    """Every reference trace, replicated in 64 lanes, with the reference's draws."""
    g = golden("env_traces.npz")
    for key in env_keys(g):
        fam, inv, n = parse_env_key(key)
        L = 64
        env = _venv(fam, inv, L, n)
        acts = torch.from_numpy(g[key + "/actions"]).to(dev)
        draws = torch.from_numpy(g[key + "/draws"]).to(dev)
        state = env.reset().clone()
        for t in range(acts.shape[0]):
            np.testing.assert_allclose(state.cpu().numpy(), np.broadcast_to(g[key + "/state"][t], state.shape),
                                       rtol=RTOL, err_msg=f"{key} t={t} state")
            ns, r, d, risk = env.step(acts[t].expand(L, -1).contiguous(), draws[t].expand(L, -1).contiguous())
            ns, r, d, risk = (x.cpu().numpy() for x in (ns, r, d, risk))
            np.testing.assert_allclose(ns, np.broadcast_to(g[key + "/next_state"][t], ns.shape), rtol=RTOL,
                                       err_msg=f"{key} t={t}")
            np.testing.assert_allclose(r, np.broadcast_to(g[key + "/reward"][t], r.shape), rtol=RTOL)
            np.testing.assert_array_equal(d.astype(bool), np.broadcast_to(g[key + "/done"][t], d.shape),
                                          err_msg=f"{key} t={t}")
            np.testing.assert_allclose(risk, np.broadcast_to(g[key + "/risk"][t], risk.shape), rtol=RTOL,
                                       equal_nan=True, err_msg=f"{key} t={t} risk")
            state = torch.from_numpy(ns).to(dev)
            if d[0, 0]:
                state = env.reset().clone()


CASES = [(f, i, n) for f in (oe.COIN, oe.DICE, oe.GBM) for i in (oe.INV_A, oe.INV_B, oe.INV_C) for n in (1, 3, 9)]
CASES += [(oe.DICE_SH, i, 1) for i in (oe.INV_INSURED, oe.INV_A, oe.INV_B, oe.INV_C)]


@pytest.mark.parametrize("fam,inv,n", CASES)
def test_philox_lanes_match_oracle(fam, inv, n, dev):
    """1024 lanes, 40 steps of Philox draws with mask resets: HIP == oracle."""
    N, T, seed = 1024, 40, 1234 + 7 * fam + inv
    env = _venv(fam, inv, N, n, seed=seed)
    ora = oe.OracleVecEnv(fam, inv, N, n, seed=seed)
    rng = np.random.default_rng(seed)
    for t in range(T):
        a = rng.uniform(-0.99, 0.99, (N, env.action_dim)).astype(np.float32)
        a[rng.random(N) < 0.05] = np.float32(0.99)
        a[rng.random(N) < 0.05] = 0.0
        ns, r, d, risk = (x.cpu().numpy() for x in env.step(torch.from_numpy(a).to(dev)))
        ons, orr, od, orisk = ora.step(a)
        np.testing.assert_array_equal(d.astype(bool), od, err_msg=f"t={t}")
        np.testing.assert_allclose(ns, ons, rtol=RTOL, atol=ATOL_STATE, err_msg=f"t={t}")
        np.testing.assert_allclose(r, orr, rtol=RTOL)
        np.testing.assert_allclose(risk, orisk, rtol=RTOL, atol=ATOL_RISK, equal_nan=True)
        mask = od[:, 0]
        if mask.any():
            s_gpu = env.reset(torch.from_numpy(mask).to(dev)).cpu().numpy()
            s_ora = ora.reset(mask)
            np.testing.assert_allclose(s_gpu[mask], s_ora[mask], rtol=RTOL)
    w, tt = env.lane_state()
    np.testing.assert_allclose(w, ora.wealth, rtol=RTOL)
    np.testing.assert_array_equal(tt, ora.time)


@pytest.mark.parametrize("inv,d", [(i, d) for i in (oe.INV_A, oe.INV_B, oe.INV_C) for d in (1, 4)])
def test_market_episode_golden(golden, dev, inv, d):
    g = golden("market_env.npz")
    key = "Market_Inv%s_%s" % ("ABC"[inv], "D1" if d == 1 else "Dx")
    ext = g[key + "/extract"]
    env = _venv(oe.MARKET, inv, 8, ext.shape[1], prices=ext, obs_days=d,
                time_length=int(g[key + "/time_length"]), shuffle_days=1, sample_days=ext.shape[0] - 1)
    acts = g[key + "/actions"]
    state = env.reset().cpu().numpy()
    for t in range(acts.shape[0]):
        np.testing.assert_allclose(state[0], g[key + "/state"][t], rtol=RTOL)
        ns, r, dn, risk = (x.cpu().numpy() for x in env.step(torch.from_numpy(np.repeat(acts[t:t + 1], 8, 0)).to(dev)))
        np.testing.assert_allclose(ns, np.broadcast_to(g[key + "/next_state"][t], ns.shape), rtol=RTOL)
        np.testing.assert_allclose(r, np.broadcast_to(g[key + "/reward"][t], r.shape), rtol=RTOL)
        np.testing.assert_array_equal(dn.astype(bool), np.broadcast_to(g[key + "/done"][t], dn.shape))
        np.testing.assert_allclose(risk, np.broadcast_to(g[key + "/risk"][t], risk.shape), rtol=RTOL, equal_nan=True)
        state = ns


@pytest.mark.parametrize("inv,d", [(oe.INV_A, 1), (oe.INV_C, 3)])
def test_market_shuffled_lanes_match_oracle(golden, dev, inv, d):
    """Philox episode starts + in-block shuffles (interval 5) on real prices."""
    prices = golden("market.npz")["prices"]  # stooq_usei[:600]
    N, tl, seed = 256, 40, 99
    sample_days = tl + d + 30
    kw = dict(obs_days=d, time_length=tl, shuffle_days=5, sample_days=sample_days)
    env = _venv(oe.MARKET, inv, N, prices.shape[1], prices=prices, seed=seed, **kw)
    ora = oe.OracleVecEnv(oe.MARKET, inv, N, prices.shape[1], prices=prices, seed=seed, **kw)
    np.testing.assert_allclose(env.reset().cpu().numpy(), ora.reset(), rtol=RTOL)
    rng = np.random.default_rng(5)
    for t in range(60):
        a = rng.uniform(-0.99, 0.99, (N, env.action_dim)).astype(np.float32)
        ns, r, dn, risk = (x.cpu().numpy() for x in env.step(torch.from_numpy(a).to(dev)))
        ons, orr, od, orisk = ora.step(a)
        np.testing.assert_array_equal(dn.astype(bool), od)
        np.testing.assert_allclose(ns, ons, rtol=RTOL)
        np.testing.assert_allclose(r, orr, rtol=RTOL)
        mask = od[:, 0]
        if mask.any():
            s_gpu = env.reset(torch.from_numpy(mask).to(dev)).cpu().numpy()
            np.testing.assert_allclose(s_gpu[mask], ora.reset(mask)[mask], rtol=RTOL)
