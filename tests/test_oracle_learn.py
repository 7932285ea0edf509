"""Pin the learn() oracle (oracle/learn.py) against the reference's learn().

tests/golden/learn.npz holds, for SAC and TD3 cases, the reference agents'
initial parameters, replay contents, injected mini-batch indices and policy
noise, and every net's parameters + the loss / logtemp / loss_params lists
after each learn() call (tests/golden/make_golden.py:learn_fixtures).
"""
import numpy as np
import pytest

from oracle import learn as ol

NETS = ["actor", "critic_1", "critic_2"]
TNETS = ["target_actor", "target_critic_1", "target_critic_2"]


def case_names(g):
    return sorted(set(k.split("/")[0] for k in g.files if k.startswith("case")))


def sd(g, prefix, net):
    pre = f"{prefix}/{net}."
    return {k[len(pre):]: g[k] for k in g.files if k.startswith(pre)}


def build(g, c):
    algo = str(g[c + "/algo"])
    S, A, h1, h2, B, k = (int(x) for x in g[c + "/dims"])
    lay, n = ol.layout(algo, S, A, h1, h2)
    p = ol.flatten({nm: sd(g, c + "/init", nm) for nm in NETS}, lay, n)
    t = ol.flatten({nm: sd(g, c + "/init", tn) for nm, tn in zip(NETS, TNETS)}, lay, n)
    return algo, (S, A, h1, h2, B, k), lay, n, p, t


@pytest.mark.parametrize("case", ["case0", "case1", "case2", "case3", "case4", "case5", "case6"])
def test_learn_steps_match_reference(golden, case):
    g = golden("learn.npz")
    algo, (S, A, h1, h2, B, k), lay, n, p, t = build(g, case)
    lt = str(g[case + "/loss_fn"])
    L = ol.OracleLearner(algo, S, A, h1, h2, B, k, lt, p, t, s_dist=str(g[case + "/s_dist"]))
    rep = {x: g[f"{case}/replay/{x}"] for x in ("state", "action", "reward", "next_state", "done")}
    for s in range(int(g[case + "/n_steps"])):
        idx = g[f"{case}/step{s}/idx"]
        if algo == "SAC":
            ea, eb = g[f"{case}/step{s}/eps_next"], g[f"{case}/step{s}/eps_cur"]
        else:
            ea, eb = g[f"{case}/step{s}/eps_target"], None
        loss, logtemp, lp = L.learn(rep["state"][idx], rep["action"][idx], rep["reward"][idx],
                                    rep["next_state"][idx], rep["done"][idx], ea, eb)
        np.testing.assert_allclose(loss, g[f"{case}/step{s}/loss"], rtol=2e-5, atol=1e-7, equal_nan=True,
                                   err_msg=f"{case} step {s} loss")
        np.testing.assert_allclose(lp, g[f"{case}/step{s}/loss_params"], rtol=2e-5, atol=1e-7)
        if algo == "SAC":
            np.testing.assert_allclose(logtemp, g[f"{case}/step{s}/logtemp"], rtol=1e-5, atol=1e-8)
        ref_p = ol.flatten({nm: sd(g, f"{case}/step{s}", nm) for nm in NETS}, lay, n)
        ref_t = ol.flatten({nm: sd(g, f"{case}/step{s}", tn) for nm, tn in zip(NETS, TNETS)}, lay, n)
        np.testing.assert_allclose(L.P.numpy(), ref_p, rtol=0, atol=2e-6, err_msg=f"{case} step {s} params")
        np.testing.assert_allclose(L.T.numpy(), ref_t, rtol=0, atol=2e-6, err_msg=f"{case} step {s} targets")


@pytest.mark.parametrize("path", ["fused", "chain"])
@pytest.mark.parametrize("case", ["case0", "case1", "case2", "case3", "case4", "case5", "case6"])
def test_explicit_gradients_match_reference(golden, case, path):
    """The explicit-gradient form (precision="bf16"'s structure with the rounding
    off) reproduces the reference's learn() like the autograd form: it pins every
    hand-written gradient formula the bf16 oracle uses."""
    g = golden("learn.npz")
    algo, (S, A, h1, h2, B, k), lay, n, p, t = build(g, case)
    lt = str(g[case + "/loss_fn"])
    L = ol.OracleLearner(algo, S, A, h1, h2, B, k, lt, p, t, s_dist=str(g[case + "/s_dist"]), explicit=True,
                         path=path)
    rep = {x: g[f"{case}/replay/{x}"] for x in ("state", "action", "reward", "next_state", "done")}
    for s in range(int(g[case + "/n_steps"])):
        idx = g[f"{case}/step{s}/idx"]
        if algo == "SAC":
            ea, eb = g[f"{case}/step{s}/eps_next"], g[f"{case}/step{s}/eps_cur"]
        else:
            ea, eb = g[f"{case}/step{s}/eps_target"], None
        loss, logtemp, lp = L.learn(rep["state"][idx], rep["action"][idx], rep["reward"][idx],
                                    rep["next_state"][idx], rep["done"][idx], ea, eb)
        np.testing.assert_allclose(loss, g[f"{case}/step{s}/loss"], rtol=2e-5, atol=1e-7, equal_nan=True,
                                   err_msg=f"{case} step {s} loss")
        np.testing.assert_allclose(lp, g[f"{case}/step{s}/loss_params"], rtol=2e-5, atol=1e-7)
        if algo == "SAC":
            np.testing.assert_allclose(logtemp, g[f"{case}/step{s}/logtemp"], rtol=1e-5, atol=1e-8)
        ref_p = ol.flatten({nm: sd(g, f"{case}/step{s}", nm) for nm in NETS}, lay, n)
        ref_t = ol.flatten({nm: sd(g, f"{case}/step{s}", tn) for nm, tn in zip(NETS, TNETS)}, lay, n)
        np.testing.assert_allclose(L.P.numpy(), ref_p, rtol=0, atol=2e-6, err_msg=f"{case} step {s} params")
        np.testing.assert_allclose(L.T.numpy(), ref_t, rtol=0, atol=2e-6, err_msg=f"{case} step {s} targets")


def test_bf16_mode_rounds_and_stays_close(golden):
    """precision="bf16": the same update with bf16 operands — differs from the
    fp32 one (the rounding is applied) by far less than an Adam step in bulk."""
    g = golden("learn.npz")
    algo, (S, A, h1, h2, B, k), lay, n, p, t = build(g, "case0")
    lt = str(g["case0/loss_fn"])
    L32 = ol.OracleLearner(algo, S, A, h1, h2, B, k, lt, p, t)
    L16 = ol.OracleLearner(algo, S, A, h1, h2, B, k, lt, p, t, precision="bf16")
    rep = {x: g[f"case0/replay/{x}"] for x in ("state", "action", "reward", "next_state", "done")}
    idx = g["case0/step0/idx"]
    args = [rep["state"][idx], rep["action"][idx], rep["reward"][idx], rep["next_state"][idx], rep["done"][idx]]
    ea, eb = (g["case0/step0/eps_next"], g["case0/step0/eps_cur"]) if algo == "SAC" else (g["case0/step0/eps_target"], None)
    l32 = L32.learn(*args, ea, eb)[0]
    l16 = L16.learn(*args, ea, eb)[0]
    d = np.abs(L16.P.numpy() - L32.P.numpy())
    assert d.max() > 0
    assert np.mean(d < 1e-4) > 0.9
    np.testing.assert_allclose(l16[:6], l32[:6], rtol=5e-2)
