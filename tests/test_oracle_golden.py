"""Pin the CPU oracle against vectors produced by the reference itself.

Golden files come from tests/golden/make_golden.py (reference imported in the
build container).  These run on CPU; they make the oracle trustworthy as the
checker of the HIP path (tests/test_*_gpu.py).
"""
import numpy as np
import pytest

from oracle import envs as oe
from oracle import philox as px

ENV_CLASSES = {
    "Coin": oe.COIN, "Dice": oe.DICE, "GBM": oe.GBM,
}
INV = {"InvA": oe.INV_A, "InvB": oe.INV_B, "InvC": oe.INV_C, "INSURED": oe.INV_INSURED}

# The oracle reproduces the reference's NumPy-2 dtype flow (oracle/envs.py);
# it is bit-exact on these traces today, the tolerance only absorbs libm ulps.
RTOL = 1e-13


def parse_env_key(key):
    parts = key.split("_")
    if parts[0] == "Dice" and parts[1] == "SH":
        return oe.DICE_SH, INV[parts[2]], 1
    fam = ENV_CLASSES[parts[0]]
    n = int(parts[2][1:])
    return fam, INV[parts[1]], n


def env_keys(g):
    return sorted(set(k.split("/")[0] for k in g.files))


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 R=10
    assert [hex(x) for x in px.philox(0, 0, 0, 0, 0)] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]
    m = 0xFFFFFFFF
    assert [hex(x) for x in px.philox((m << 32) | m, m, m, m, m)] == [
        "0x408f276d", "0x41c83b0e", "0xa20bc7c6", "0x6d5451fd"]
    key = 0xA4093822 | (0x299F31D0 << 32)
    assert [hex(x) for x in px.philox(key, 0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344)] == [
        "0xd16cfe09", "0x94fdcceb", "0x5001e420", "0x24126ea1"]


def test_choice_convention_matches_numpy_legacy(golden):
    g = golden("rng_kat.npz")
    for name, vals, p in (("coin", oe.COIN_VALS, oe.COIN_P), ("dice", oe.DICE_VALS, oe.DICE_P)):
        idx = oe.choice_index(g[name + "_u"], p)
        np.testing.assert_array_equal(vals[idx], g[name + "_choice"])


def test_uniform_is_numpy_random_sample_construction():
    # 53-bit construction: (a>>5)*2^26 + (b>>6) over 2^53, as RandomState.random_sample
    a = np.array([0xFFFFFFFF, 0, 0x80000000], dtype=np.uint32)
    b = np.array([0xFFFFFFFF, 0, 0], dtype=np.uint32)
    u = px.u01(a, b)
    assert u[0] < 1.0 and u[1] == 0.0 and u[2] == 0.5


@pytest.mark.parametrize("key", env_keys(np.load(
    __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "env_traces.npz"))))
def test_env_trace_matches_reference(golden, key):
    g = golden("env_traces.npz")
    fam, inv, n = parse_env_key(key)
    env = oe.OracleVecEnv(fam, inv, 1, n)
    acts, draws = g[key + "/actions"], g[key + "/draws"]
    S, S2, R, D, RK = (g[key + "/" + x] for x in ("state", "next_state", "reward", "done", "risk"))
    state = env.reset()
    for t in range(acts.shape[0]):
        np.testing.assert_allclose(state[0], S[t], rtol=RTOL, atol=0, err_msg=f"{key} t={t} state")
        ns, rew, dn, risk = env.step(acts[t:t + 1], draws[t:t + 1])
        np.testing.assert_allclose(ns[0], S2[t], rtol=RTOL, atol=0, err_msg=f"{key} t={t}")
        np.testing.assert_allclose(rew[0], R[t], rtol=RTOL, err_msg=f"{key} t={t} reward")
        np.testing.assert_array_equal(dn[0], D[t], err_msg=f"{key} t={t} done")
        np.testing.assert_allclose(risk[0], RK[t], rtol=RTOL, equal_nan=True, err_msg=f"{key} t={t} risk")
        state = ns
        if dn[0, 0]:
            state = env.reset()


# ---------------------------------------------------------------------------
# market slicing / shuffling / observation (tools/env_resources.py:203-291)
# ---------------------------------------------------------------------------
def test_market_time_slice(golden):
    g = golden("market.npz")
    prices = g["prices"]
    for i in range(4):
        st = int(g[f"slice{i}/start"])
        # time_slice(prices, extract_days=100, action_days=1, sample_days=130)
        np.testing.assert_array_equal(prices[st: st + 100 * 1 + 1], g[f"slice{i}/extract"])


def test_market_shuffle_rows(golden):
    g = golden("market.npz")
    for i in range(4):
        x = g[f"shuffle{i}/input"]
        d = int(g[f"shuffle{i}/interval"])
        flat = g[f"shuffle{i}/perms"]
        L = x.shape[0]
        sizes = [d] * (L // d) + ([L % d] if L % d else [])
        perms, o = [], 0
        for s in sizes:
            perms.append(flat[o:o + s])
            o += s
        rows = oe.shuffle_rows(L, d, perms)
        np.testing.assert_array_equal(x[rows], g[f"shuffle{i}/output"])


def test_market_observed_state(golden):
    g = golden("market.npz")
    ext = g["obs_extract"]
    n = ext.shape[1]
    for d in (1, 5):
        obs = g[f"obs_d{d}"]
        for t in range(obs.shape[0]):
            rows, assets = oe.observed_rows(t, 1, d, n)
            np.testing.assert_array_equal(ext[rows, assets], obs[t])


@pytest.mark.parametrize("key", ["Market_Inv%s_%s" % (i, d) for i in "ABC" for d in ("D1", "Dx")])
def test_market_env_episode_matches_reference(golden, key):
    g = golden("market_env.npz")
    ext = g[key + "/extract"]
    d = int(g[key + "/obs_days"])
    tl = int(g[key + "/time_length"])
    inv = {"A": oe.INV_A, "B": oe.INV_B, "C": oe.INV_C}[key[10]]
    # the extract is the episode's window: no shuffle, start fixed at 0
    env = oe.OracleVecEnv(oe.MARKET, inv, 1, ext.shape[1], prices=ext, obs_days=d,
                          time_length=tl, shuffle_days=1, sample_days=ext.shape[0] - 1)
    acts = g[key + "/actions"]
    state = env.reset()
    for t in range(acts.shape[0]):
        np.testing.assert_allclose(state[0], g[key + "/state"][t], rtol=RTOL)
        ns, r, dn, risk = env.step(acts[t:t + 1])
        np.testing.assert_allclose(ns[0], g[key + "/next_state"][t], rtol=RTOL, err_msg=f"t={t}")
        np.testing.assert_allclose(r[0], g[key + "/reward"][t], rtol=RTOL)
        np.testing.assert_array_equal(dn[0], g[key + "/done"][t])
        np.testing.assert_allclose(risk[0], g[key + "/risk"][t], rtol=RTOL, equal_nan=True)
        state = ns
    assert g[key + "/done"][-1][0]  # the episode ran to its done flag


# ---------------------------------------------------------------- F4 multi-step
@pytest.mark.parametrize("stream", ["a", "b", "c"])
@pytest.mark.parametrize("n", [3, 5, 7])
@pytest.mark.parametrize("dyn", ["A", "M"])
def test_multistep_history_matches_reference(golden, stream, n, dyn):
    """oracle.replay.MultiStepRing (one lane) vs the reference ReplayBuffer's
    multi-step reward / initial state / initial action / eff for every stored
    step after every checkpoint (tools/replay.py:93-332)."""
    from oracle.replay import MultiStepRing

    g = golden("multistep.npz")
    st, act, rew, s2, done = (g[f"{stream}/{k}"] for k in ("state", "action", "reward", "next_state", "done"))
    ring = MultiStepRing(4096, 2, 1, 1, n, dyn, 0.99)
    checked = 0
    for t in range(len(rew)):
        ring.insert(st[t], act[t], rew[t], s2[t], done[t])
        key = f"{stream}/n{n}{dyn}/T{t + 1}"
        if key + "/eff" not in g:
            continue
        R, S0, A0, S2, D, eff = ring.gather(np.arange(t + 1))
        np.testing.assert_array_equal(eff, g[key + "/eff"], err_msg=key)
        np.testing.assert_allclose(R, g[key + "/reward"], rtol=1e-15, atol=0, err_msg=key)
        np.testing.assert_array_equal(S0, g[key + "/state"], err_msg=key)
        np.testing.assert_array_equal(A0, g[key + "/action"].astype(np.float32).astype(np.float64), err_msg=key)
        checked += 1
    assert checked >= 8


# ---------------------------------------------------------------- F7 evaluation
def _eval_case(g, c):
    modname, cls = (str(x) for x in g[f"case{c}/spec"])
    n, cum, warm, sw, n_eval, max_steps = (int(x) for x in g[f"case{c}/params"])
    fam, inv, _ = parse_env_key(f"{cls}_n{n}")
    return fam, inv, n, cum, warm, sw, n_eval, max_steps


@pytest.mark.parametrize("c", range(10))
def test_eval_rollout_matches_reference(golden, c):
    """oracle.eval.rollout vs the reference's eval_multiplicative on the same
    injected draws: last reward, steps and last risk vector of every episode."""
    from oracle import eval as oev

    g = golden("eval.npz")
    fam, inv, n, cum, warm, sw, n_eval, max_steps = _eval_case(g, c)
    rew, steps, risk = oev.rollout(fam, inv, n, g[f"case{c}/action"], cum, warm, sw, n_eval, max_steps,
                                   g[f"case{c}/draws"])
    np.testing.assert_array_equal(steps, g[f"case{c}/steps"])
    np.testing.assert_allclose(rew, g[f"case{c}/reward"], rtol=RTOL, atol=0)
    np.testing.assert_allclose(risk, g[f"case{c}/risk"], rtol=RTOL, atol=0, equal_nan=True)
    st = oev.summary(rew, steps, risk, inv)
    assert np.isfinite(st[:15]).all()


def _eval_market_case(g, c):
    algo, inv, _ = (str(x) for x in g[f"case{c}/spec"])
    d, n, test_days, cum, warm, sw, n_eval, _, h1, h2 = (int(x) for x in g[f"case{c}/params"])
    return algo, "ABC".index(inv), d, n, test_days, cum, warm, sw, n_eval, h1, h2


def _golden_actor(g, c):
    import torch

    pre = f"case{c}/init/actor."
    return {k[len(pre):]: torch.from_numpy(g[k]) for k in g.files if k.startswith(pre)}


@pytest.mark.parametrize("fixture,c", [("eval_market.npz", c) for c in range(4)]
                         + [("eval_market_full.npz", c) for c in range(4)])
def test_eval_market_matches_reference(golden, fixture, c):
    """oracle.eval.market_rollout vs the reference's eval_market (real agent,
    deterministic policy on every state, injected gaps, unshuffled test slice):
    steps exact; last reward / risk within fp32-policy noise (the actor runs in
    float32 in both, on the same f32 states — rtol 1e-6 covers ulp-level matmul
    summation-order differences propagated through tanh and three env steps).
    eval_market_full.npz: the production widths (SAC 256/256, TD3 400/300),
    32 episodes x 60 days."""
    from oracle import eval as oev

    g = golden(fixture)
    algo, inv, d, n, test_days, cum, warm, sw, n_eval, _, _ = _eval_market_case(g, c)
    rew, steps, risk = oev.market_rollout(algo, _golden_actor(g, c), g[f"case{c}/prices"], inv, d, test_days,
                                          g[f"case{c}/gaps"], cum, warm, sw)
    np.testing.assert_array_equal(steps, g[f"case{c}/steps"])
    np.testing.assert_allclose(rew, g[f"case{c}/reward"], rtol=1e-6, atol=0)
    # risk holds the float32 leverages 3 a: at 256 / 400 hidden units the fp32
    # summation order (the oracle's F.linear vs the reference module's addmm) moves a
    # by a few float32 ulps
    rr = 1e-6 if fixture == "eval_market.npz" else 1e-5
    np.testing.assert_allclose(risk, g[f"case{c}/risk_log"][:, 1:], rtol=rr, atol=1e-12, equal_nan=True)
    st = oev.market_summary(rew, steps, np.concatenate([g[f"case{c}/risk_log"][:, :1], risk], 1))
    ref = oev.market_summary(g[f"case{c}/reward"], g[f"case{c}/steps"], g[f"case{c}/risk_log"])
    np.testing.assert_allclose(st, ref, rtol=1e-5, atol=1e-9)


# ---------------------------------------------------------------- A9 shadow means
def test_shadow_means_match_reference(golden):
    """oracle.shadow vs the reference's shadow_means (float64 grid) and
    agent_shadow_mean on float32 loss rows (its float32 dtype flow): exact up to
    NumPy's own float32 exp / pow, i.e. bit-equal here."""
    from oracle import shadow as osh

    g = golden("shadow.npz")
    got = np.array([osh.shadow_means(a, lo, hi, 1.0, 10.0, dtype=np.float64)
                    for a, lo, hi in zip(g["alpha"], g["min"], g["max"])])
    np.testing.assert_allclose(got, g["shadow"], rtol=1e-14)
    rows = np.stack([osh.agent_shadow_mean(r) for r in g["loss_rows"]])
    np.testing.assert_array_equal(rows, g["agent_shadow"])


@pytest.mark.filterwarnings("ignore::RuntimeWarning")  # SciPy's hybrd probes overflow exp on the way
def test_shadow_equiv_matches_reference(golden):
    """oracle.shadow.shadow_equiv (SciPy hybrd, the reference's own solver) vs the
    reference's utils.shadow_equiv as aggregate_data.py calls it."""
    from oracle import shadow as osh

    g = golden("shadow.npz")
    with np.errstate(all="ignore"):
        got = np.array([osh.shadow_equiv(m, a, lo, m, 1) for m, a, lo in zip(g["eq_mean"], g["eq_alpha"], g["eq_min"])])
    np.testing.assert_allclose(got, g["eq_out"], rtol=1e-12)
    assert (g["eq_out"][g["eq_alpha"] >= 1] == 1).all()


@pytest.mark.parametrize("fixture,fam", [("c1_trace.npz", oe.COIN), ("c1_gbm_trace.npz", oe.GBM)])
def test_stored_state_rule_matches_reference_loop(golden, fixture, fam):
    """F6 / F6-GBM: the reference's own C1 loop (scripts/rl_multiplicative.py,
    2,500 steps), recorded at store_transistion.  The oracle env replays its
    actions and draws (dtype as received: f64 in warm-up / window, f32 after);
    OracleVecEnv.stored_state gives what the loop stored — the reset state on an
    episode's first step, the aliased post-step state after (the env's one
    self.next_state array, gbm_envs.py:125, 184-186, 212; rl_multiplicative.py:
    213-245) — and step() gives the stored next states and rewards."""
    f = golden(fixture)
    ora = oe.OracleVecEnv(fam, oe.INV_A, 1, 1)
    obs = ora.reset()
    n = int(f["n_steps"])
    for t in range(n):
        a = f["action"][t].reshape(1, -1)
        a = a.astype(np.float64) if f["action_dtype"][t] else a.astype(np.float32)
        ns, r, d, _ = ora.step(a, draws=f["draw"][t].reshape(1, -1))
        np.testing.assert_allclose(ora.stored_state(obs, ns)[0], f["stored_state"][t], rtol=1e-12, atol=0,
                                   err_msg=f"t={t}")
        np.testing.assert_allclose(ns[0], f["stored_next_state"][t], rtol=1e-12, atol=0, err_msg=f"t={t}")
        np.testing.assert_allclose(r[0], f["reward"][t], rtol=1e-12, atol=0)
        assert list(d[0]) == list(f["done"][t]), t
        obs = ora.reset() if d[0, 0] else ns.copy()
    aliased = np.all(f["stored_state"] == f["stored_next_state"], 1)
    assert aliased.sum() == n - int(f["done"][:, 0].sum()) - (0 if f["done"][-1, 0] else 1)
