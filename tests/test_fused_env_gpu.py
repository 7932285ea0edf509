"""The steady-state kernel (env.hip act_env_kernel: policy acting + env step +
replay insert + auto-reset + episode rows in one launch) for every env family
and investor, at both acting widths (SAC 256/256, TD3 400/300) — GPU only.

Post-window policy steps (warm-up 0, smoothing 0, bf16 nets): every step's
ring rows (s, a, r, s', learn_done) are replayed through the oracle env
(oracle/envs.py, pinned to the reference's own traces) with the recorded f32
policy actions and the same Philox draws: f32-exact rows, f64 wealth within
1e-12 (Box-Muller libm ulps), done flags exact, and the per-episode rows the
kernel appends (ballot-compacted per wave) equal to the oracle's episode ends.
Reference steps covered: envs/coin_flip_envs.py:150-521,
envs/dice_roll_envs.py:153-524, envs/dice_roll_sh_envs.py:160-645,
envs/gbm_envs.py:147-515, envs/market_envs.py:133-202 / :283-358 / :440-528
(D1), dones tools/env_resources.py:26-200.

Two gambles / assets and market Dx windows run the kernel's run-time-n
instantiations (WIDE).  Three and four actions (the C investors, Dice_SH B / C,
market InvC at one day) run the wide-action instantiation (act_env_kernel<...,
MA = 4>: twice the head registers and partials); shapes with more actions AND
run-time n keep the two-launch path (acting kernel + env_train_kernel); the test
asserts which path ran (rlmd_train_last_fused) and checks both.

Fused vs unfused: the same seeded loop with rlmd_train_set_fused(1) and (0),
learning on (K = 1), must produce bit-identical rings, wealth and parameters
(act.hip and the fused kernel share rlmd_act_rows.h and both compile with FP
contraction off).
"""
import numpy as np
import pytest
import torch

from oracle import envs as oe
from tests.test_train_gpu import _market_kw, read_ring

pytestmark = pytest.mark.gpu

FAMS = {"coin": oe.COIN, "dice": oe.DICE, "gbm": oe.GBM, "dice_sh": oe.DICE_SH, "market": oe.MARKET}
INVS = {"A": oe.INV_A, "B": oe.INV_B, "C": oe.INV_C, "INSURED": oe.INV_INSURED}
CASES = ([(f, i) for f in ("coin", "dice", "gbm") for i in "ABC"]
         + [("dice_sh", i) for i in ("INSURED", "A", "B", "C")] + [("market", i) for i in "ABC"])


def _lib():
    from rlmd_amd import _abi

    return _abi.lib()


def _trainer(dev, golden, env, inv, algo, N, T, k=0, seed=11, n=1, obs_days=1):
    from rlmd_amd.trainer import VecTrainer

    kw = {}
    if env == "market":  # n assets: stooq_usei's first n columns
        kw = _market_kw(golden, obs_days)
        kw["prices"] = np.ascontiguousarray(kw["prices"][:, :n])
    return VecTrainer(env=env, investor=inv, n_lanes=N, n_gambles=n, algo=algo, k_updates=k, seed=seed,
                      init_seed=seed, warmup_steps=0, smoothing_window=0, replay_capacity=N * T, precision="bf16",
                      device=dev, **kw), kw


# the fused kernel's run-time-n instantiations (act_env_kernel<F, 0, ...>): two
# gambles / assets, and market Dx observation windows at the 16-float staging
# pitch (gbm_envs.py:147-212's n-gamble branches, market_envs.py:611-682)
WIDE = [("gbm", "A", 2, 1), ("coin", "A", 2, 1), ("dice", "A", 2, 1), ("market", "A", 2, 1),
        ("market", "A", 1, 5), ("market", "B", 1, 5), ("market", "A", 2, 3)]


@pytest.mark.parametrize("algo", ["SAC", "TD3"])
@pytest.mark.parametrize("env,inv", CASES)
def test_policy_steps_match_oracle(golden, dev, env, inv, algo):
    _replay_policy_steps(golden, dev, env, inv, algo, 1, 1)


@pytest.mark.parametrize("algo", ["SAC", "TD3"])
@pytest.mark.parametrize("env,inv,n,obs_days", WIDE)
def test_wide_shapes_match_oracle(golden, dev, env, inv, n, obs_days, algo):
    _replay_policy_steps(golden, dev, env, inv, algo, n, obs_days)


def _replay_policy_steps(golden, dev, env, inv, algo, n, obs_days):
    N, T, seed = 4000, 16, 11  # 4000 lanes: a ragged last 64-lane block
    tr, kw = _trainer(dev, golden, env, inv, algo, N, T, seed=seed, n=n, obs_days=obs_days)
    tr.set_fused(1)
    ora = oe.OracleVecEnv(FAMS[env], INVS[inv], N, n, seed=seed, **kw)
    obs = ora.reset()
    tr.episode_log(64)
    at = 1e-45 if env == "market" else 1e-30
    length = np.ones(N, dtype=np.int64)
    ng1 = n == 1 and obs_days == 1
    expect_fused = (ora.A <= 2 and (ora.S <= 8 or (env == "market" and ora.S <= 16))) or (
        ora.A <= 4 and ng1 and ora.S <= 8)
    ended = 0
    for t in range(T):
        tr.step()
        assert tr.last_fused() == expect_fused, "unexpected acting + env path"
        s_r, a_r, r_r, s2_r, d_r = read_ring(tr, t * N, N)
        assert np.all(np.abs(a_r) <= 0.99) and np.all(np.isfinite(a_r))
        ns, r, d, risk = ora.step(a_r.astype(np.float32))  # post-window policy actions: f32
        np.testing.assert_allclose(s_r, ora.stored_state(obs, ns).astype(np.float32), rtol=1e-6, atol=at, err_msg=f"t={t} s")
        np.testing.assert_allclose(r_r, r.astype(np.float32), rtol=1e-6, err_msg=f"t={t} r")
        np.testing.assert_allclose(s2_r, ns.astype(np.float32), rtol=1e-6, atol=at, err_msg=f"t={t} s2")
        np.testing.assert_array_equal(d_r.astype(bool), d[:, 1], err_msg=f"t={t} learn_done")
        w_gpu, t_gpu = tr.env.lane_state()
        live = ~d[:, 0]
        np.testing.assert_allclose(w_gpu[live], ora.wealth[live], rtol=1e-12, atol=0, err_msg=f"t={t} wealth")
        np.testing.assert_array_equal(t_gpu[live], ora.time[live])
        m = d[:, 0]
        rows, dropped = tr.drain_episodes()
        assert dropped == 0
        np.testing.assert_array_equal(rows[:, 1], np.nonzero(m)[0], err_msg=f"t={t} finished lanes")
        np.testing.assert_array_equal(rows[:, 0], np.full(len(rows), t), err_msg=f"t={t} step column")
        np.testing.assert_array_equal(rows[:, 2], r[m].astype(np.float32), err_msg=f"t={t} final rewards")
        np.testing.assert_array_equal(rows[:, 3], length[m], err_msg=f"t={t} lengths")
        np.testing.assert_allclose(rows[:, 4:], risk[m].astype(np.float32), rtol=1e-6, atol=0, err_msg=f"t={t} risk")
        ended += int(m.sum())
        length += 1
        length[m] = 1
        obs = ns.copy()
        if m.any():
            obs[m] = ora.reset(m)[m]
    np.testing.assert_allclose(tr.obs.cpu().numpy(), obs.astype(np.float32), rtol=1e-6, atol=at)
    assert np.unique(a_r[:, 0]).size > N // 4  # stochastic policy actions
    if env == "market":
        assert ended > 0  # 12-day episodes: lanes finish and restart inside the test


@pytest.mark.parametrize("algo", ["SAC", "TD3"])
@pytest.mark.parametrize("env,inv,n,obs_days", [("coin", "B", 1, 1), ("dice", "A", 1, 1), ("gbm", "A", 1, 1),
                                                ("dice_sh", "INSURED", 1, 1), ("dice_sh", "A", 1, 1),
                                                ("market", "B", 1, 1), ("gbm", "A", 2, 1), ("market", "A", 1, 5),
                                                ("gbm", "C", 1, 1), ("coin", "C", 1, 1), ("dice_sh", "B", 1, 1),
                                                ("dice_sh", "C", 1, 1), ("market", "C", 1, 1)])
def test_fused_equals_unfused(golden, dev, env, inv, n, obs_days, algo):
    N, T = 2048, 12
    out = []
    for fused in (1, 0):
        tr, _ = _trainer(dev, golden, env, inv, algo, N, T, k=1, seed=5, n=n, obs_days=obs_days)
        tr.set_fused(fused)  # per env handle
        for t in range(T):
            tr.step()
            assert tr.last_fused() == bool(fused)
        ring = read_ring(tr, 0, N * T)
        w, tt = tr.env.lane_state()
        out.append((ring, w, tt, tr.obs.cpu().numpy(), tr.agent.params.cpu().numpy().copy()))
        del tr
    (ra, wa, ta, oa, pa), (rb, wb, tb, ob, pb) = out
    for name, x, y in zip(("s", "a", "r", "s2", "d"), ra, rb):
        np.testing.assert_array_equal(x, y, err_msg=f"ring {name}")
    np.testing.assert_array_equal(wa, wb)
    np.testing.assert_array_equal(ta, tb)
    np.testing.assert_array_equal(oa, ob)
    np.testing.assert_array_equal(pa, pb)  # the K = 1 updates learned from identical rings


@pytest.mark.parametrize("algo", ["SAC", "TD3"])
def test_fused_equals_unfused_four_per_cu(golden, dev, algo):
    """As above at 65,600 lanes (1,025 acting blocks): both the fused act_env_kernel and
    the two-launch path's acting kernel run 4 workgroups per CU with their per-row
    values parked in LDS (act_env: the lane state and draw too)."""
    N, T = 65600, 4
    out = []
    for fused in (1, 0):
        tr, _ = _trainer(dev, golden, "gbm", "A", algo, N, T, k=1, seed=9, n=1, obs_days=1)
        tr.set_fused(fused)
        for t in range(T):
            tr.step()
            assert tr.last_fused() == bool(fused)
        ring = read_ring(tr, 0, N * T)
        w, tt = tr.env.lane_state()
        out.append((ring, w, tt, tr.obs.cpu().numpy(), tr.agent.params.cpu().numpy().copy()))
        del tr
    (ra, wa, ta, oa, pa), (rb, wb, tb, ob, pb) = out
    for name, x, y in zip(("s", "a", "r", "s2", "d"), ra, rb):
        np.testing.assert_array_equal(x, y, err_msg=f"ring {name}")
    np.testing.assert_array_equal(wa, wb)
    np.testing.assert_array_equal(ta, tb)
    np.testing.assert_array_equal(oa, ob)
    np.testing.assert_array_equal(pa, pb)
    assert np.unique(ra[1][:, 0]).size > N  # stochastic policy actions over the T steps


@pytest.mark.parametrize("fused", [1, 0])
@pytest.mark.parametrize("env,inv,n,obs_days", [("gbm", "A", 1, 1), ("coin", "B", 1, 1), ("dice", "C", 1, 1),
                                                ("market", "A", 1, 1), ("market", "B", 1, 5),
                                                ("dice_sh", "A", 1, 1)])
def test_stored_state_modes(golden, dev, env, inv, n, obs_days, fused):
    """rlmd_train_set_stored_state: RLMD_STORE_REFERENCE (the default) stores the
    reference loop's aliased state — s == s' from an episode's second step on
    for coin / dice / GBM / market (their envs mutate one self.next_state,
    gbm_envs.py:184-186; the loop stores state after state = next_state,
    rl_multiplicative.py:213-245), the reset state on an episode's first step,
    and the pre-step state for Dice_SH (a new array per step,
    dice_roll_sh_envs.py:336).  RLMD_STORE_PRESTEP stores the pre-step state
    everywhere.  Everything else in the two runs is bit-identical (no updates:
    the same policy acts on the same observations).  market B at obs_days 5 has
    S = 9 > 8 (the run-time-width store path of both kernels)."""
    N, T = 1000, 14
    rings, times = {}, {}
    for mode in ("reference", "prestep"):
        tr, _ = _trainer(dev, golden, env, inv, "SAC", N, T, k=0, seed=3, n=n, obs_days=obs_days)
        tr.set_fused(fused)
        if mode == "prestep":
            tr.set_stored_state("prestep")
        assert tr.stored_state() == ("prestep" if mode == "prestep" and env != "dice_sh" else "reference")
        tb = []
        for _ in range(T):
            tb.append(tr.env.lane_state()[1].copy())
            tr.step()
        rings[mode], times[mode] = read_ring(tr, 0, N * T), np.concatenate(tb)
        del tr
    ref, pre = rings["reference"], rings["prestep"]
    np.testing.assert_array_equal(times["reference"], times["prestep"])
    for i, name in ((1, "a"), (2, "r"), (3, "s2"), (4, "d")):
        np.testing.assert_array_equal(ref[i], pre[i], err_msg=name)
    later = times["reference"] > 1
    assert later.any() and (~later).any()  # both first steps (incl. auto-resets) and later steps
    if env == "dice_sh":
        np.testing.assert_array_equal(ref[0], pre[0])
    else:
        np.testing.assert_array_equal(ref[0][later], ref[3][later])  # s == s' (aliased)
        np.testing.assert_array_equal(ref[0][~later], pre[0][~later])  # the reset state
        assert not np.array_equal(pre[0][later], pre[3][later])
