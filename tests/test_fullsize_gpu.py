"""The BASELINE configs at their full sizes (GPU).

C2 exactly as bench.py runs it: 65,536 GBM_InvA lanes, SAC 256/256 in bf16,
a 1,048,576-transition ring (16 vector steps: it wraps during the test), K = 8
updates of B = 512 per vector step.  Every step's 65,536 new ring rows (the
actions the env received, its rewards, next states and learn_done flags) are
replayed through the oracle env with the same Philox draws: f32-exact.  After
the run: learn counter = steps x K, status word clear, finite statistics.

C5's ring: 16,777,216 transitions (256 per lane over 65,536 lanes), n = 5
step returns (dynamics A), TD3 400/300 acting; 250 vector steps fill 16.4M
rows without overwriting (the reference requires buffer >= cumulative steps,
tools/replay.py:163).  For 256 lanes spread over the whole ring, every row's
n-step gather (eff, initial state / action, discounted return) is compared with
oracle/replay.MultiStepRing fed those lanes' raw rows: bit-exact / f32.
"""
import numpy as np
import pytest
import torch

from oracle import envs as oe
from oracle.replay import MultiStepRing
from tests.test_train_gpu import read_ring

pytestmark = pytest.mark.gpu


def test_c2_full_size_ring_and_learner(dev):
    from rlmd_amd.trainer import VecTrainer

    N, T, K, seed = 65536, 20, 8, 420
    tr = VecTrainer("gbm", "A", N, algo="SAC", k_updates=K, replay_capacity=1 << 20, seed=seed, warmup_steps=0,
                    smoothing_window=0, precision="bf16", device=dev, init_seed=seed)
    ora = oe.OracleVecEnv(oe.GBM, oe.INV_A, N, 1, seed=seed)
    obs = ora.reset()
    cap = 1 << 20
    for t in range(T):
        tr.step()
        s_r, a_r, r_r, s2_r, d_r = read_ring(tr, (t * N) % cap, N)
        ns, r, d, _ = ora.step(a_r.astype(np.float32))  # policy actions: f32 (NumPy-2 dtype flow)
        np.testing.assert_allclose(s_r, ora.stored_state(obs, ns).astype(np.float32), rtol=1e-6, atol=1e-30, err_msg=f"t={t} s")
        np.testing.assert_allclose(r_r, r.astype(np.float32), rtol=1e-6, err_msg=f"t={t} r")
        np.testing.assert_allclose(s2_r, ns.astype(np.float32), rtol=1e-6, atol=1e-30, err_msg=f"t={t} s2")
        np.testing.assert_array_equal(d_r.astype(bool), d[:, 1], err_msg=f"t={t} learn_done")
        obs = ns.copy()
        m = d[:, 0]
        if m.any():
            obs[m] = ora.reset(m)[m]
    assert np.abs(a_r).max() <= 0.99 and np.unique(a_r).size > N // 2  # stochastic policy actions
    sc = tr.agent.scalars()
    assert sc["learn_step_cntr"] == T * K and sc["nan_flag"] == 0
    assert tr.agent.status()[0] == 0  # no NaN flag (nan_update -1: never set)
    st = tr.last_stats()
    assert np.all(np.isfinite(st[[0, 1, 2, 3, 4, 5, 10, 11]])), st
    assert tr.replay.mem_idx == T * N


def test_c5_full_ring_multistep_gathers(dev):
    from rlmd_amd.trainer import VecTrainer

    N, T, n, cap = 65536, 250, 5, 1 << 24

    def make():
        return VecTrainer("gbm", "A", N, algo="TD3", k_updates=0, replay_capacity=cap, seed=7, init_seed=7,
                          warmup_steps=0, smoothing_window=0, precision="bf16", device=dev, multi_steps=n,
                          dynamics="A")

    # the run is deterministic (seeded Philox and initial parameters, no updates): a first pass finds the
    # lanes whose episodes end (rare: |action| < 1e-5 / lev_factor), so that the
    # tracked lanes include episode boundaries inside the n-step histories
    tr = make()
    ended = np.zeros(N, dtype=bool)
    for t in range(T):
        tr.step()
        ended |= read_ring(tr, t * N, N)[4].astype(bool)
    del tr
    torch.cuda.empty_cache()
    spread = np.linspace(0, N - 1, 256).astype(np.int64)
    with_end = np.flatnonzero(ended)[:64]
    lanes = np.unique(np.concatenate([with_end, spread]))[:256]
    if lanes.size < 256:
        lanes = np.unique(np.concatenate([lanes, np.setdiff1d(np.arange(N), lanes)[:256 - lanes.size]]))
    lanes = np.sort(lanes)
    tr = make()
    S, A = tr.env.state_dim, tr.env.action_dim
    ora = MultiStepRing(256 * (cap // N), S, A, 256, n, "A", 0.99)
    done_seen = 0
    for t in range(T):
        tr.step()
        s, a, r, s2, d = read_ring(tr, t * N, N)
        ora.insert(s[lanes], a[lanes], r[lanes], s2[lanes], d[lanes].astype(bool))
        done_seen += int(d[lanes].sum())
    assert tr.replay.mem_idx == T * N
    assert ended.any(), "no episode ended in 250 steps on any lane"
    assert done_seen > 0  # episode boundaries inside the tracked lanes' histories
    pos = np.arange(T)
    rows = (pos[:, None] * N + lanes[None, :]).ravel()  # GPU row of (position p, lane)
    orows = (pos[:, None] * 256 + np.arange(256)[None, :]).ravel()
    S0, A0, R, S2, D, eff = (x.cpu().numpy() for x in tr.replay.gather(rows))
    oR, oS, oA, _, _, oE = ora.gather(orows)
    np.testing.assert_array_equal(eff, oE)
    assert eff.min() >= 1 and eff.max() == n
    np.testing.assert_array_equal(S0, oS.astype(np.float32))
    np.testing.assert_array_equal(A0, oA.astype(np.float32))
    np.testing.assert_allclose(R, oR.astype(np.float32), rtol=1e-7, atol=0)
    # and one learner mini-batch from the full ring (TD3, B = 200, gamma^eff)
    st = tr.agent.learn(tr.replay, 2)
    assert np.all(np.isfinite(st.cpu().numpy()[:, [0, 1, 2, 3, 4, 5]]))
    f, _ = tr.agent.status()
    assert f == 0


def _replay_steps(tr, ora, T, cap, atol=1e-30):
    """Step the trainer T times, replaying every step's ring rows through the
    oracle env (f32 policy actions, the same Philox draws)."""
    N = tr.n_lanes
    obs = ora.reset()
    for t in range(T):
        tr.step()
        s_r, a_r, r_r, s2_r, d_r = read_ring(tr, (t * N) % cap, N)
        ns, r, d, _ = ora.step(a_r.astype(np.float32))
        np.testing.assert_allclose(s_r, ora.stored_state(obs, ns).astype(np.float32), rtol=1e-6, atol=atol, err_msg=f"t={t} s")
        np.testing.assert_allclose(r_r, r.astype(np.float32), rtol=1e-6, err_msg=f"t={t} r")
        np.testing.assert_allclose(s2_r, ns.astype(np.float32), rtol=1e-6, atol=atol, err_msg=f"t={t} s2")
        np.testing.assert_array_equal(d_r.astype(bool), d[:, 1], err_msg=f"t={t} learn_done")
        w_gpu, _ = tr.env.lane_state()
        live = ~d[:, 0]
        np.testing.assert_allclose(w_gpu[live], ora.wealth[live], rtol=1e-12, atol=0, err_msg=f"t={t} wealth")
        obs = ns.copy()
        m = d[:, 0]
        if m.any():
            obs[m] = ora.reset(m)[m]
    return a_r


@pytest.mark.parametrize("loss", ["MSE", "HUB", "MAE", "HSC"])
def test_c3_full_size_dice_sh_td3(dev, loss):
    """C3 at its size: 65,536 Dice_SH_InvA lanes (key 18: S = 6, A = 2), TD3
    400/300 bf16 (the fused act_env_kernel<DICE_SH, 416>), K = 8 updates of
    B = 200 / top-k 100 per vector step, one critic loss of the sweep; every
    step's ring rows replayed through the oracle env (envs/dice_roll_sh_envs.py:
    290-365), then the learner's counters and statistics."""
    from rlmd_amd import _abi
    from rlmd_amd.trainer import VecTrainer

    N, T, K, cap, seed = 65536, 4, 8, 1 << 20, 18
    tr = VecTrainer("dice_sh", "A", N, algo="TD3", loss=loss, k_updates=K, replay_capacity=cap, seed=seed,
                    warmup_steps=0, smoothing_window=0, precision="bf16", device=dev, init_seed=seed)
    ora = oe.OracleVecEnv(oe.DICE_SH, oe.INV_A, N, 1, seed=seed)
    a_r = _replay_steps(tr, ora, T, cap)
    assert tr.last_fused()
    assert tr.batch == 200 and tr.topk == 100 and a_r.shape == (N, 2)
    assert np.abs(a_r).max() <= 0.99 and np.unique(a_r[:, 0]).size > N // 4
    sc = tr.agent.scalars()
    assert sc["learn_step_cntr"] == T * K and sc["nan_flag"] == 0
    st = tr.last_stats()
    assert np.all(np.isfinite(st[[0, 1, 2, 3, 4, 5, 10]])), st


def test_c4_full_size_market_on_stooq_snp(golden, dev):
    """C4's per-GPU shard at its size: 8,192 Market_InvA_D1 lanes on the
    S&P 500 closes (stooq_snp, committed data fixture), train slices of 1,000
    days shuffled in blocks of 5, SAC 256/256 bf16, K = 8 updates of B = 512;
    every step's ring rows replayed through the oracle env
    (envs/market_envs.py:133-202, env_resources.py:203-291 with the Philox
    starts / permutations), then one evaluation event (100 episodes x 250
    test days, blocks of 3, gaps 5..20) on the device."""
    from rlmd_amd import _abi
    from rlmd_amd.trainer import VecTrainer

    N, T, K, cap, seed = 8192, 12, 8, 1 << 20, 0
    prices = golden("stooq_snp.npz")["prices"]
    kw = dict(prices=prices, obs_days=1, time_length=1000, shuffle_days=5, sample_days=1000 + 250 + 1 + 20 - 1)
    tr = VecTrainer("market", "A", N, algo="SAC", k_updates=K, replay_capacity=cap, seed=seed, warmup_steps=0,
                    smoothing_window=0, precision="bf16", device=dev, init_seed=seed, **kw)
    ora = oe.OracleVecEnv(oe.MARKET, oe.INV_A, N, 1, seed=seed, **kw)
    _replay_steps(tr, ora, T, cap, atol=1e-45)
    assert tr.last_fused()
    np.testing.assert_array_equal(tr.env.lane_start(), ora.start)
    sc = tr.agent.scalars()
    assert sc["learn_step_cntr"] == T * K and sc["nan_flag"] == 0
    ev = tr.evaluate_market(n_eval=100, test_days=250)
    assert ev["steps"].min() >= 1 and ev["steps"].max() <= 250 and np.isfinite(ev["reward"]).all()
    assert ev["stats"].shape == (14,) and np.isfinite(ev["stats"]).all()
