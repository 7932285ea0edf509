"""Fused vector step (rlmd_train_step) vs the oracle, and acting parity — GPU only."""
import ctypes as C
import math

import numpy as np
import pytest
import torch

from oracle import envs as oe
from oracle import learn as ol
from oracle import philox as px
from tests.test_oracle_learn import NETS, TNETS

pytestmark = pytest.mark.gpu


def read_ring(tr, start, n):
    from rlmd_amd import _abi

    S, A, dev = tr.replay.S, tr.replay.A, tr.device
    s = torch.empty(n, S, device=dev)
    a = torch.empty(n, A, device=dev)
    r = torch.empty(n, device=dev)
    s2 = torch.empty(n, S, device=dev)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_replay_read(tr.replay.h, start, n, P(s), P(a), P(r), P(s2), P(d), _abi.stream_ptr()))
    return [x.cpu().numpy() for x in (s, a, r, s2, d)]


def warmup_actions(seed, N, A, t, absw):
    """Warm-up actions of step t: gym Box(-0.99, 0.99, float64).sample() =
    low + (high - low) * random_sample() on the Philox uniforms (np.abs unless GBM)."""
    a = np.empty((N, A), dtype=np.float64)
    for i in range(A):
        v = px.philox(seed, np.arange(N), t, px.TAG_WARMUP_ACTION, i >> 1)
        u = px.u01(v[0], v[1]) if i % 2 == 0 else px.u01(v[2], v[3])
        a[:, i] = -0.99 + 2 * 0.99 * u
    return np.abs(a) if absw else a


def _market_kw(golden, obs_days):
    # stooq_usei[:600]; 12-day episodes so lanes finish and restart inside the test
    return dict(prices=golden("market.npz")["prices"], obs_days=obs_days, time_length=12 + obs_days - 1,
                shuffle_days=5, sample_days=12 + obs_days + 40)


@pytest.mark.parametrize("env,inv,fam,oinv,n", [("gbm", "A", oe.GBM, oe.INV_A, 1), ("coin", "B", oe.COIN, oe.INV_B, 2),
                                                ("dice_sh", "C", oe.DICE_SH, oe.INV_C, 1),
                                                ("market", "B", oe.MARKET, oe.INV_B, 3),
                                                ("market", "C", oe.MARKET, oe.INV_C, -3)])
def test_warmup_steps_fill_ring_like_oracle(golden, dev, env, inv, fam, oinv, n):
    """Warm-up steps (rl_multiplicative.py:192-201, rl_market.py:217-226): Philox
    action samples (|.| unless GBM / market) through the fused step into the
    ring, auto-reset of finished lanes (market: new Philox slice + shuffle;
    n < 0 marks a Dx market env with obs_days 3), episode statistics."""
    from rlmd_amd.trainer import VecTrainer

    N, T, seed = 512, 25, 17
    kw = {}
    if fam == oe.MARKET:
        kw = _market_kw(golden, 1 if n > 0 else 3)
        n = abs(n)
    tr = VecTrainer(env=env, investor=inv, n_lanes=N, n_gambles=n, algo="SAC", k_updates=0, seed=seed,
                    warmup_steps=10_000, smoothing_window=20_000, replay_capacity=N * T, precision="fp32",
                    device=dev, **kw)
    ora = oe.OracleVecEnv(fam, oinv, N, n, seed=seed, **kw)
    obs = ora.reset()
    tr.episode_log(64)  # per-episode rows, drained every step (at most 64 per wave per step)
    absw = fam not in (oe.GBM, oe.MARKET)
    at = 1e-45 if fam == oe.MARKET else 1e-30  # market states are O(1e-30) (MAX_VALUE 1e34)
    length = np.ones(N, dtype=np.int64)  # current episode's step index (the env's t)
    exp_n, exp_r, exp_l = 0, 0.0, 0.0
    for t in range(T):
        tr.step()
        a = warmup_actions(seed, N, ora.A, t, absw)
        ns, r, d, risk = ora.step(a)  # float64 actions, as action_space.sample() gives
        s_r, a_r, r_r, s2_r, d_r = read_ring(tr, t * N, N)
        np.testing.assert_array_equal(a_r, a.astype(np.float32), err_msg=f"t={t} actions")
        np.testing.assert_allclose(s_r, ora.stored_state(obs, ns).astype(np.float32), rtol=1e-6, atol=at, err_msg=f"t={t} s")
        np.testing.assert_allclose(s2_r, ns.astype(np.float32), rtol=1e-6, atol=at, err_msg=f"t={t} s2")
        np.testing.assert_allclose(r_r, r.astype(np.float32), rtol=1e-6)
        np.testing.assert_array_equal(d_r.astype(bool), d[:, 1], err_msg=f"t={t} learn_done")
        obs = ns.copy()
        m = d[:, 0]
        rows, dropped = tr.drain_episodes()
        assert dropped == 0
        lanes = np.nonzero(m)[0]
        np.testing.assert_array_equal(rows[:, 1], lanes, err_msg=f"t={t} finished lanes")
        assert np.all(rows[:, 0] == rows[0, 0]) if len(rows) else True
        np.testing.assert_array_equal(rows[:, 2], r[m].astype(np.float32), err_msg=f"t={t} final rewards")
        np.testing.assert_array_equal(rows[:, 3], length[m], err_msg=f"t={t} lengths")
        np.testing.assert_allclose(rows[:, 4:], risk[m].astype(np.float32), rtol=1e-6, atol=0, err_msg=f"t={t} risk")
        exp_n += int(m.sum())
        exp_r += float(r[m].sum())
        exp_l += float(length[m].sum())
        length += 1
        length[m] = 1
        if m.any():
            obs[m] = ora.reset(m)[m]
        if t in (7, 8, T - 1):  # flushed reads, also back to back (nothing pending the second time)
            n_ep, r_sum, l_sum, _ = tr.flush_stats().cpu().numpy()
            assert n_ep == exp_n, f"t={t}"
            np.testing.assert_allclose([r_sum, l_sum], [exp_r, exp_l], rtol=1e-12)
    np.testing.assert_allclose(tr.obs.cpu().numpy(), obs.astype(np.float32), rtol=1e-6, atol=at)
    st = tr.episode_stats()
    assert st["episodes"] == exp_n


def _flat_init(algo, S, A, h1, h2, init):
    lay, n = ol.layout(algo, S, A, h1, h2)
    names = {nm: [x[0] for x in lay[nm]] for nm in NETS}
    p = ol.flatten({nm: dict(zip(names[nm], [t.numpy() for t in init[nm]])) for nm in NETS}, lay, n)
    t = ol.flatten({nm: dict(zip(names[nm], [t.numpy() for t in init[tn]])) for nm, tn in zip(NETS, TNETS)}, lay, n)
    return p, t


@pytest.mark.parametrize("algo,S,A,h1,h2", [("SAC", 5, 1, 256, 256), ("TD3", 6, 2, 400, 300), ("SAC", 6, 4, 256, 256)])
def test_act_matches_oracle_policy(dev, algo, S, A, h1, h2):
    from rlmd_amd.agent import DeviceAgent, reference_init

    init = reference_init(algo, S, A, h1, h2, seed=2)
    ag = DeviceAgent(algo, S, A, h1, h2, 512, 256, init=init, precision="fp32", device=dev)
    p, t = _flat_init(algo, S, A, h1, h2, init)
    ora = ol.OracleLearner(algo, S, A, h1, h2, 512, 256, "MSE", p, t)
    rng = np.random.default_rng(0)
    n = 4099
    obs = torch.from_numpy(rng.standard_normal((n, S)).astype(np.float32))
    eps = torch.from_numpy(rng.standard_normal((n, A)).astype(np.float32))
    Pn = ora.nets(ora.P)
    with torch.no_grad():
        det = ag.act(obs, mode=1).cpu()
        ref_det = ora.policy(Pn["actor"], obs, None, stochastic=False)[0]
        torch.testing.assert_close(det, ref_det, rtol=1e-5, atol=1e-6)
        sto = ag.act(obs, mode=0, eps=eps).cpu()
        if algo == "SAC":
            ref = ora.policy(Pn["actor"], obs, eps)[0]
        else:  # select_next_action: actor(s) + N(0, policy_noise), clamp to +-max_action
            ref = (ref_det + eps * ora.policy_noise).clamp(-ora.max_action, ora.max_action)
        torch.testing.assert_close(sto, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dist", ["L", "MVN"])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_act_policy_dists_match_oracle(dev, dist, precision):
    """Laplace and MVN samplers (networks_sac.py:180-258) in acting: injected noise vs
    the oracle (fp32: rows kernels' head path; bf16: the fused acting kernel, against
    the oracle within bf16 tolerance), Philox draws finite and inside the bounds."""
    from rlmd_amd.agent import DeviceAgent, reference_init

    S, A = 6, 2
    init = reference_init("SAC", S, A, 256, 256, seed=4)
    ag = DeviceAgent("SAC", S, A, 256, 256, 512, 256, init=init, precision=precision, policy_dist=dist, device=dev)
    p, t = _flat_init("SAC", S, A, 256, 256, init)
    ora = ol.OracleLearner("SAC", S, A, 256, 256, 512, 256, "MSE", p, t, s_dist=dist)
    rng = np.random.default_rng(7)
    n = 4099
    obs = torch.from_numpy(rng.standard_normal((n, S)).astype(np.float32))
    if dist == "L":
        noise = rng.uniform(np.finfo(np.float32).eps - 1.0, 1.0, (n, A))
    else:
        noise = rng.standard_normal((n, A))
    eps = torch.from_numpy(noise.astype(np.float32))
    with torch.no_grad():
        ref = ora.policy(ora.nets(ora.P)["actor"], obs, eps)[0]
        got = ag.act(obs, mode=0, eps=eps).cpu()
        phil = ag.act(obs, mode=0).cpu()
    err = (got - ref).abs()
    if precision == "fp32":
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    else:
        assert (err <= 2e-3).float().mean().item() >= 0.99, err.max().item()
    assert torch.isfinite(phil).all() and (phil.abs() <= ora.max_action).all()


def _bf16_act_reference(p, obs, eps, algo, max_action, ls_min, ls_max, noise):
    """The fused bf16 acting numerics restated in torch: layer 1 in f32, its output and
    fc2.weight rounded to bf16 (RNE), f32 accumulation, f32 heads and sampling."""
    import torch.nn.functional as F

    h1 = F.relu(F.linear(obs, p["fc1.weight"], p["fc1.bias"])).bfloat16().float()
    h2 = F.relu(F.linear(h1, p["fc2.weight"].bfloat16().float(), p["fc2.bias"]))
    head = "pi" if algo == "SAC" else "mu"
    mu = F.linear(h2, p[head + ".weight"], p[head + ".bias"])
    if algo == "TD3":
        a = torch.tanh(mu) * max_action
        return a, (a + eps * noise).clamp(-max_action, max_action)
    ls = F.linear(h2, p["log_scale.weight"], p["log_scale.bias"]).clamp(ls_min, ls_max)
    return torch.tanh(mu) * max_action, torch.tanh(mu + eps * ls.exp()) * max_action


@pytest.mark.parametrize("algo,S,A,h1,h2", [("SAC", 5, 1, 256, 256), ("SAC", 6, 2, 256, 256), ("TD3", 5, 1, 256, 256),
                                            ("SAC", 5, 1, 128, 256), ("TD3", 6, 2, 400, 300), ("TD3", 5, 1, 400, 300)])
def test_fused_bf16_act_matches_emulated_reference(dev, algo, S, A, h1, h2):
    """act.hip (one launch: VALU layer 1, bf16 MFMA layer 2, fused heads + sampling)
    against the same numerics restated in torch (bf16 rounding emulated exactly).  The
    f32 accumulation order of layer 1 differs, which now and then flips one h1 element
    to the neighbouring bf16 value: >= 99.9% of actions within 1e-4, all within 1e-3.
    The ragged last block (4099 rows) exercises the row guard; TD3 400/300 the
    zero-padded K (416) and column (320) tails of the compute copy."""
    from rlmd_amd.agent import DeviceAgent, reference_init

    init = reference_init(algo, S, A, h1, h2, seed=3)
    ag = DeviceAgent(algo, S, A, h1, h2, 512, 256, init=init, precision="bf16", device=dev)
    p, t = _flat_init(algo, S, A, h1, h2, init)
    ora = ol.OracleLearner(algo, S, A, h1, h2, 512, 256, "MSE", p, t)
    rng = np.random.default_rng(1)
    n = 4099
    obs = torch.from_numpy(rng.standard_normal((n, S)).astype(np.float32))
    eps = torch.from_numpy(rng.standard_normal((n, A)).astype(np.float32))
    Pn = ora.nets(ora.P)
    ref_det, ref_sto = _bf16_act_reference(Pn["actor"], obs, eps, algo, ora.max_action, ora.ls_min, ora.ls_max,
                                           ora.policy_noise)
    with torch.no_grad():
        det = ag.act(obs, mode=1).cpu()
        sto = ag.act(obs, mode=0, eps=eps).cpu()
        sto_philox = ag.act(obs, mode=0).cpu()
    for got, ref in ((det, ref_det), (sto, ref_sto)):
        err = (got - ref).abs()
        assert (err <= 1e-4).float().mean().item() >= 0.999, err.max().item()
        assert err.max().item() <= 1e-3
    assert torch.isfinite(sto_philox).all() and (sto_philox.abs() <= ora.max_action).all()
    assert not torch.equal(sto_philox, det)


@pytest.mark.parametrize("algo,S,A", [("SAC", 5, 1), ("SAC", 6, 2), ("TD3", 5, 1)])
def test_fused_act_four_per_cu_bit_equal(dev, algo, S, A):
    """At 65,539 rows (1,025 blocks, more than 3 per CU fit in one dispatch round) the
    256-wide acting kernel runs 4 workgroups per CU with its sampling rows' head
    biases and noise parked in LDS (rlmd_act_rows.h act_park); at 4,099 rows the same
    body runs 3 per CU with them in registers.  Actions of the shared rows are
    bit-equal — deterministic, injected noise and Philox noise (keyed by row and
    counter) — and the large launch matches the torch restatement like the small one."""
    from rlmd_amd.agent import DeviceAgent, reference_init

    h1 = h2 = 256
    init = reference_init(algo, S, A, h1, h2, seed=5)
    ag = DeviceAgent(algo, S, A, h1, h2, 512, 256, init=init, precision="bf16", device=dev)
    p, t = _flat_init(algo, S, A, h1, h2, init)
    ora = ol.OracleLearner(algo, S, A, h1, h2, 512, 256, "MSE", p, t)
    rng = np.random.default_rng(2)
    big, small = 65539, 4099
    obs = torch.from_numpy(rng.standard_normal((big, S)).astype(np.float32))
    eps = torch.from_numpy(rng.standard_normal((big, A)).astype(np.float32))
    with torch.no_grad():
        got = {n: (ag.act(obs[:n], mode=1).cpu(), ag.act(obs[:n], mode=0, eps=eps[:n]).cpu(),
                   ag.act(obs[:n], mode=0, noise_ctr=7).cpu()) for n in (big, small)}
    for i, name in enumerate(("deterministic", "injected noise", "Philox noise")):
        assert torch.equal(got[big][i][:small], got[small][i]), name
    ref_det, ref_sto = _bf16_act_reference(ora.nets(ora.P)["actor"], obs, eps, algo, ora.max_action, ora.ls_min,
                                           ora.ls_max, ora.policy_noise)
    for g, ref in ((got[big][0], ref_det), (got[big][1], ref_sto)):
        err = (g - ref).abs()
        assert (err <= 1e-4).float().mean().item() >= 0.999, err.max().item()
        assert err.max().item() <= 1e-3
    phil = got[big][2]
    assert torch.isfinite(phil).all() and (phil.abs() <= ora.max_action).all()
    assert np.unique(phil.numpy()).size > big // 2


def test_policy_steps_apply_action_window_and_learn(dev):
    from rlmd_amd.trainer import VecTrainer

    N = 2048
    tr = VecTrainer(env="gbm", investor="A", n_lanes=N, algo="SAC", k_updates=2, seed=4, warmup_steps=3,
                    smoothing_window=8, replay_capacity=N * 16, precision="fp32", device=dev)
    for t in range(12):
        tr.step()
        cs = t
        if cs >= 3:  # policy acted: tr.actions holds the raw policy actions
            raw = tr.actions.cpu().numpy()
            _, stored, _, _, _ = read_ring(tr, (t * N) % (N * 16), N)
            if 3 < cs <= 8:  # utils.action_window: np.clip with np.float64 bounds -> f64, stored as f32
                w = (math.sin(math.pi * (cs / 8 - 0.5)) + 1) / 2
                np.testing.assert_array_equal(stored, np.clip(raw.astype(np.float64), w * -0.99, w * 0.99).astype(np.float32))
            else:
                np.testing.assert_array_equal(stored, raw)
    st = tr.last_stats()
    assert np.all(np.isfinite(st[[0, 1, 2, 3, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15]])), st
    assert tr.agent.scalars()["learn_step_cntr"] == 2 * 12
    assert tr.agent.scalars()["nan_flag"] == 0


def test_profile_modes_count_the_timed_launches(dev):
    """rlmd_profile_enable: 2 times only the env kernel's dispatch (fused steps:
    act_env_kernel), every stride-th; 3 times the acting and the env kernel of
    unfused steps by their own dispatches (bench.py's in-step acting reference)."""
    from rlmd_amd.trainer import VecTrainer

    tr = VecTrainer(env="gbm", investor="A", n_lanes=4096, algo="SAC", k_updates=1, seed=5, warmup_steps=0,
                    smoothing_window=0, replay_capacity=4096 * 8, precision="bf16", device=dev)
    tr.step()
    tr.profile(2)
    tr.profile_stride(2)
    for _ in range(6):
        tr.step()
    ms, cnt = tr.profile_read()
    assert list(cnt) == [0, 3, 0] and ms[1] > 0
    samples = tr.profile_samples(1)
    assert len(samples) == 3 and abs(sum(samples) - ms[1]) < 1e-6 * max(ms[1], 1.0)
    assert tr.last_fused()
    tr.profile_stride(1)
    tr.set_fused(0)
    tr.profile(3)
    for _ in range(4):
        tr.step()
    ms, cnt = tr.profile_read()
    tr.profile(0)
    tr.set_fused(1)
    assert list(cnt) == [4, 4, 0] and ms[0] > 0 and ms[1] > 0, (ms, cnt)


@pytest.mark.parametrize("env,inv,fam,oinv", [("gbm", "A", oe.GBM, oe.INV_A), ("dice_sh", "B", oe.DICE_SH, oe.INV_B)])
def test_window_steps_feed_the_env_float64_actions(dev, env, inv, fam, oinv):
    """During warm-up (float64 action space sample) and inside the smoothing window
    (np.clip with np.float64 bounds) the reference env receives FLOAT64 actions:
    GBM leverage, stop-loss and safe-haven weights are then f64, not f32; policy
    actions after the window are f32.  The fused step must follow, against the
    oracle driven by the same actions and Philox draws."""
    from rlmd_amd.trainer import VecTrainer

    N, T, seed, warm, sw = 512, 14, 29, 3, 2000
    tr = VecTrainer(env=env, investor=inv, n_lanes=N, algo="SAC", k_updates=0, seed=seed, warmup_steps=warm,
                    smoothing_window=sw, replay_capacity=N * T, precision="fp32", device=dev)
    ora = oe.OracleVecEnv(fam, oinv, N, 1, seed=seed)
    obs = ora.reset()
    for t in range(T):
        tr.step()
        if t < warm:
            a = warmup_actions(seed, N, ora.A, t, fam != oe.GBM)
        else:
            raw = tr.actions.cpu().numpy()
            w = (math.sin(math.pi * (t / sw - 0.5)) + 1) / 2 if t > warm else None
            a = raw if w is None else np.clip(raw.astype(np.float64), w * -0.99, w * 0.99)
        ns, r, d, _ = ora.step(a)
        _, a_r, r_r, s2_r, d_r = read_ring(tr, t * N, N)
        np.testing.assert_array_equal(a_r, a.astype(np.float32), err_msg=f"t={t} actions")
        np.testing.assert_allclose(s2_r, ns.astype(np.float32), rtol=1e-6, atol=1e-30, err_msg=f"t={t} s2")
        np.testing.assert_allclose(r_r, r.astype(np.float32), rtol=1e-6, err_msg=f"t={t} r")
        np.testing.assert_array_equal(d_r.astype(bool), d[:, 1], err_msg=f"t={t} learn_done")
        w_gpu = tr.env.lane_state()[0]
        live = ~d[:, 0]
        # GBM draws go through Box-Muller (libm ulps, see test_env_gpu.py): 1e-12
        np.testing.assert_allclose(w_gpu[live], ora.wealth[live], rtol=1e-12, atol=0, err_msg=f"t={t} wealth")
        obs = ns.copy()
        m = d[:, 0]
        if m.any():
            obs[m] = ora.reset(m)[m]


def test_run_experiment_writes_reference_logs(dev, tmp_path):
    """Two short trials with evaluations: the four .npy arrays in the reference
    layout under utils.save_directory's stem (rlmd_amd/logs.py)."""
    from rlmd_amd.experiment import run_experiment

    path, lg = run_experiment("coin", "B", 1, algo="SAC", n_lanes=512, n_cumsteps=12, eval_freq=5, n_eval=20,
                              max_eval_steps=30, n_trials=2, k_updates=1, warmup_steps=3, smoothing_window=6,
                              buffer=512 * 16, precision="fp32", results_root=str(tmp_path), device=dev)
    assert path.endswith("Coin_InvB_n1--M_SAC-N_MSE-E_B81e2_M1_S12e0_N2")
    tr = np.load(path + "_trial.npy")
    ev = np.load(path + "_eval.npy")
    trk = np.load(path + "_trial_risk.npy")
    # one trial row per finished episode (rl_multiplicative.py:400-414), truncated to
    # the longer trial
    assert tr.shape[0] == 2 and tr.shape[2] == 19 and trk.shape[:2] == tr.shape[:2] and trk.shape[2] == 5
    assert tr.shape[1] == lg.rows.max() and lg.rows.min() > 0
    for t in range(2):
        k = int(lg.rows[t])
        assert np.all((tr[t, :k, 2] >= 1) & (tr[t, :k, 2] <= 12)) and np.all(tr[t, :k, 0] > 0)
        assert np.all(tr[t, k:] == 0)
        assert np.all(np.isfinite(trk[t, :k]))  # each episode's own last risk vector
        assert np.all(trk[t, :k, 0] == tr[t, :k, 1])  # risk[0] is the final reward (the score)
        assert np.isfinite(tr[t, k - 1, 3])  # learning from step 4 (mem_idx > batch)
    assert ev.shape == (2, 2, 20, 20)
    assert np.load(path + "_eval_risk.npy").shape == (2, 2, 20, 5)
    assert (ev[:, :, :, 19] == np.array([5, 10])[None, :, None]).all()
    assert (ev[..., 2] >= 1).all() and (ev[..., 2] <= 30).all()
