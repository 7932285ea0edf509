"""Evaluation episodes + summary statistics on the GPU.

rlmd_eval_rollout vs the reference's eval_multiplicative (tests/golden/eval.npz,
same injected draws): steps exact, last reward / risk within the env tolerance;
rlmd_eval_stats vs the reference's NumPy summary on the same arrays: bit-exact
(pairwise means, std, median_unbiased percentiles restated op for op)."""
import numpy as np
import pytest
import torch

from oracle import eval as oev
from tests.test_oracle_golden import RTOL, _eval_case

pytestmark = pytest.mark.gpu


def _stats(rew, steps, risk, inv, dev):
    from rlmd_amd import _abi

    out = torch.empty(17, dtype=torch.float64, device=dev)
    t = [torch.as_tensor(x, device=dev) for x in (np.asarray(rew, np.float64), np.asarray(steps, np.int32),
                                                 np.ascontiguousarray(risk, np.float64))]
    _abi.check(_abi.lib().rlmd_eval_stats(_abi.ptr(t[0]), _abi.ptr(t[1]), _abi.ptr(t[2]), len(rew), risk.shape[1],
                                          inv, _abi.ptr(out), _abi.stream_ptr()))
    return out.cpu().numpy()


@pytest.mark.parametrize("c", range(10))
def test_eval_rollout_and_stats_match_reference(golden, dev, c):
    from rlmd_amd import _abi
    from rlmd_amd.envs import VecEnv

    g = golden("eval.npz")
    fam, inv, n, cum, warm, sw, n_eval, max_steps = _eval_case(g, c)
    env = VecEnv(fam, inv, n_eval, n, device=dev)
    env.reset()
    act = torch.from_numpy(np.repeat(g[f"case{c}/action"][None, :], n_eval, 0)).to(dev)
    draws = torch.from_numpy(np.ascontiguousarray(g[f"case{c}/draws"])).to(dev)
    rew = torch.empty(n_eval, dtype=torch.float64, device=dev)
    steps = torch.empty(n_eval, dtype=torch.int32, device=dev)
    risk = torch.empty(n_eval, env.risk_dim, dtype=torch.float64, device=dev)
    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_eval_rollout(env.h, P(act), max_steps, cum, warm, sw, P(draws), P(rew), P(steps),
                                            P(risk), _abi.stream_ptr()))
    rew, steps, risk = (x.cpu().numpy() for x in (rew, steps, risk))
    np.testing.assert_array_equal(steps, g[f"case{c}/steps"])
    np.testing.assert_allclose(rew, g[f"case{c}/reward"], rtol=RTOL, atol=0)
    np.testing.assert_allclose(risk, g[f"case{c}/risk"], rtol=RTOL, atol=0, equal_nan=True)
    # the summary on the reference's own arrays: exactly NumPy's
    ref = oev.summary(g[f"case{c}/reward"], g[f"case{c}/steps"], g[f"case{c}/risk"], inv)
    got = _stats(g[f"case{c}/reward"], g[f"case{c}/steps"], g[f"case{c}/risk"], inv, dev)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 100, 129, 333, 1024])
def test_stats_numpy_exact_across_sizes(dev, n):
    """Pairwise-sum block boundaries (8, 128) and ties: bit-exact with NumPy."""
    from oracle import envs as oe

    rng = np.random.default_rng(n)
    rew = rng.lognormal(0, 0.3, n)
    rew[: n // 4] = rew[0]  # ties
    steps = rng.integers(1, 101, n)
    risk = rng.standard_normal((n, 6)) * 10 ** rng.uniform(-2, 4, (n, 6))
    got = _stats(rew, steps, risk, oe.INV_C, dev)
    np.testing.assert_array_equal(got, oev.summary(rew, steps, risk, oe.INV_C))


def test_trainer_evaluate(dev):
    from rlmd_amd.trainer import VecTrainer

    tr = VecTrainer("coin", "A", 1024, algo="SAC", k_updates=0, warmup_steps=2, smoothing_window=4,
                    replay_capacity=1024 * 8, precision="fp32", device=dev)
    for _ in range(3):
        tr.step()
    ev = tr.evaluate(n_eval=100, max_steps=100)
    assert set(ev) >= {"reward", "steps", "risk", "stats"}
    assert ev["steps"].min() >= 1 and ev["steps"].max() <= 100
    assert np.isfinite(ev["stats"][:15]).all()


def _market_agent(g, c, dev):
    from rlmd_amd.agent import DeviceAgent, layer_names
    from tests.test_oracle_golden import _eval_market_case

    algo, inv, d, n, test_days, cum, warm, sw, n_eval, h1, h2 = _eval_market_case(g, c)
    S, A = 4 + d * n, n + (1 if inv == 1 else 2 if inv == 2 else 0)
    init = {}
    for net in ("actor", "critic_1", "critic_2"):
        for nm in (net, "target_" + net):
            init[nm] = [torch.from_numpy(g[f"case{c}/init/{nm}.{pn}"]) for pn in layer_names(algo, net)]
    return DeviceAgent(algo, S, A, h1, h2, 16, 8, precision="fp32", init=init, device=dev)


@pytest.mark.parametrize("c", range(4))
def test_eval_market_matches_reference(golden, dev, c):
    """rlmd_eval_market vs the reference's eval_market (tests/golden/eval_market.npz:
    real SAC / TD3 agents, D1 and Dx, inside / outside the action window, injected
    gaps, unshuffled test slice).  Steps exact; last reward / risk within the
    fp32-policy tolerance of the oracle test (rtol 1e-6: the GPU and torch-CPU
    actor forwards differ in summation order); the 14 summary statistics within
    rtol 1e-5 of the reference's NumPy expressions on its own arrays."""
    from rlmd_amd.trainer import market_evaluate
    from tests.test_oracle_golden import _eval_market_case

    g = golden("eval_market.npz")
    algo, inv, d, n, test_days, cum, warm, sw, n_eval, _, _ = _eval_market_case(g, c)
    ag = _market_agent(g, c, dev)
    out = market_evaluate(ag, g[f"case{c}/prices"], inv, d, test_days, g[f"case{c}/gaps"], cum, warm, sw,
                          shuffle_days=1, device=dev)
    np.testing.assert_array_equal(out["steps"], g[f"case{c}/steps"])
    np.testing.assert_allclose(out["reward"], g[f"case{c}/reward"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(out["risk"], g[f"case{c}/risk_log"][:, 1:], rtol=1e-6, atol=1e-12)
    ref = oev.market_summary(g[f"case{c}/reward"], g[f"case{c}/steps"], g[f"case{c}/risk_log"])
    np.testing.assert_allclose(out["stats"], ref, rtol=1e-5, atol=1e-9)
    # the device summary is NumPy-exact on the same arrays
    got = oev.market_summary(out["reward"], out["steps"], out["risk_log"])
    np.testing.assert_array_equal(out["stats"], got)


@pytest.mark.parametrize("c", [0, 1])
def test_eval_market_shuffled_matches_oracle(golden, dev, c):
    """Test slices re-shuffled in blocks of 3 (Philox block permutations, E8) and
    a start that would leave the price table refused per lane: GPU vs oracle."""
    from rlmd_amd.trainer import market_evaluate
    from tests.test_oracle_golden import _eval_market_case, _golden_actor

    g = golden("eval_market.npz")
    algo, inv, d, n, test_days, cum, warm, sw, _, _, _ = _eval_market_case(g, c)
    prices = golden("market.npz")["prices"][:, :n]  # stooq_usei[:600]
    rng = np.random.default_rng(40 + c)
    starts = rng.integers(0, prices.shape[0] - test_days - d - 1, size=200)
    ag = _market_agent(g, c, dev)
    out = market_evaluate(ag, prices, inv, d, test_days, starts, cum, warm, sw, shuffle_days=3, seed=77, device=dev)
    rew, steps, risk = oev.market_rollout(algo, _golden_actor(g, c), prices, inv, d, test_days, starts, cum, warm,
                                          sw, shuffle_days=3, seed=77)
    np.testing.assert_array_equal(out["steps"], steps)
    np.testing.assert_allclose(out["reward"], rew, rtol=1e-6, atol=0)
    # risk holds float32 leverages 3 * a: the fp32 policy's summation order (GPU
    # GEMM vs torch-CPU) moves a by a few float32 ulps on 200 x 40 steps
    np.testing.assert_allclose(out["risk"], risk, rtol=1e-5, atol=1e-12)
    with pytest.raises(ValueError):
        market_evaluate(ag, prices, inv, d, test_days, [0, prices.shape[0] - test_days], cum, warm, sw, device=dev)


def test_trainer_evaluate_market(golden, dev):
    """C4's loop shape on a small table: policy steps on market lanes, then
    eval_market from the lanes' positions (gap 5..20 ahead)."""
    from rlmd_amd.trainer import VecTrainer

    prices = golden("market.npz")["prices"]  # stooq_usei[:600]
    tr = VecTrainer("market", "A", 256, n_gambles=3, algo="SAC", k_updates=1, warmup_steps=2, smoothing_window=4,
                    replay_capacity=256 * 16, precision="fp32", prices=prices, obs_days=1, time_length=12,
                    shuffle_days=5, sample_days=12 + 1 + 20 + 16 + 2, device=dev)
    for _ in range(6):
        tr.step()
    ev = tr.evaluate_market(n_eval=100, test_days=15)
    assert ev["steps"].min() >= 1 and ev["steps"].max() <= 15
    assert np.isfinite(ev["reward"]).all() and np.isfinite(ev["stats"]).all()
    assert ev["stats"].shape == (14,)


@pytest.mark.parametrize("algo,h1,h2", [("SAC", 256, 256), ("TD3", 400, 300)])
@pytest.mark.parametrize("inv,n,d", [("A", 1, 1), ("B", 1, 5), ("A", 2, 3)])
@pytest.mark.parametrize("window", [False, True])
def test_eval_market_one_launch_matches_day_loop(golden, dev, algo, h1, h2, inv, n, d, window):
    """rlmd_eval_market's one-launch form (eval_market_loop_kernel: bf16 policy +
    market step per lane, a day loop in the kernel) against the per-day host loop
    of fused acting + step launches (rlmd_train_set_fused(0)) on the same bf16
    agent: the same arithmetic, so rewards, steps and risk are bit-equal; D1 and
    Dx (S = 5, 9, 10: both LDS observation pitches), one and two assets, float32
    and (inside the action window) float64 actions, ragged 16-lane blocks, shuffled
    slices."""
    from rlmd_amd import _abi
    from rlmd_amd.agent import DeviceAgent
    from rlmd_amd.trainer import market_evaluate

    prices = golden("market.npz")["prices"][:, :n]
    S, A = 4 + d * n, n + (1 if inv == "B" else 0)
    ag = DeviceAgent(algo, S, A, h1, h2, 16, 8, precision="bf16", seed=5, device=dev)
    test_days = 40
    starts = np.random.default_rng(7).integers(0, prices.shape[0] - test_days - d - 1, size=203)
    cum, warm, sw = (50, 10, 100) if window else (500, 10, 100)
    outs = []
    for fused in (True, False):  # the evaluation env's switch (per handle)
        outs.append(market_evaluate(ag, prices, inv, d, test_days, starts, cum, warm, sw, shuffle_days=3, seed=11,
                                    device=dev, fused=fused))
    a, b = outs
    np.testing.assert_array_equal(a["steps"], b["steps"])
    np.testing.assert_array_equal(a["reward"], b["reward"])
    np.testing.assert_array_equal(a["risk"], b["risk"])
    np.testing.assert_array_equal(a["stats"], b["stats"])
    assert a["steps"].max() == test_days and np.isfinite(a["reward"]).all()


def test_eval_market_one_launch_time(dev):
    """C4's evaluation event (100 episodes x 250 test days, SAC 256/256 bf16,
    Market_InvA_D1) on a synthetic 9,167-day table: the one-launch form and the
    per-day loop, timed with events; the one-launch form must be faster."""
    from rlmd_amd import _abi
    from rlmd_amd.agent import DeviceAgent
    from rlmd_amd.trainer import market_evaluate

    rng = np.random.default_rng(3)
    prices = 100.0 * np.exp(np.cumsum(0.01 * rng.standard_normal((9167, 1)), axis=0))
    ag = DeviceAgent("SAC", 5, 1, 256, 256, 16, 8, precision="bf16", seed=1, device=dev)
    starts = rng.integers(0, 9167 - 260, size=100)
    from rlmd_amd.envs import VecEnv

    ms = {}
    for fused in (1, 0):
        env = VecEnv("market", "A", 100, 1, seed=1, prices=prices, obs_days=1, time_length=250, shuffle_days=3,
                     sample_days=251, device=dev)
        market_evaluate(ag, prices, "A", 1, 250, starts, 5000, 10, 100, device=dev, env=env, fused=bool(fused))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            out = market_evaluate(ag, prices, "A", 1, 250, starts, 5000, 10, 100, device=dev, env=env)
        e1.record()
        torch.cuda.synchronize()
        ms[fused] = e0.elapsed_time(e1) / 5
        assert out["steps"].max() == 250
    print(f"C4 eval event: one launch {ms[1]:.3f} ms, per-day loop {ms[0]:.3f} ms")
    assert ms[1] < ms[0]


def _bf16_actor(actor):
    """The one-launch kernel's policy numerics restated in torch (as
    test_train_gpu._bf16_act_reference): layer 1 f32, h1 and fc2.weight rounded
    to bf16, f32 accumulation and heads."""
    import torch.nn.functional as F

    def policy(state, head):
        h1 = F.relu(F.linear(state, actor["fc1.weight"], actor["fc1.bias"])).bfloat16().float()
        h2 = F.relu(F.linear(h1, actor["fc2.weight"].bfloat16().float(), actor["fc2.bias"]))
        return None, F.linear(h2, actor[head + ".weight"], actor[head + ".bias"])

    return policy


@pytest.mark.parametrize("c", range(4))
def test_eval_market_one_launch_matches_reference(golden, dev, c):
    """The one-launch bf16 evaluation (eval_market_loop_kernel) at the production
    widths (SAC 256/256, TD3 400/300; tests/golden/eval_market_full.npz: the
    reference's own eval_market with those agents, 32 episodes x 60 test days,
    D1 and Dx, inside / outside the action window) — the C4 evaluation path:
      * against the oracle rollout with the kernel's bf16 policy numerics
        restated (layer 1 f32, bf16 h1 / fc2.weight, f32 heads): steps exact,
        rewards within 1e-5 (layer 1's f32 summation order now and then moves
        one h1 element to its bf16 neighbour);
      * against the reference's fp32 run: steps exact, rewards within the bf16
        policy tolerance 2e-3 (the actions differ by bf16 rounding of layer 2)."""
    from rlmd_amd import _abi
    from rlmd_amd.agent import DeviceAgent, layer_names, reference_init
    from rlmd_amd.trainer import market_evaluate
    from tests.test_oracle_golden import _eval_market_case, _golden_actor

    g = golden("eval_market_full.npz")
    algo, inv, d, n, test_days, cum, warm, sw, n_eval, h1, h2 = _eval_market_case(g, c)
    S, A = 4 + d * n, n + inv
    init = reference_init(algo, S, A, h1, h2, seed=1)
    init["actor"] = [torch.from_numpy(g[f"case{c}/init/actor.{pn}"]) for pn in layer_names(algo, "actor")]
    ag = DeviceAgent(algo, S, A, h1, h2, 16, 8, precision="bf16", init=init, device=dev)
    out = market_evaluate(ag, g[f"case{c}/prices"], inv, d, test_days, g[f"case{c}/gaps"], cum, warm, sw,
                          shuffle_days=1, device=dev, fused=True)
    head = "pi" if algo == "SAC" else "mu"
    pol = _bf16_actor(_golden_actor(g, c))
    rew, steps, risk = oev.market_rollout(algo, None, g[f"case{c}/prices"], inv, d, test_days, g[f"case{c}/gaps"],
                                          cum, warm, sw, policy=lambda s: pol(s, head)[1])
    np.testing.assert_array_equal(out["steps"], steps)
    np.testing.assert_allclose(out["reward"], rew, rtol=1e-5, atol=0)
    np.testing.assert_array_equal(out["steps"], g[f"case{c}/steps"])
    np.testing.assert_allclose(out["reward"], g[f"case{c}/reward"], rtol=2e-3, atol=0)
    assert out["steps"].max() == test_days


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_state_dict_write_reaches_the_compute_copies(dev, precision):
    """A torch-side write through state_dict() without params_written() is still
    seen (version counters, DeviceAgent.sync_written): the next act runs on the
    new fc2.weight, bit-equal to acting after an explicit params_written()."""
    from rlmd_amd.agent import DeviceAgent

    ag = DeviceAgent("SAC", 5, 1, 256, 256, 16, 8, precision=precision, seed=3, device=dev)
    obs = torch.randn(256, 5, device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 0.5
    a0 = ag.act(obs, mode=1).clone()
    w2 = ag.state_dict("actor")["fc2.weight"]
    w2.mul_(-1.0)  # in place through the view; no params_written()
    a1 = ag.act(obs, mode=1).clone()
    ag.params_written()
    a2 = ag.act(obs, mode=1).clone()
    assert not torch.equal(a0, a1)
    assert torch.equal(a1, a2)
