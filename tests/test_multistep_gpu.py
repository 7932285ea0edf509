"""Multi-step replay (tools/replay.py:93-332) on the GPU — SURVEY §8a R3 / Q7.

1. single stream vs the REFERENCE fixtures (multistep.npz): eff and the initial
   state/action exact, the n-step return within f32 rounding (the ring stores
   f32 rewards; the return is accumulated in f64 and rounded once);
2. several interleaved lanes (transition p of lane l at row p*lanes + l) vs the
   oracle's MultiStepRing fed the same f32 data: bit-exact;
3. the fused env step writes the same tags: its ring rows, replayed through the
   oracle in insertion order, give the GPU's gather bit for bit;
4. learn() consumes eff: gamma^eff bootstrapping matches the oracle learner.
"""
import numpy as np
import pytest
import torch

from oracle.replay import MultiStepRing

pytestmark = pytest.mark.gpu


def _gpu_ring(cap, S, A, n, dyn, lanes=1):
    from rlmd_amd.agent import ReplayMemory

    return ReplayMemory(cap, S, A, device="cuda:0", multi_steps=n, lanes=lanes, dynamics=dyn, gamma=0.99)


@pytest.mark.parametrize("stream", ["a", "b", "c"])
@pytest.mark.parametrize("n,dyn", [(3, "A"), (3, "M"), (5, "A"), (7, "M")])
def test_single_stream_matches_reference(golden, dev, stream, n, dyn):
    g = golden("multistep.npz")
    st, act, rew, s2, done = (g[f"{stream}/{k}"] for k in ("state", "action", "reward", "next_state", "done"))
    ring = _gpu_ring(4096, 2, 1, n, dyn)
    checked = 0
    for t in range(len(rew)):
        ring.store_exp(st[t], act[t], rew[t], s2[t], bool(done[t]))
        key = f"{stream}/n{n}{dyn}/T{t + 1}"
        if key + "/eff" not in g:
            continue
        S0, A0, R, S2, D, eff = (x.cpu().numpy() for x in ring.gather(np.arange(t + 1)))
        np.testing.assert_array_equal(eff, g[key + "/eff"], err_msg=key)
        np.testing.assert_array_equal(S0, g[key + "/state"].astype(np.float32), err_msg=key)
        np.testing.assert_array_equal(A0, g[key + "/action"].astype(np.float32), err_msg=key)
        np.testing.assert_allclose(R, g[key + "/reward"], rtol=3e-7, atol=0, err_msg=key)
        np.testing.assert_array_equal(S2, s2[: t + 1].astype(np.float32))
        np.testing.assert_array_equal(D, done[: t + 1])
        checked += 1
    assert checked >= 8


@pytest.mark.parametrize("n,dyn", [(3, "A"), (5, "M")])
def test_interleaved_lanes_match_oracle(dev, n, dyn):
    lanes, steps, S, A = 8, 40, 3, 2
    rng = np.random.default_rng(4)
    ring = _gpu_ring(lanes * 64, S, A, n, dyn, lanes=lanes)
    ora = MultiStepRing(lanes * 64, S, A, lanes, n, dyn, 0.99)
    for t in range(steps):
        s = rng.standard_normal((lanes, S)).astype(np.float32)
        a = rng.uniform(-1, 1, (lanes, A)).astype(np.float32)
        r = rng.uniform(0.5, 1.5, lanes).astype(np.float32)
        s2 = rng.standard_normal((lanes, S)).astype(np.float32)
        d = rng.random(lanes) < (0.3 if t % 7 else 0.9)
        ring.store_exp(s, a, r, s2, d)
        ora.insert(s, a, r, s2, d)
    rows = np.arange(lanes * steps)
    S0, A0, R, S2, D, eff = (x.cpu().numpy() for x in ring.gather(rows))
    oR, oS, oA, oS2, oD, oE = ora.gather(rows)
    np.testing.assert_array_equal(eff, oE)
    np.testing.assert_array_equal(S0, oS.astype(np.float32))
    np.testing.assert_array_equal(A0, oA.astype(np.float32))
    np.testing.assert_allclose(R, oR.astype(np.float32), rtol=1e-7, atol=0)
    np.testing.assert_array_equal(D, oD)


def test_fused_env_step_tags(dev):
    from rlmd_amd import _abi
    from rlmd_amd.trainer import VecTrainer

    N, steps = 256, 24
    tr = VecTrainer("coin", "A", N, algo="SAC", k_updates=0, replay_capacity=N * 32, warmup_steps=1000,
                    smoothing_window=2000, precision="fp32", device="cuda:0", multi_steps=3, dynamics="M")
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    M = N * steps
    S, A = tr.env.state_dim, tr.env.action_dim
    s, a, s2 = torch.empty(M, S, device=dev), torch.empty(M, A, device=dev), torch.empty(M, S, device=dev)
    r, d = torch.empty(M, device=dev), torch.empty(M, dtype=torch.uint8, device=dev)
    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_replay_read(tr.replay.h, 0, M, P(s), P(a), P(r), P(s2), P(d), _abi.stream_ptr()))
    ora = MultiStepRing(N * 32, S, A, N, 3, "M", 0.99)
    for t in range(steps):
        sl = slice(t * N, (t + 1) * N)
        ora.insert(s[sl].cpu().numpy(), a[sl].cpu().numpy(), r[sl].cpu().numpy(), s2[sl].cpu().numpy(),
                   d[sl].cpu().numpy().astype(bool))
    assert d.sum().item() > N // 4  # coin episodes end often: the episode logic is exercised
    rows = np.arange(M)
    S0, A0, R, S2, D, eff = (x.cpu().numpy() for x in tr.replay.gather(rows))
    oR, oS, oA, _, _, oE = ora.gather(rows)
    np.testing.assert_array_equal(eff, oE)
    np.testing.assert_array_equal(S0, oS.astype(np.float32))
    np.testing.assert_array_equal(A0, oA.astype(np.float32))
    np.testing.assert_allclose(R, oR.astype(np.float32), rtol=1e-7, atol=0)


def test_learn_bootstraps_with_gamma_pow_eff(dev):
    from oracle import learn as ol
    from rlmd_amd.agent import DeviceAgent, reference_init
    from tests.test_train_gpu import _flat_init

    algo, S, A, h1, h2, B, k = "TD3", 5, 1, 64, 48, 200, 100
    init = reference_init(algo, S, A, h1, h2, seed=9)
    ag = DeviceAgent(algo, S, A, h1, h2, B, k, precision="fp32", init=init, device=dev)
    p, t = _flat_init(algo, S, A, h1, h2, init)
    ora = ol.OracleLearner(algo, S, A, h1, h2, B, k, "MSE", p, t)
    rng = np.random.default_rng(2)
    for step in range(3):
        s = rng.standard_normal((B, S)).astype(np.float32)
        a = rng.uniform(-0.99, 0.99, (B, A)).astype(np.float32)
        r = rng.uniform(0.5, 1.5, B).astype(np.float32)
        s2 = rng.standard_normal((B, S)).astype(np.float32)
        d = rng.random(B) < 0.1
        eff = rng.integers(1, 6, B).astype(np.int32)
        ea = rng.standard_normal((B, A)).astype(np.float32)
        st = ag.learn_batch(*(torch.from_numpy(x) for x in (s, a, r, s2, d)), torch.from_numpy(ea), None,
                            eff=torch.from_numpy(eff)).double().cpu().numpy()
        ref = ora.learn(s, a, r, s2, d, ea, None, eff=eff)[0]
        np.testing.assert_allclose(st[:6], np.asarray(ref, np.float64)[:6], rtol=1e-4, atol=1e-6, err_msg=f"step {step}")
