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
