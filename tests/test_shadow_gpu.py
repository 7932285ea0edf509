"""Shadow means on the device: rlmd_shadow_means vs the
reference's agent_shadow_mean (tests/golden/shadow.npz, float32 loss rows) and
vs the oracle (SciPy gamma / gammaincc) on a wide random grid.

Tolerance: rtol 2e-6 (a few float32 ulps): the device's expf / powf and the
Cephes igamc restatement in double round differently from NumPy's float32 exp /
power and SciPy's own igamc in the last bits; inf / NaN positions must match."""
import numpy as np
import pytest
import torch

from oracle import shadow as osh

pytestmark = pytest.mark.gpu


def _device_shadow(rows, dev, in_place=False):
    from rlmd_amd import _abi

    st = torch.full((rows.shape[0], 16), float("nan"), dtype=torch.float32, device=dev)
    st[:, :11] = torch.from_numpy(rows).to(dev)
    if in_place:
        out, ldo, optr = st, 16, st.data_ptr() + 6 * 4
    else:
        out = torch.empty(rows.shape[0], 2, dtype=torch.float32, device=dev)
        ldo, optr = 2, out.data_ptr()
    _abi.check(_abi.lib().rlmd_shadow_means(_abi.ptr(st), rows.shape[0], 16, 1.0, 10.0, optr, ldo, _abi.stream_ptr()))
    res = (st[:, 6:8] if in_place else out).cpu().numpy()
    if in_place:  # nothing else in the row moved
        np.testing.assert_array_equal(st[:, :6].cpu().numpy(), rows[:, :6])
        np.testing.assert_array_equal(st[:, 8:11].cpu().numpy(), rows[:, 8:11])
    return res


def _check(got, ref):
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(np.isinf(got), np.isinf(ref))
    f = np.isfinite(ref)
    np.testing.assert_allclose(got[f], ref[f], rtol=2e-6, atol=0)


@pytest.mark.parametrize("in_place", [False, True])
def test_shadow_means_match_reference(golden, dev, in_place):
    g = golden("shadow.npz")
    _check(_device_shadow(g["loss_rows"], dev, in_place), g["agent_shadow"])


def test_shadow_means_match_oracle_grid(dev):
    rng = np.random.default_rng(3)
    n = 4096
    rows = np.full((n, 11), np.nan, dtype=np.float32)
    rows[:, 0:2] = rng.uniform(0.01, 10, (n, 2))
    rows[:, 2:4] = 10 ** rng.uniform(-6, 0, (n, 2))
    rows[:, 4:6] = rows[:, 2:4] * 10 ** rng.uniform(0, 6, (n, 2))  # max >= min, as for real losses
    rows[:, 8:10] = rng.uniform(-3, 1.2, (n, 2))
    ref = np.stack([osh.agent_shadow_mean(r) for r in rows])
    _check(_device_shadow(rows, dev), ref)


def test_trainer_last_stats_shadow(dev):
    from rlmd_amd.trainer import VecTrainer

    tr = VecTrainer("gbm", "A", 2048, algo="SAC", k_updates=2, warmup_steps=0, smoothing_window=0,
                    replay_capacity=2048 * 8, precision="fp32", device=dev)
    for _ in range(3):
        tr.step()
    raw = tr.last_stats()
    st = tr.last_stats(shadow=True)
    ref = osh.agent_shadow_mean(raw[:11].astype(np.float32))
    _check(st[6:8].astype(np.float32), ref)
    np.testing.assert_array_equal(st[:6], raw[:6])


def test_shadow_equiv_matches_reference(golden, dev):
    """rlmd_shadow_equiv (1-D Newton restatement of hybrd) vs the reference's
    MINPACK root: the same root within rtol 1e-6 (hybrd's xtol is 1.5e-8
    relative; the two iterations stop at different points inside it)."""
    from rlmd_amd import _abi

    g = golden("shadow.npz")
    t = [torch.from_numpy(np.ascontiguousarray(g[k])).to(dev) for k in ("eq_mean", "eq_alpha", "eq_min")]
    out = torch.empty_like(t[0])
    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_shadow_equiv(P(t[0]), P(t[1]), P(t[2]), P(t[0]), 1.0, t[0].numel(), P(out),
                                            _abi.stream_ptr()))
    np.testing.assert_allclose(out.cpu().numpy(), g["eq_out"], rtol=1e-6)
