"""rlmd_lev_coin_sweep (lev.hip) against the reference's coin_smart_lev
fixtures and the oracle (lev/lev_exp.py:128-237).  Final values are the
reference's sequential float32 products, bit-exact; the summary table is
computed from up-count histograms with each bin's value rounded once, so it
agrees with the reference's step-by-step products to a few f32 ulps
(rtol 1e-5; mad / std rows also within 1e-5 of their group mean)."""
import os

import numpy as np
import pytest
import torch

from oracle import lev as olev
from tests.test_lev_cpu import CASES, Z, close_table

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", CASES)
def test_sweep_matches_reference(case):
    from rlmd_amd import lev

    a = Z[case + "_args"]
    inv, hor, top = int(a[0]), int(a[1]), int(a[2])
    d, dT = lev.coin_smart_lev("cuda:0", torch.from_numpy(Z[case + "_outcomes"]), inv, hor, top, *a[3:])
    d, dT = d.cpu().numpy(), dT.cpu().numpy()
    np.testing.assert_array_equal(dT, Z[case + "_data_T"])
    ok = close_table(d, Z[case + "_data"], 1e-5)
    assert ok.all(), np.argwhere(~ok)[:5]


@pytest.mark.parametrize("inv,hor,top,up,dn,extremes", [(20000, 300, 40, 0.5, -0.4, False),
                                                         (3000, 520, 10, 0.5, -0.4, True),
                                                         (4097, 130, 4097, 0.2, -0.2, False),
                                                         (5000, 64, 0, 0.5, -0.6, False)])
def test_sweep_matches_oracle(inv, hor, top, up, dn, extremes):
    """Larger random matrices; `extremes` adds all-up / all-down investors so a
    hist workgroup's up-count window exceeds its LDS (global-atomic path);
    top = investors leaves the adjusted group empty (NaN rows), top = 0 the top group."""
    from rlmd_amd import lev

    rng = np.random.default_rng(inv + hor)
    o = (rng.random((inv, hor)) < 0.5).astype(np.uint8)
    if extremes:
        o[0], o[1] = 1, 0
    d, dT = lev.coin_smart_lev("cuda:0", o, inv, hor, top, 100.0, up, dn, 0.25, 1.0, 0.25)
    od, odT = olev.coin_smart_lev(o, top, 100.0, up, dn, 0.25, 1.0, 0.25)
    d, dT = d.cpu().numpy(), dT.cpu().numpy()
    np.testing.assert_array_equal(dT, odT)
    fin = np.isfinite(od)
    bad = np.isfinite(d) != fin
    assert not bad.any(), (np.argwhere(bad)[:6], d[bad][:6], od[bad][:6])
    ok = close_table(np.where(fin, d, 0), np.where(fin, od, 0), 1e-5)
    assert ok.all(), np.argwhere(~ok)[:5]


@pytest.mark.parametrize("inv,hor,lo,hi", [(2000, 3500, 1.0, 1.0), (1500, 2400, 2.0, 2.0)])
def test_sweep_long_horizon_matches_oracle(inv, hor, lo, hi):
    """Horizons / leverages where gu^k and gd^(n-k) leave the double range on
    their own (lev 1: n = 3300, k = 1751 gives inf * 0; lev 2: gu = 2, gd = 0.2
    at n ~ 2050): the bin value is formed in log space, so populated bins stay
    finite.  Tolerance 1e-4: the reference's 3500 sequential f32 roundings
    drift up to ~n ulp from the once-rounded bin value."""
    from rlmd_amd import lev

    rng = np.random.default_rng(inv + hor)
    o = (rng.random((inv, hor)) < 0.5).astype(np.uint8)
    d, dT = lev.coin_smart_lev("cuda:0", o, inv, hor, 10, 100.0, 0.5, -0.4, lo, hi, 1.0)
    od, odT = olev.coin_smart_lev(o, 10, 100.0, 0.5, -0.4, lo, hi, 1.0)
    d, dT = d.cpu().numpy(), dT.cpu().numpy()
    np.testing.assert_array_equal(dT, odT)
    assert np.isfinite(od).all()
    assert np.isfinite(d).all(), np.argwhere(~np.isfinite(d))[:6]
    ok = close_table(d, od, 1e-4)
    assert ok.all(), np.argwhere(~ok)[:5]


def test_workspace_size_is_checked():
    from rlmd_amd import _abi, lev

    lib = _abi.lib()
    o, hor = lev.pack_outcomes(np.ones((64, 100), dtype=np.uint8))
    need = int(lib.rlmd_lev_workspace_bytes(64, hor))
    ws = torch.empty(need, dtype=torch.uint8, device="cuda:0")
    levs = np.array([0.5], dtype=np.float32)
    data = torch.empty((1, 13, hor - 1), dtype=torch.float32, device="cuda:0")
    P = _abi.ptr
    rc = lib.rlmd_lev_coin_sweep(P(o), 64, hor, o.stride(0), 1, 1.0, 0.5, -0.4, levs.ctypes.data, 1, P(ws),
                                 need - 1, P(data), None, _abi.stream_ptr())
    assert rc != 0 and b"workspace" in lib.rlmd_last_error()


def test_bad_arguments_fail_loudly():
    from rlmd_amd import _abi, lev

    o = np.ones((8, 10), dtype=np.uint8)
    with pytest.raises(_abi.RlmdError):  # gd = 1 + 3 * -0.4 < 0: values not monotone in the up-count
        lev.coin_smart_lev("cuda:0", o, 8, 10, 1, 1.0, 0.5, -0.4, 3.0, 3.0, 1.0)
    with pytest.raises(ValueError):
        lev.coin_smart_lev("cuda:0", o, 9, 10, 1, 1.0, 0.5, -0.4, 0.5, 0.5, 0.5)
    assert _abi.lib().rlmd_lev_workspace_bytes(10, 0) == -1


from tests.test_lev_cpu import SORTED, sorted_oracle  # noqa: E402


def _sorted_device(case, outcomes=None, top=None):
    from rlmd_amd import lev

    a, rets = Z[case + "_args"], Z[case + "_rets"]
    inv, hor = int(a[0]), int(a[1])
    top = int(a[2]) if top is None else top
    v0, lo, hi, inc = a[3], a[4], a[5], a[6]
    o = torch.from_numpy(Z[case + "_outcomes"] if outcomes is None else outcomes)
    inv, hor = o.shape
    if case == "gbm":
        d, dT = lev.gbm_smart_lev("cuda:0", o, inv, hor, top, v0, lo, hi, inc)
    elif case == "dicesh":
        d, dT = lev.dice_sh_smart_lev("cuda:0", o, inv, hor, top, v0, *rets, lo, hi, inc)
    else:
        d, dT = lev.dice_smart_lev("cuda:0", o, inv, hor, top, v0, *rets, lo, hi, inc)
    return d.cpu().numpy(), dT.cpu().numpy()


@pytest.mark.parametrize("case", SORTED)
def test_sorted_sweep_matches_reference(case):
    """rlmd_lev_sweep_sorted vs the reference's dice / dice_sh / gbm sweeps
    (tests/golden/lev.npz): categorical final values bit-exact (the same f32
    factors and sequential products), GBM within 2e-5 (device vs torch expf);
    the table within 2e-6 / 2e-5 (f64 group sums of the sorted values)."""
    d, dT = _sorted_device(case)
    ref_d, ref_dT = Z[case + "_data"], Z[case + "_data_T"]
    assert d.shape == ref_d.shape
    if case == "gbm":
        np.testing.assert_allclose(dT, ref_dT, rtol=2e-5, atol=0)
        ok = close_table(d, ref_d, 2e-5)
    else:
        np.testing.assert_array_equal(dT, ref_dT)
        ok = close_table(d, ref_d, 2e-6)
    assert ok.all(), np.argwhere(~ok)[:5]


@pytest.mark.parametrize("case,inv,hor,top", [("dice", 60000, 120, 600), ("dicesh", 40000, 90, 0),
                                              ("gbm", 50000, 100, 50000), ("diceneg", 7777, 60, 3)])
def test_sorted_sweep_matches_oracle_larger(case, inv, hor, top):
    """Larger outcome matrices (incl. top = 0 and top = investors: one group
    empty, NaN rows) against oracle/lev.py."""
    rng = np.random.default_rng(inv)
    if case == "gbm":
        o = (0.0540025395205692 - 0.1897916175617430 ** 2 / 2
             + 0.1897916175617430 * rng.standard_normal((inv, hor))).astype(np.float32)
    else:
        u = rng.random((inv, hor))
        o = np.where(u < 1 / 6, 0, np.where(u < 2 / 6, 1, 2)).astype(np.float32)
    d, dT = _sorted_device(case, o, top)
    od, odT = sorted_oracle_top(case, o, top)
    fin = np.isfinite(od)
    assert (np.isfinite(d) == fin).all()
    if case == "gbm":
        np.testing.assert_allclose(dT, odT, rtol=2e-5, atol=0)
        assert close_table(np.where(fin, d, 0), np.where(fin, od, 0), 2e-5).all()
    else:
        np.testing.assert_array_equal(dT, odT)
        assert close_table(np.where(fin, d, 0), np.where(fin, od, 0), 2e-6).all()


def sorted_oracle_top(case, o, top):
    from oracle import lev as olev

    a, rets = Z[case + "_args"], Z[case + "_rets"]
    v0, lo, hi, inc = a[3], a[4], a[5], a[6]
    if case == "gbm":
        return olev.gbm_smart_lev(o, top, v0, lo, hi, inc)
    if case == "dicesh":
        return olev.dice_sh_smart_lev(o, top, v0, *rets, lo, hi, inc)
    return olev.dice_smart_lev(o, top, v0, *rets, lo, hi, inc)


ZF = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lev_final.npz"))


@pytest.mark.parametrize("case", ["coin", "dice", "dicesh", "gbm"])
def test_fixed_final_matches_reference(case):
    """*_fixed_final_lev (lev_exp.py:56, :508, :935, :1121): the statistics the
    reference computed (recorded at its torch calls, make_golden.lev_final_fixtures)
    and its final values.  The device multiplies sequentially where the reference
    reduces with gambles.prod(dim=1) (torch's order): rtol 1e-5 on values and
    statistics (the dispersion rows also 1e-5 of the group mean)."""
    from rlmd_amd import lev

    a, rets = ZF[case + "_args"], [float(x) for x in ZF[case + "_rets"]]
    inv, hor, top, v0, lo, hi, inc = int(a[0]), int(a[1]), int(a[2]), a[3], a[4], a[5], a[6]
    o = torch.from_numpy(ZF[case + "_outcomes"])
    fn = {"coin": lev.coin_fixed_final_lev, "dice": lev.dice_fixed_final_lev, "dicesh": lev.dice_sh_fixed_final_lev,
          "gbm": lev.gbm_fixed_final_lev}[case]
    st, vals = fn("cuda:0", o, top, v0, *rets, lo, hi, inc)
    st, vals = st.cpu().numpy(), vals.cpu().numpy()
    np.testing.assert_allclose(vals, ZF[case + "_values"], rtol=1e-5, atol=0)
    ref = ZF[case + "_stats"]
    means = ref[:, [0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1, 2]]
    disp = (np.arange(12) >= 3) & (np.arange(12) < 9)
    tol = 1e-5 * np.abs(ref) + 1e-5 * np.abs(means) * disp[None, :]
    assert (np.abs(st[:, :12] - ref) <= tol + 1e-30).all(), (st[:, :12], ref)


from tests.test_lev_cpu import BRAIN, brain_inputs, close26  # noqa: E402


@pytest.mark.parametrize("case", BRAIN)
def test_big_brain_matches_reference(case):
    """rlmd_lev_brain vs the reference's coin / dice big-brain tables: 2e-6 (the
    same arithmetic per investor; f64 group sums of the sorted values)."""
    from rlmd_amd import lev

    inv, hor, top, v0, lf, st, rl, rets, o = brain_inputs(case)
    fn = lev.coin_big_brain_lev if case == "coinbrain" else lev.dice_big_brain_lev
    d = fn("cuda:0", torch.from_numpy(o), inv, hor, top, v0, *rets, torch.tensor(lf), *st, *rl).cpu().numpy()
    ok = close26(d, ZF[case + "_data"], 2e-6)
    assert ok.all(), np.argwhere(~ok)[:5]


@pytest.mark.parametrize("case,inv,hor", [("coin", 30000, 60), ("dice", 20000, 50)])
def test_big_brain_rolling_matches_oracle(case, inv, hor):
    """Larger matrices with retention ratios > 0 (coin included: the build's
    reading of the reference's TypeError path) against oracle/lev.py."""
    from oracle import lev as olev
    from rlmd_amd import lev

    rng = np.random.default_rng(inv)
    u = rng.random((inv, hor))
    stops, rolls = (0.1, 0.5, 0.2), (0.0, 0.9, 0.3)
    if case == "coin":
        o = (u < 0.5).astype(np.float32)
        d = lev.coin_big_brain_lev("cuda:0", o, inv, hor, 30, 100.0, 0.5, -0.4, 1.8, *stops, *rolls).cpu().numpy()
        od = olev.brain_lev((o == 1).astype(np.int64), [np.float32(-0.4), np.float32(0.5), np.float32(0.5)], 30, 100.0,
                            np.float32(1.8), np.array(olev.param_range(*stops), np.float32),
                            np.array(olev.param_range(*rolls), np.float32))
    else:
        o = np.where(u < 1 / 6, 0, np.where(u < 2 / 6, 1, 2)).astype(np.float32)
        d = lev.dice_big_brain_lev("cuda:0", o, inv, hor, 30, 100.0, 0.5, -0.5, 0.05, 1.6, *stops, *rolls).cpu().numpy()
        od = olev.brain_lev(o.astype(np.int64), [0.5, -0.5, 0.05], 30, 100.0, np.float32(1.6),
                            np.array(olev.param_range(*stops), np.float32),
                            np.array(olev.param_range(*rolls), np.float32), f64=True)
    assert d.shape == od.shape
    ok = close26(d, od, 2e-6)
    assert ok.all(), np.argwhere(~ok)[:5]
