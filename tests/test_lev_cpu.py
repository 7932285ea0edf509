"""The leverage-sweep oracle (oracle/lev.py) against the reference's own
coin_smart_lev run (tests/golden/lev.npz, make_golden.py:lev_fixtures)."""
import os

import numpy as np
import pytest

from oracle import lev as olev

Z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lev.npz"))
CASES = ["pos", "neg", "odd"]


def close_table(d, ref, rtol):
    """Entry-wise within rtol of the reference, with the dispersion rows (mad,
    std) also allowed rtol of their group's mean (they cancel)."""
    means = ref[:, [0, 1, 2, 0, 1, 2, 0, 1, 2, 0, 1, 2, 0], :]
    tol = rtol * np.abs(ref) + rtol * np.abs(means) * (np.arange(13) >= 3)[None, :, None] * (np.arange(13) < 9)[None, :, None]
    return np.abs(d - ref) <= tol + 1e-30


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    a = Z[case + "_args"]
    inv, hor, top = int(a[0]), int(a[1]), int(a[2])
    d, dT = olev.coin_smart_lev(Z[case + "_outcomes"], top, *a[3:])
    assert d.shape == (len(Z[case + "_levs"]), 13, hor - 1) and dT.shape == (len(Z[case + "_levs"]), inv)
    np.testing.assert_array_equal(dT, Z[case + "_data_T"])  # the same sequential f32 products
    assert close_table(d, Z[case + "_data"], 2e-6).all()


def test_param_range_matches_reference_grid():
    for case in CASES:
        a = Z[case + "_args"]
        np.testing.assert_allclose(olev.param_range(*a[6:9]), Z[case + "_levs"], rtol=0, atol=0)


def test_facade_param_range_is_the_oracle_grid():
    from rlmd_amd import lev

    for args in [(0.05, 1.0, 0.05), (0.1, 1.0, 0.1), (0.0, 0.0, 0.1), (0.25, 1.0, 0.25)]:
        assert lev.param_range(*args) == olev.param_range(*args)


SORTED = ["dice", "diceneg", "dicesh", "gbm"]


def sorted_oracle(case, outcomes=None):
    """oracle/lev.py's dice / dice_sh / gbm sweeps on a fixture case's inputs."""
    a, rets = Z[case + "_args"], Z[case + "_rets"]
    top, v0, lo, hi, inc = int(a[2]), a[3], a[4], a[5], a[6]
    o = Z[case + "_outcomes"] if outcomes is None else outcomes
    if case == "gbm":
        return olev.gbm_smart_lev(o, top, v0, lo, hi, inc)
    if case == "dicesh":
        return olev.dice_sh_smart_lev(o, top, v0, *rets, lo, hi, inc)
    return olev.dice_smart_lev(o, top, v0, *rets, lo, hi, inc)


@pytest.mark.parametrize("case", SORTED)
def test_sorted_oracle_matches_reference(case):
    """dice_smart_lev / dice_sh_smart_lev / gbm_smart_lev (lev_exp.py:586, :1209,
    :1008) run by the reference on torch CPU: final values bit-equal for the
    categorical gambles (the same f32 factors and products) and within 2 f32 ulps
    for GBM (NumPy's vs torch's expf); the table within 2e-6 / 2e-5."""
    d, dT = sorted_oracle(case)
    ref_d, ref_dT = Z[case + "_data"], Z[case + "_data_T"]
    assert d.shape == ref_d.shape and dT.shape == ref_dT.shape
    if case == "gbm":
        np.testing.assert_allclose(dT, ref_dT, rtol=2e-5, atol=0)
        assert close_table(d, ref_d, 2e-5).all()
    else:
        np.testing.assert_array_equal(dT, ref_dT)
        assert close_table(d, ref_d, 2e-6).all()


ZF = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lev_final.npz"))


def test_galaxy_brain_matches_reference():
    """coin_galaxy_brain_lev (lev_exp.py:455-505) run by the reference: the
    Kelly-fraction grid, bit-equal (host arithmetic in Python floats, f32 table)."""
    from rlmd_amd import lev

    got = lev.coin_galaxy_brain_lev("cpu", *ZF["galaxy_args"]).numpy()
    np.testing.assert_array_equal(got, ZF["galaxy"])


BRAIN = ["coinbrain", "dicebrain", "dicebrain0"]


def close26(d, ref, rtol):
    """close_table for the big-brain tables (value rows 0-11, leverage rows 12-23)."""
    idx = [0, 1, 2] * 4
    means = np.concatenate([ref[:, :, idx, :], ref[:, :, [12 + i for i in idx], :], ref[:, :, 24:26, :]], 2)
    disp = np.zeros(26, bool)
    disp[3:9] = disp[15:21] = True
    tol = rtol * np.abs(ref) + rtol * np.abs(means) * disp[None, None, :, None]
    return np.abs(d - ref) <= tol + 1e-30


def brain_inputs(case):
    a, rets = ZF[case + "_args"], ZF[case + "_rets"]
    inv, hor, top, v0, lf = int(a[0]), int(a[1]), int(a[2]), a[3], a[4]
    o = ZF[case + "_outcomes"]
    return inv, hor, top, v0, lf, tuple(a[5:8]), tuple(a[8:11]), rets, o


@pytest.mark.parametrize("case", BRAIN)
def test_brain_oracle_matches_reference(case):
    """coin_big_brain_lev (roll 0: a ratio > 0 raises TypeError in the reference)
    and dice_big_brain_lev (f64 values; roll 0 and > 0) run by the reference:
    the oracle within 2e-6 (dispersion rows 2e-6 of their group mean)."""
    inv, hor, top, v0, lf, st, rl, rets, o = brain_inputs(case)
    stops = np.array(olev.param_range(*st), np.float32)
    rolls = np.array(olev.param_range(*rl), np.float32)
    if case == "coinbrain":
        d = olev.brain_lev((o == 1).astype(np.int64), [np.float32(rets[1]), np.float32(rets[0]), np.float32(rets[0])],
                           top, v0, np.float32(lf), stops, rolls)
    else:
        d = olev.brain_lev(o.astype(np.int64), list(rets), top, v0, np.float32(lf), stops, rolls, f64=True)
    assert d.shape == ZF[case + "_data"].shape
    assert close26(d, ZF[case + "_data"], 2e-6).all()
