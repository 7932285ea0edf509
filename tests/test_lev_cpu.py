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
