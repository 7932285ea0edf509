"""rlmd_amd.env_resources (the market driver's host slicing) against the
reference's tools/env_resources.py run with the same seeded np.random
(tests/golden/env_resources_kat.npz, make_golden.env_resources_kat): start
rows, shuffled extracts and observations exact, and the generator left in the
same state (the next uniform draw equal), so a seeded driver consumes the
stream as the reference does."""
import numpy as np

from rlmd_amd import env_resources as er


def test_slicing_matches_reference_draw_for_draw(golden):
    g = golden("env_resources_kat.npz")
    prices = g["prices"]
    np.random.seed(123)
    for i in range(4):
        ext_days, sample_days, interval = (int(x) for x in g[f"case{i}/params"])
        sl, st = er.time_slice(prices, ext_days, 1, sample_days)
        assert st == int(g[f"case{i}/start"])
        sh = er.shuffle_data(sl, interval)
        np.testing.assert_array_equal(sh, g[f"case{i}/shuffled"])
        assert np.random.random_sample() == float(g[f"case{i}/next_u"])
        for d in (1, 3):
            for t in (0, 2):
                np.testing.assert_array_equal(er.observed_market_state(sh, t, 1, d), g[f"case{i}/obs_d{d}_t{t}"])


def test_market_keys_and_price_files(tmp_path):
    import pytest

    from rlmd_amd.config import GYM_ENVS
    from rlmd_amd.main import load_market_data, market_env_keys

    assert market_env_keys(GYM_ENVS) == [23, 26]
    np.save(tmp_path / "stooq_usei.npy", np.ones((5, 3)))
    assert load_market_data(25, GYM_ENVS, {"market_dir": str(tmp_path)}).shape == (5, 3)
    with pytest.raises(FileNotFoundError):
        load_market_data(21, GYM_ENVS, {"market_dir": str(tmp_path)})
