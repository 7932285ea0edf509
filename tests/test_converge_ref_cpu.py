"""The reference convergence band the GPU convergence test asserts against
(tests/test_converge_gpu.py): five reference seeds per env, made by the
reference's own rl_multiplicative loop (tests/golden/run_reference_loop.py),
with the last-third statistics its docstring states."""
import pytest

from tests.test_converge_gpu import KEYS, REF_SEEDS, ref_stats

BAND = {  # (growth min, max %/step), (lev min, max): last thirds of the five seeds
    "coin": ((-0.178, 0.315), (0.013, 0.105)),
    "dice": ((-0.136, 0.303), (-0.040, 0.123)),
    "dice_sh": ((-4.750, 2.037), (0.863, 0.929)),
}


@pytest.mark.parametrize("env", sorted(KEYS))
def test_reference_band(golden, env):
    st = ref_stats(golden, env)
    assert len(st) == len(REF_SEEDS) == 5
    (g0, g1), (l0, l1) = BAND[env]
    assert min(g for g, _ in st) == pytest.approx(g0, abs=1e-3)
    assert max(g for g, _ in st) == pytest.approx(g1, abs=1e-3)
    assert min(lv for _, lv in st) == pytest.approx(l0, abs=1e-3)
    assert max(lv for _, lv in st) == pytest.approx(l1, abs=1e-3)
    for s in REF_SEEDS:
        d = golden(f"converge_ref_{KEYS[env]}_s{s}.npz")
        assert int(d["key"]) == KEYS[env] and int(d["seed"]) == s and int(d["steps"]) == 50000
