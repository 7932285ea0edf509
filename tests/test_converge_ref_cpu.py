"""The reference convergence bands the GPU convergence test asserts against
(tests/test_converge_gpu.py): five reference seeds per workload, made by the
reference's own rl_multiplicative / rl_market loops
(tests/golden/run_reference_loop.py; C5 with 5-step returns, C4 through
market_env);
the last-third statistics (growth %/step, leverage) its docstring states."""
import pytest

from tests.test_converge_gpu import REF_SEEDS, WORKLOADS, bands, ref_stats

BAND = {  # (growth min, max %/step), (lev min, max): last thirds of the five seeds
    "coin": ((-0.178, 0.315), (0.013, 0.105)),
    "dice": ((-0.136, 0.303), (-0.040, 0.123)),
    "gbm": ((1.023, 5.181), (0.279, 1.411)),
    "dice_sh": ((-4.750, 2.037), (0.863, 0.929)),
    "dice_sh_a_mse": ((-6.244, 1.895), (0.481, 1.980)),
    "dice_sh_a_hub": ((-16.640, 0.756), (0.263, 1.980)),
    "gbm_td3_n5": ((-17.530, 13.979), (-3.633, 4.165)),
    "market": ((1.131, 5.921), (0.207, 1.708)),
}


@pytest.mark.parametrize("workload", sorted(WORKLOADS))
def test_reference_band(golden, workload):
    st = ref_stats(golden, workload)
    assert len(st) == len(REF_SEEDS) == 5
    (g0, g1), (l0, l1) = BAND[workload]
    assert min(g for g, _ in st) == pytest.approx(g0, abs=1e-3)
    assert max(g for g, _ in st) == pytest.approx(g1, abs=1e-3)
    assert min(lv for _, lv in st) == pytest.approx(l0, abs=1e-3)
    assert max(lv for _, lv in st) == pytest.approx(l1, abs=1e-3)
    stem = WORKLOADS[workload][3]
    for s in REF_SEEDS:
        d = golden(f"{stem}_s{s}.npz")
        assert int(d["seed"]) == s and int(d["steps"]) == WORKLOADS[workload][6]
        assert int(d["multi_steps"]) == WORKLOADS[workload][4] if "multi_steps" in d else WORKLOADS[workload][4] == 1


@pytest.mark.parametrize("workload", ["gbm", "gbm_td3_n5"])
def test_gbm_band_is_one_sided_from_the_reference_median(golden, workload):
    (g0, g1), (l0, l1) = bands(golden, workload)
    med = {"gbm": (2.502, 0.679), "gbm_td3_n5": (13.796, 3.820)}[workload]  # the reference seeds' medians
    assert g0 == pytest.approx(med[0], abs=1e-3) and g1 == float("inf")
    assert l0 == pytest.approx(med[1], abs=1e-3) and l1 == pytest.approx(4.95)
