"""The reference seeds the GPU convergence test compares against
(tests/test_converge_gpu.py): five reference seeds per workload (ten for
GBM_InvA SAC, C2's env; Dice_SH_InvA TD3 / MSE, C3's env and loss; GBM_InvA
TD3 with 5-step returns, C5), made by
the reference's own rl_multiplicative / rl_market loops
(tests/golden/run_reference_loop.py; C5 with 5-step returns, C4 through
market_env); the ranges of their last-third statistics (growth %/step,
leverage), as its docstring states them."""
import pytest

from tests.test_converge_gpu import REF_SEED_SETS, REF_SEEDS, WORKLOADS, ref_stats

BAND = {  # (growth min, max %/step), (lev min, max): last thirds of the five seeds
    "coin": ((-0.178, 0.315), (0.013, 0.105)),
    "dice": ((-0.136, 0.303), (-0.040, 0.123)),
    "gbm": ((0.508, 8.464), (0.129, 2.343)),  # ten seeds
    "dice_sh": ((-4.750, 2.037), (0.863, 0.929)),
    "dice_sh_a_mse": ((-47.535, 1.895), (-0.027, 1.980)),  # ten seeds
    "dice_sh_a_hub": ((-16.640, 0.756), (0.263, 1.980)),
    "gbm_td3_n5": ((-23.365, 37.114), (-4.950, 4.421)),  # ten seeds
    "market": ((1.131, 5.921), (0.207, 1.708)),
}


@pytest.mark.parametrize("workload", sorted(WORKLOADS))
def test_reference_band(golden, workload):
    st = ref_stats(golden, workload)
    seeds = REF_SEED_SETS.get(workload, REF_SEEDS)
    assert len(st) == len(seeds) == (10 if workload in REF_SEED_SETS else 5)
    (g0, g1), (l0, l1) = BAND[workload]
    assert min(g for g, _ in st) == pytest.approx(g0, abs=1e-3)
    assert max(g for g, _ in st) == pytest.approx(g1, abs=1e-3)
    assert min(lv for _, lv in st) == pytest.approx(l0, abs=1e-3)
    assert max(lv for _, lv in st) == pytest.approx(l1, abs=1e-3)
    stem = WORKLOADS[workload][3]
    for s in seeds:
        d = golden(f"{stem}_s{s}.npz")
        assert int(d["seed"]) == s and int(d["steps"]) == WORKLOADS[workload][6]
        assert int(d["multi_steps"]) == WORKLOADS[workload][4] if "multi_steps" in d else WORKLOADS[workload][4] == 1
