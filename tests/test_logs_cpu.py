"""Experiment logs in the reference layout, CPU only.

save_directory / multi_log_dim / market_log_dim vs the reference's own
tools/utils.py outputs (tests/golden/logs.npz); ExperimentLog array shapes,
row layout and the reference's trial truncation (rl_multiplicative.py:437-450)."""
import os

import numpy as np

from rlmd_amd import logs


def _inputs(c):
    env_id, dyn, algo, sd, lf, buf, ms, ncs, nt, test, n = c
    return {"env_id": env_id, "dynamics": dyn, "algo": algo, "s_dist": sd, "loss_fn": lf, "critic_mean_type": "E",
            "buffer": float(buf), "multi_steps": int(ms), "n_cumsteps": float(ncs), "n_trials": int(nt),
            "test_agent": test == "True", "trial": 2}, int(n)


def test_names_and_dims_match_reference(golden):
    g = golden("logs.npz")
    for i, c in enumerate(g["cases"]):
        inp, n = _inputs(c)
        assert logs.save_directory(inp, results=True) == str(g["results"][i])
        assert logs.save_directory(inp, results=False) == str(g["models"][i])
        dim = logs.market_log_dim(inp["env_id"], n) if inp["dynamics"] == "MKT" else logs.multi_log_dim(inp["env_id"], n)
        assert dim == int(g["risk_dim"][i])


def test_experiment_log_layout_and_truncation(tmp_path):
    lg = logs.ExperimentLog(n_trials=2, n_rows=10, n_evals=3, n_eval=4, risk_dim=5, market=True)
    st = np.arange(16, dtype=np.float32)
    for t, rows in ((0, 3), (1, 6)):
        for k in range(rows):
            lg.log_row(t, 0.5 + k, 1.01, 7.0, st)
    ev = {"reward": np.full(4, 1.02), "steps": np.full(4, 9), "risk_log": np.ones((4, 6))}
    lg.log_eval(1, 2, ev, 0.8, st, 3000)
    d = str(tmp_path / "results" / "x" / "exp")
    m = lg.save(d)
    assert m == 6
    tr = np.load(d + "_trial.npy")
    assert tr.shape == (2, 6, 19) and tr.dtype == np.float32
    np.testing.assert_array_equal(tr[1, 0, 3:14], st[:11])
    assert tr[1, 0, 14] == st[11] and tr[0, 3, 0] == 0
    np.testing.assert_array_equal(tr[1, 0, 15:19], st[12:16])
    e = np.load(d + "_eval.npy")
    assert e.shape == (2, 3, 4, 20)
    np.testing.assert_allclose(e[1, 2, :, [0, 1, 2, 19]], np.array([[0.2] * 4, [1.02] * 4, [9] * 4, [3000] * 4]),
                               rtol=1e-6)
    assert np.load(d + "_eval_risk.npy").shape == (2, 3, 4, 6)
    assert np.load(d + "_trial_risk.npy").shape == (2, 6, 5)


def test_env_ids_follow_reference_naming():
    from rlmd_amd.experiment import env_id

    assert env_id("gbm", "A", 1) == "GBM_InvA_n1"
    assert env_id("coin", "C", 5) == "Coin_InvC_n5"
    assert env_id("dice_sh", "INSURED") == "Dice_SH_INSURED_n1"
    assert env_id("dice_sh", "B") == "Dice_SH_InvB_n1"
    assert env_id("market", "B", obs_days=5) == "SNP_InvB_D5_T1"


def test_reference_readers_accept_build_logs(golden, tmp_path, monkeypatch):
    """tests/golden/aggregate.npz holds what the reference's own readers
    (tools/aggregate_data.py:289-447: mul_inv_aggregate + mul_inv_n_summary, the
    inputs of scripts/gen_figures.py:344-359) returned on log files written by
    this build's run_experiment (make_golden.write_build_logs: Coin_InvA/B/C,
    deterministic stub trainer).  Rewriting those files now must give the same
    arrays the readers consumed: eval || eval_risk per investor, and the summary's
    reward / leverage / loss / tail / shadow columns at the readers' offsets."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("mg", os.path.join(os.path.dirname(__file__), "golden",
                                                                     "make_golden_logs.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    monkeypatch.chdir(tmp_path)
    paths = mg.write_build_logs(".")
    g = golden("aggregate.npz")
    agg = g["aggregate"]
    n_eval, n_tr = mg.AGG_INPUTS["n_eval"], mg.AGG_INPUTS["n_trials"]
    for i, p in enumerate(paths):
        ev, rk = np.load(p + "_eval.npy"), np.load(p + "_eval_risk.npy")
        both = np.concatenate([ev, rk], axis=3)
        np.testing.assert_array_equal(agg[i, :, :, :, 1:both.shape[3]], both[..., 1:])  # col 0: wall time
        for t in range(ev.shape[1]):
            for n in range(n_tr):
                sl = slice(n * n_eval, (n + 1) * n_eval)
                np.testing.assert_array_equal(g["summary_reward"][i, t, sl], ev[n, t, :, 1])
                np.testing.assert_array_equal(g["summary_lev"][i, t, sl], rk[n, t, :, 3])
                np.testing.assert_array_equal(g["summary_loss"][i, t, 2 * n:2 * n + 2], ev[n, t, 0, 3:5])
                np.testing.assert_array_equal(g["summary_tail"][i, t, 2 * n:2 * n + 2], ev[n, t, 0, 11:13])
                np.testing.assert_array_equal(g["summary_shadow"][i, t, 2 * n:2 * n + 2], ev[n, t, 0, 9:11])
    assert np.all(np.isfinite(g["summary_keqv"]))  # the reference's equivalence solver ran on them
