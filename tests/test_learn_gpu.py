"""HIP learn() (SAC / TD3) vs the reference's learn() and the oracle — GPU only.

fp32 mode (exact-f32 MFMA operands): loss statistics within 1e-4 relative;
parameters after each update within 2e-6 absolute of the reference / oracle
(Adam steps are lr = 3e-4..1e-3, so < 1 % of one step) on >= 99.9 % of
entries and within 10 % of one Adam step on all: where |grad| ~ Adam's eps
(1e-8), update = lr*m/(sqrt(v)+eps) turns fp32 summation-order noise of a
cancelling gradient into a visible fraction of lr.
bf16 mode (bf16 MFMA operands, f32 accumulate, f32 master weights) against the
bf16 oracle (oracle/learn.py precision="bf16": the same rounding points as the
fused update kernels): statistics within 1e-4 relative, parameters within 2e-6
on >= 99.9 % of entries and within 10 % of one Adam step on all, over 4
consecutive updates.
"""
import numpy as np
import pytest
import torch

from oracle import learn as ol
from tests.test_oracle_learn import NETS, TNETS, build, sd

pytestmark = pytest.mark.gpu


def device_agent(algo, S, A, h1, h2, B, k, loss, init, precision="fp32", **kw):
    from rlmd_amd.agent import DeviceAgent

    return DeviceAgent(algo, S, A, h1, h2, B, k, loss=loss, precision=precision, init=init, **kw)


def golden_init(g, case):
    out = {}
    for nm, tn in zip(NETS, TNETS):
        out[nm] = [torch.from_numpy(v) for v in sd(g, case + "/init", nm).values()]
        out[tn] = [torch.from_numpy(v) for v in sd(g, case + "/init", tn).values()]
    return out


@pytest.mark.parametrize("case", ["case0", "case1", "case2", "case3", "case4", "case5", "case6"])
def test_learn_matches_reference_golden(golden, dev, case):
    g = golden("learn.npz")
    algo, (S, A, h1, h2, B, k), lay, n, _, _ = build(g, case)
    lt = str(g[case + "/loss_fn"])
    ag = device_agent(algo, S, A, h1, h2, B, k, lt, golden_init(g, case), policy_dist=str(g[case + "/s_dist"]))
    rep = {x: torch.from_numpy(g[f"{case}/replay/{x}"]) for x in ("state", "action", "reward", "next_state", "done")}
    for s in range(int(g[case + "/n_steps"])):
        idx = torch.from_numpy(g[f"{case}/step{s}/idx"])
        if algo == "SAC":
            ea, eb = (torch.from_numpy(g[f"{case}/step{s}/eps_{x}"]) for x in ("next", "cur"))
        else:
            ea, eb = torch.from_numpy(g[f"{case}/step{s}/eps_target"]), None
        st = ag.learn_batch(rep["state"][idx], rep["action"][idx], rep["reward"][idx], rep["next_state"][idx],
                            rep["done"][idx], ea, eb).double().cpu().numpy()
        ref_loss = g[f"{case}/step{s}/loss"]
        np.testing.assert_allclose(st[:11], ref_loss, rtol=1e-4, atol=1e-6, equal_nan=True, err_msg=f"step {s}")
        np.testing.assert_allclose(st[12:16], g[f"{case}/step{s}/loss_params"], rtol=1e-4, atol=1e-6)
        if algo == "SAC":
            np.testing.assert_allclose(st[11], g[f"{case}/step{s}/logtemp"], rtol=1e-5, atol=1e-7)
        ref_p = ol.flatten({nm: sd(g, f"{case}/step{s}", nm) for nm in NETS}, lay, n)
        ref_t = ol.flatten({nm: sd(g, f"{case}/step{s}", tn) for nm, tn in zip(NETS, TNETS)}, lay, n)
        np.testing.assert_allclose(ag.params.cpu().numpy(), ref_p, rtol=0, atol=2e-6, err_msg=f"step {s} params")
        np.testing.assert_allclose(ag.target.cpu().numpy(), ref_t, rtol=0, atol=2e-6, err_msg=f"step {s} targets")


def assert_params_close(got, ref, lr, msg, max_lr_frac=0.1):
    # Adam divides by sqrt(v): a near-zero gradient whose fp32 summation order
    # differs can move one element by a visible fraction of lr, so the bound on
    # the worst element is a fraction of lr and the bulk must agree to 2e-6.
    diff = np.abs(got - ref)
    frac = np.mean(diff <= 2e-6)
    assert frac >= 0.999, f"{msg}: only {frac:.6f} within 2e-6 (max {diff.max():.3g})"
    assert diff.max() <= max_lr_frac * lr, f"{msg}: max diff {diff.max():.3g} > {max_lr_frac:.0%} of lr"


FULL = [("SAC", 5, 1, 256, 256, 512, 256), ("TD3", 6, 2, 400, 300, 200, 100), ("SAC", 6, 2, 256, 256, 512, 256)]


def _random_batch(rng, B, S, A):
    s = torch.from_numpy((rng.random((B, S)) * 3e-14).astype(np.float32))
    a = torch.from_numpy(rng.uniform(-0.99, 0.99, (B, A)).astype(np.float32))
    r = torch.from_numpy(rng.uniform(0.5, 1.5, B).astype(np.float32))
    s2 = torch.from_numpy((rng.random((B, S)) * 3e-14).astype(np.float32))
    d = torch.from_numpy(rng.random(B) < 0.1)
    return s, a, r, s2, d


@pytest.mark.parametrize("algo,S,A,h1,h2,B,k", FULL)
@pytest.mark.parametrize("loss", ["MSE", "HUB", "MAE", "HSC"])
def test_full_size_fp32_matches_oracle(dev, algo, S, A, h1, h2, B, k, loss, max_lr_frac=0.1, s_dist="N", dup=False):
    from rlmd_amd.agent import reference_init

    init = reference_init(algo, S, A, h1, h2, seed=11)
    lay, n = ol.layout(algo, S, A, h1, h2)
    p = ol.flatten({nm: dict(zip([x[0] for x in lay[nm]], [t.numpy() for t in init[nm]])) for nm in NETS}, lay, n)
    t = ol.flatten({nm: dict(zip([x[0] for x in lay[nm]], [t.numpy() for t in init[tn]]))
                    for nm, tn in zip(NETS, TNETS)}, lay, n)
    ora = ol.OracleLearner(algo, S, A, h1, h2, B, k, loss, p, t, s_dist=s_dist)
    ag = device_agent(algo, S, A, h1, h2, B, k, loss, init, policy_dist=s_dist)
    rng = np.random.default_rng(3)
    lo = np.finfo(np.float32).eps - 1.0
    draw = (lambda: rng.uniform(lo, 1.0, (B, A))) if s_dist == "L" else (lambda: rng.standard_normal((B, A)))
    for step in range(4):
        s, a, r, s2, d = _random_batch(rng, B, S, A)
        ea = torch.from_numpy(draw().astype(np.float32))
        eb = torch.from_numpy(draw().astype(np.float32))
        if dup:  # rows 2i + 1 repeat rows 2i: equal losses and actor objectives, ranked by row
            for x in (s, a, r, s2, d, ea, eb):
                x[1::2] = x[0::2]
        st = ag.learn_batch(s, a, r, s2, d, ea, eb if algo == "SAC" else None).double().cpu().numpy()
        loss_o, lt_o, lp_o = ora.learn(s.numpy(), a.numpy(), r.numpy(), s2.numpy(), d.numpy(), ea.numpy(),
                                       eb.numpy() if algo == "SAC" else None)
        np.testing.assert_allclose(st[:11], loss_o, rtol=2e-4, atol=1e-6, equal_nan=True, err_msg=f"step {step}")
        np.testing.assert_allclose(st[12:16], lp_o, rtol=2e-4, atol=1e-6)
        lr = 3e-4 if algo == "SAC" else 1e-3
        assert_params_close(ag.params.cpu().numpy(), ora.P.numpy(), lr, f"step {step} params", max_lr_frac)
        assert_params_close(ag.target.cpu().numpy(), ora.T.numpy(), lr, f"step {step} targets", max_lr_frac)


@pytest.mark.parametrize("algo,S,A,h1,h2,B,k", FULL[:2])
def test_tied_rows_match_oracle(dev, algo, S, A, h1, h2, B, k):
    """Mini-batches of repeated rows: every critic loss and actor objective value
    occurs twice, so the top-k selections break ties by row (the oracle's stable
    argsort, the kernels' (value, row) keys, rlmd_block.h block_rank)."""
    test_full_size_fp32_matches_oracle(dev, algo, S, A, h1, h2, B, k, "MSE", dup=True)


@pytest.mark.parametrize("loss", ["CAU", "TCAU", "CIM", "MSE2", "MSE4", "MSE6"])
def test_remaining_losses_fp32(dev, loss):
    test_full_size_fp32_matches_oracle(dev, "SAC", 5, 1, 256, 256, 512, 256, loss)


@pytest.mark.parametrize("splits", ["4", "1"])
@pytest.mark.parametrize("algo,S,A,h1,h2,B,k", FULL[:2])
def test_fused_optimiser_epilogue(dev, monkeypatch, algo, S, A, h1, h2, B, k, splits):
    """RLMD_FUSE_ADAM=1: the weight-gradient GEMM's last arriving split steps the
    parameters (write-through slabs + arrival tickets; with one split straight from
    the accumulators); same numerics as adam_kernel up to the K-sum order."""
    monkeypatch.setenv("RLMD_FUSE_ADAM", "1")
    monkeypatch.setenv("RLMD_FUSE_SPLITS", splits)
    monkeypatch.setenv("RLMD_NO_FUSED_UPDATE", "1")  # the critic step through the GEMM too
    test_full_size_fp32_matches_oracle(dev, algo, S, A, h1, h2, B, k, "MSE")


@pytest.mark.parametrize("algo,S,A,h1,h2,B,k", FULL[:2])
@pytest.mark.parametrize("loss", ["MSE", "HUB"])
def test_launch_chain_critic_step_matches_oracle(dev, monkeypatch, algo, S, A, h1, h2, B, k, loss):
    """RLMD_NO_FUSED_UPDATE=1: the critic step as row backward + weight-gradient
    GEMM + Adam launches (the path B > 512 takes) against the same oracle."""
    monkeypatch.setenv("RLMD_NO_FUSED_UPDATE", "1")
    test_full_size_fp32_matches_oracle(dev, algo, S, A, h1, h2, B, k, loss)


@pytest.mark.parametrize("s_dist", ["L", "MVN"])
def test_full_size_policy_dists(dev, s_dist):
    """Laplace / MVN samplers through the whole update at full size (SAC 256/256)."""
    test_full_size_fp32_matches_oracle(dev, "SAC", 6, 2, 256, 256, 512, 256, "MSE", s_dist=s_dist)


@pytest.mark.parametrize("algo", ["SAC", "TD3"])
def test_batch_1024_separate_actor_loss(dev, algo):
    """B > 512 routes the actor loss through actor_loss_kernel instead of abwd_rows."""
    # 1024-row sums: twice the reduction length of the 512-row cases
    test_full_size_fp32_matches_oracle(dev, algo, 5, 1, 256, 256, 1024, 512, "MSE", max_lr_frac=0.2)


def bf16_vs_oracle(algo, S, A, h1, h2, B, k, loss, steps=4, seed=5, path="fused"):
    """The headline precision's learner against the bf16 oracle (oracle/learn.py
    precision="bf16"), state rows O(1) so that the bf16 operands carry signal.
    Every oracle update starts from the device's state (parameters, targets,
    Adam moments, Cauchy scales, log alpha): bf16 rounding makes a run chaotic in
    the few elements whose gradient is ~ Adam's eps, so each update is checked on
    its own arithmetic, over consecutive updates (Adam step counts, Polyak and
    TD3's delayed actor steps)."""
    from rlmd_amd.agent import reference_init

    init = reference_init(algo, S, A, h1, h2, seed=seed)
    lay, n = ol.layout(algo, S, A, h1, h2)
    p = ol.flatten({nm: dict(zip([x[0] for x in lay[nm]], [t.numpy() for t in init[nm]])) for nm in NETS}, lay, n)
    t = ol.flatten({nm: dict(zip([x[0] for x in lay[nm]], [t.numpy() for t in init[tn]]))
                    for nm, tn in zip(NETS, TNETS)}, lay, n)
    ora = ol.OracleLearner(algo, S, A, h1, h2, B, k, loss, p, t, precision="bf16", path=path)
    ag = device_agent(algo, S, A, h1, h2, B, k, loss, init, precision="bf16")
    rng = np.random.default_rng(seed + 100)
    lr = 3e-4 if algo == "SAC" else 1e-3
    # elements stepped with an ill-conditioned gradient (|g| < 1e-6, within 100x
    # of Adam's eps): there a one-ulp difference in one of the B summands (an
    # operand an f32 ulp from a bf16 rounding boundary rounds the other way in
    # one of the two) changes m / (sqrt(v) + eps) by a large fraction of a step
    for step in range(steps):
        sc = ag.scalars()
        ora.load_state(ag.params.cpu(), ag.target.cpu(), ag.adam_m.cpu(), ag.adam_v.cpu(), sc["cauchy"],
                       sc["log_alpha"])
        s, a, r, s2, d = _random_batch(rng, B, S, A)
        s = torch.from_numpy(rng.normal(0, 1, (B, S)).astype(np.float32))
        s2 = torch.from_numpy(rng.normal(0, 1, (B, S)).astype(np.float32))
        ea = torch.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
        eb = torch.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
        st = ag.learn_batch(s, a, r, s2, d, ea, eb if algo == "SAC" else None).double().cpu().numpy()
        lo, lt_o, lp_o = ora.learn(s.numpy(), a.numpy(), r.numpy(), s2.numpy(), d.numpy(), ea.numpy(),
                                   eb.numpy() if algo == "SAC" else None)
        np.testing.assert_allclose(st[:11], lo, rtol=1e-4, atol=1e-6, equal_nan=True, err_msg=f"step {step}")
        np.testing.assert_allclose(st[12:16], lp_o, rtol=1e-4, atol=1e-6, err_msg=f"step {step} loss_params")
        if algo == "SAC":
            np.testing.assert_allclose(st[11], lt_o, rtol=1e-5, atol=1e-7)
        g = ora.last_grad.numpy()
        ill = np.abs(np.nan_to_num(g, nan=1.0)) < 1e-6  # this update's ill-conditioned elements
        # bulk: >= 99.9 % of all parameters within 2e-6; well-conditioned elements
        # (|g| >= 1e-6 in this update): all within 10 % of one Adam step
        for nm, got, ref in (("params", ag.params, ora.P), ("targets", ag.target, ora.T)):
            dp = np.abs(got.cpu().numpy() - ref.numpy())
            frac = np.mean(dp <= 2e-6)
            print(f"{algo} {loss} step {step} {nm}: within 2e-6 {frac:.6f}, max {dp.max():.3g}, "
                  f"max well-conditioned {dp[~ill].max():.3g}, ill-conditioned {ill.mean():.5f}")
            assert frac >= 0.999, f"step {step} {nm}: only {frac:.6f} within 2e-6"
            assert dp[~ill].max() <= 0.1 * lr, f"step {step} {nm}: {dp[~ill].max():.3g} > 10 % of lr"


@pytest.mark.parametrize("algo,S,A,h1,h2,B,k", FULL[:2])
@pytest.mark.parametrize("loss", ["MSE", "HUB", "MAE", "HSC"])
def test_bf16_matches_bf16_oracle(dev, algo, S, A, h1, h2, B, k, loss):
    """C2's SAC 256/256 (B = 512) and C3's TD3 400/300 (B = 200) in bf16 through
    the fused update kernels (critic_update_kernel / actor_update_kernel)."""
    bf16_vs_oracle(algo, S, A, h1, h2, B, k, loss)


@pytest.mark.parametrize("algo,S,A,h1,h2,B,k", FULL[:2])
@pytest.mark.parametrize("loss", ["MSE", "HUB"])
def test_bf16_launch_chain_matches_bf16_oracle(dev, monkeypatch, algo, S, A, h1, h2, B, k, loss):
    """RLMD_NO_FUSED_UPDATE=1 (the path every B > 512 takes): cbwd_rows / abwd_rows
    + the weight-gradient GEMM + Adam, against the bf16 oracle's chain rounding."""
    monkeypatch.setenv("RLMD_NO_FUSED_UPDATE", "1")
    bf16_vs_oracle(algo, S, A, h1, h2, B, k, loss, path="chain")


@pytest.mark.parametrize("algo", ["SAC", "TD3"])
def test_nan_guard_sets_status(dev, algo):
    """The reference's NaN guards (tests/test_live_learning.py:29-255) as the
    sticky status word of rlmd_status_poll: a NaN reward in one mini-batch
    makes the critic target NaN (bit 0, *_critic_stability) and the critic
    statistics NaN (bit 1, critic_learning's exit() condition).  Finite batches
    before it leave the word 0; later batches do not clear it."""
    from rlmd_amd import _abi
    from rlmd_amd.agent import reference_init

    S, A, h1, h2, B, k = 5, 1, 64, 48, 64, 32
    ag = device_agent(algo, S, A, h1, h2, B, k, "MSE", reference_init(algo, S, A, h1, h2, seed=3))
    rng = np.random.default_rng(0)

    def batch(nan_row=None):
        s = torch.from_numpy(rng.normal(size=(B, S)).astype(np.float32))
        a = torch.from_numpy(rng.uniform(-0.9, 0.9, (B, A)).astype(np.float32))
        r = torch.from_numpy(rng.normal(1.0, 0.1, B).astype(np.float32))
        if nan_row is not None:
            r[nan_row] = float("nan")
        s2 = torch.from_numpy(rng.normal(size=(B, S)).astype(np.float32))
        d = torch.zeros(B, dtype=torch.uint8)
        e = torch.from_numpy(rng.normal(size=(B, A)).astype(np.float32))
        return s, a, r, s2, d, e, (e.clone() if algo == "SAC" else None)

    for _ in range(3):
        ag.learn_batch(*batch())
    assert ag.status() == (0, -1)
    st = ag.learn_batch(*batch(nan_row=7)).cpu().numpy()
    assert np.isnan(st[0])
    flags, upd = ag.status()
    assert flags & _abi.STATUS_NAN_BATCH and flags & _abi.STATUS_NAN_STATS, flags
    assert upd >= 0
    ag.learn_batch(*batch())
    assert ag.status()[0] == flags  # sticky
    assert ag.scalars()["nan_flag"] == flags


@pytest.mark.parametrize("loss", ["CAU", "TCAU"])
def test_fused_actor_statistics_use_prestep_scalars(dev, monkeypatch, loss):
    """The fused actor step runs its two critic-statistics workgroups beside the
    workgroups that write log_alpha (temperature step) and the Nagy Cauchy scales
    in the same launch.  The scalars live in update-parity slots of LearnState
    (update n reads slot (n - 1) & 1 and writes slot n & 1), so the statistics
    read the starting values without ordering against their writers; their
    statistics, the Cauchy scales (the next
    update's CAU / TCAU loss scale) and log alpha must match the launch chain
    (RLMD_NO_FUSED_ACTOR=1: statistics in abwd_rows' own workgroup, temperature in
    adam_kernel after it) over consecutive SAC updates with a temperature step."""
    from rlmd_amd.agent import reference_init

    S, A, h1, h2, B, k = 5, 1, 256, 256, 512, 256
    init = reference_init("SAC", S, A, h1, h2, seed=21)
    rng = np.random.default_rng(8)
    batches = []
    for _ in range(6):
        s, a, r, s2, d = _random_batch(rng, B, S, A)
        r = r * 3.0  # targets well away from q: the Nagy update moves the scale
        batches.append((s, a, r, s2, d, torch.from_numpy(rng.standard_normal((B, A)).astype(np.float32)),
                        torch.from_numpy(rng.standard_normal((B, A)).astype(np.float32))))
    out = {}
    for mode in ("fused", "chain"):
        if mode == "chain":
            monkeypatch.setenv("RLMD_NO_FUSED_ACTOR", "1")
        ag = device_agent("SAC", S, A, h1, h2, B, k, loss, init)
        rows = []
        for bt in batches:
            st = ag.learn_batch(*bt).double().cpu().numpy().copy()
            sc = ag.scalars()
            rows.append((st, sc["cauchy"], sc["log_alpha"]))
        out[mode] = rows
    for i, ((sf, cf, af), (sc_, cc, ac)) in enumerate(zip(out["fused"], out["chain"])):
        np.testing.assert_allclose(sf[:16], sc_[:16], rtol=1e-5, atol=1e-7, equal_nan=True, err_msg=f"update {i}")
        np.testing.assert_allclose(cf, cc, rtol=1e-5, err_msg=f"update {i} Cauchy scales")
        np.testing.assert_allclose(af, ac, rtol=1e-5, atol=1e-7, err_msg=f"update {i} log alpha")
    # the scales moved: the Nagy update is exercised, not held at its initial 1.0
    assert abs(out["fused"][-1][1][0] - 1.0) > 1e-3
