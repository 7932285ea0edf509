"""Several seeds per GPU (rlmd_amd.trainer.SeedGroup): T = 2 and 4
independent trainers on their own HIP streams, stepped together, each
bit-equal to the same seed run alone — replay ring rows, lane wealth / time,
learner parameters and statistics — for the C2 shape (GBM_InvA, SAC 256/256
bf16, fused acting + env) and the C4 shape (Market_InvA_D1 on stooq_snp).  The
solo run takes the group's CU budget (rlmd_agent_set_cu_budget): the budget
decides the learner's column split, which changes f32 summation order."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _state(tr, steps, n):
    from rlmd_amd import _abi

    N, S, A = n, tr.env.state_dim, tr.env.action_dim
    rows = N * steps
    dev = tr.device
    s, s2 = torch.empty(rows, S, device=dev), torch.empty(rows, S, device=dev)
    a, r = torch.empty(rows, A, device=dev), torch.empty(rows, device=dev)
    d = torch.empty(rows, dtype=torch.uint8, device=dev)
    _abi.check(_abi.lib().rlmd_replay_read(tr.replay.h, 0, rows, _abi.ptr(s), _abi.ptr(a), _abi.ptr(r), _abi.ptr(s2),
                                           _abi.ptr(d), _abi.stream_ptr()))
    w, t = tr.env.lane_state()
    return {"s": s.cpu().numpy(), "a": a.cpu().numpy(), "r": r.cpu().numpy(), "s2": s2.cpu().numpy(),
            "d": d.cpu().numpy(), "w": w, "t": t, "p": tr.agent.params.cpu().numpy().copy(),
            "tg": tr.agent.target.cpu().numpy().copy(), "st": tr.stats.cpu().numpy().copy()}


def _kw(golden, config):
    if config == "c2":
        return dict(env="gbm", investor="A", n_lanes=8192, algo="SAC")
    prices = golden("stooq_snp.npz")["prices"]
    return dict(env="market", investor="A", n_lanes=4096, algo="SAC", prices=prices, obs_days=1, time_length=1000,
                shuffle_days=5, sample_days=1000 + 250 + 1 + 20 - 1)


@pytest.mark.parametrize("config,T,streams", [("c2", 2, "pool"), ("c2", 4, "pool"), ("c4", 2, "pool"), ("c4", 4, "pool"),
                                              ("c2", 3, "hip"), ("c2", 3, "cu"), ("c2", 3, "cu_split"),
                                              ("c4", 4, "cu_split")])
def test_seed_group_bit_equal_to_solo(golden, dev, config, T, streams):
    """streams="hip": the group's streams come from the library's runtime
    (rlmd_stream_create) instead of torch's pool; "cu" / "cu_split": CU-masked
    streams (rlmd_stream_create_cu, every CU / a 1/T interleaved share each).
    A CU mask only restricts where workgroups run, so results stay bit-equal."""
    from rlmd_amd.trainer import SeedGroup, VecTrainer

    steps, K = 6, 4
    kw = dict(_kw(golden, config), k_updates=K, replay_capacity=1 << 16, warmup_steps=2, smoothing_window=4,
              precision="bf16")
    seeds = [420 + i for i in range(T)]
    grp = SeedGroup(seeds, device=dev, streams=streams, **kw)
    for _ in range(steps):
        grp.step()
    grp.synchronize()
    got = [_state(tr, steps, kw["n_lanes"]) for tr in grp.trainers]
    assert all(tr.last_fused() for tr in grp.trainers)  # the post-window steps fused, per handle
    for i, s in enumerate(seeds):
        solo = VecTrainer(seed=s, init_seed=s, device=dev, cu_budget=grp.cu_budget, **kw)
        for _ in range(steps):
            solo.step()
        torch.cuda.synchronize()
        ref = _state(solo, steps, kw["n_lanes"])
        for key in ref:
            np.testing.assert_array_equal(got[i][key], ref[key], err_msg=f"seed {s} {key}")
        del solo
    # the seeds differ from each other (independent draws, inits)
    assert not np.array_equal(got[0]["p"], got[1]["p"])
