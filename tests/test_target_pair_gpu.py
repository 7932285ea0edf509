"""TD3 target pairing (learn.hip PairCtl, rows.hip fwd_rows_kernel npair / y0):
when an update changes no target network (td3_target_critic_update = 2,
td3_target_actor_update = 2, main.py:243-244), the next update's target path —
target actor on its s', clipped noise at its counter, both target critics — runs
in the current update's forward launch.  Same kernel code on the same
parameters: the training loop must be bit-identical with and without it
(RLMD_TARGET_PAIR=1 against 0), at C3's shape (Dice_SH_InvA) and C5's (GBM, 5-step
returns), through the warm-up / smoothing window into policy steps.
Reference: algos/algo_td3.py:363-531 (learn), :302-361 (the target)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(dev, env, ms, steps=14, intervals=None):
    from rlmd_amd.trainer import VecTrainer

    n = 4096
    kw = None
    if intervals is not None:
        tc, ta, au = intervals
        kw = dict(target_critic_update=tc, target_actor_update=ta, actor_update_interval=au)
    tr = VecTrainer(env, "A", n_lanes=n, algo="TD3", k_updates=8, replay_capacity=n * 16, seed=3, init_seed=3,
                    warmup_steps=2, smoothing_window=4, precision="bf16", multi_steps=ms, device=dev, agent_kw=kw)
    stats = []
    for _ in range(steps):
        tr.step()
        stats.append(tr.last_stats().copy())
    torch.cuda.synchronize()
    return (tr.agent.params.cpu().numpy().copy(), tr.agent.target.cpu().numpy().copy(), np.stack(stats),
            tr.obs.cpu().numpy().copy())


@pytest.mark.parametrize("env,ms", [("dice_sh", 1), ("gbm", 5)])
def test_td3_target_pairing_is_bit_identical(dev, monkeypatch, env, ms):
    monkeypatch.setenv("RLMD_TARGET_PAIR", "0")
    off = _run(dev, env, ms)
    monkeypatch.setenv("RLMD_TARGET_PAIR", "1")
    on = _run(dev, env, ms)
    for name, x, y in zip(("params", "target", "stats", "obs"), on, off):
        np.testing.assert_array_equal(x, y, err_msg=name)
    assert np.isfinite(on[2][-1][:6]).all()  # real updates ran (not NaN placeholders)
    assert np.abs(on[1]).sum() > 0  # target networks populated


# (target critic, target actor, actor step) intervals: pairing only where an update
# changes no target net; interval 1 never pairs, an actor-only target change can
# fall on a non-critic boundary
@pytest.mark.parametrize("intervals", [(1, 1, 1), (3, 2, 2), (2, 5, 3)])
def test_td3_target_pairing_intervals(dev, monkeypatch, intervals):
    monkeypatch.setenv("RLMD_TARGET_PAIR", "0")
    off = _run(dev, "dice_sh", 1, steps=10, intervals=intervals)
    monkeypatch.setenv("RLMD_TARGET_PAIR", "1")
    on = _run(dev, "dice_sh", 1, steps=10, intervals=intervals)
    for name, x, y in zip(("params", "target", "stats", "obs"), on, off):
        np.testing.assert_array_equal(x, y, err_msg=f"{name} {intervals}")
    assert np.isfinite(on[2][-1][:6]).all()
