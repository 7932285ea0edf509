"""The N>1 path of bench.py on CPU: world_size 2 over gloo (127.0.0.1).

Ranks are independent seed shards with no data-path collective; the only
exchange is bench.reduce_ranks at logging time (max wall time + all_gather of
the per-rank log slabs).  The whole-job value must be sum(steps) / max(time)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    ep = torch.tensor([3.0 + rank, 1.5 * (rank + 1), 40.0 + rank, 7.0])
    t_max, slab = bench.reduce_ranks(1.0 + 0.25 * rank, ep, 65536.0 * 50, world, torch.device("cpu"))
    out[rank] = (t_max, slab.tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_ranks_world2_gloo():
    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        t_max, slab = res[rank]
        assert t_max == pytest.approx(1.25)  # max over ranks
        assert [row[0] for row in slab] == [3.0, 4.0]  # rank-ordered gather
        assert sum(row[4] for row in slab) / t_max == pytest.approx(2 * 65536 * 50 / 1.25)
    assert res[0][1] == res[1][1]  # every rank sees the same slabs


def test_single_rank_no_collective():
    import bench

    t_max, slab = bench.reduce_ranks(2.0, torch.zeros(4), 10.0, 1, torch.device("cpu"))
    assert t_max == 2.0 and slab.shape == (1, 5) and slab[0, 4] == 10.0


from tests.stub_trainer import StubTrainer as _StubTrainer  # noqa: E402


def _exp_worker(rank, world, port, root, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rlmd_amd.experiment import run_experiment

    path, lg = run_experiment(env="coin", investor="A", n_trials=5, n_cumsteps=40, eval_freq=20, n_eval=6,
                              log_every=10, seed=3, results_root=root, trainer_factory=_StubTrainer,
                              checkpoint=False)
    out[rank] = (path, lg.trial.tolist(), lg.eval.tolist(), lg.rows.tolist())
    dist.barrier()
    dist.destroy_process_group()


def test_run_experiment_trial_shards_world2_gloo(tmp_path):
    """Trials 0..4 shard as t % 2 over two gloo ranks; after the one all_gather
    every rank holds all five trials, identical to a single-process run, and
    rank 0 alone wrote the .npy files."""
    import numpy as np

    from rlmd_amd.experiment import run_experiment

    world, port = 2, _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_exp_worker, args=(world, port, str(tmp_path / "mr"), out), nprocs=world, join=True)
        res = dict(out)
    _, ref = run_experiment(env="coin", investor="A", n_trials=5, n_cumsteps=40, eval_freq=20, n_eval=6,
                            log_every=10, seed=3, results_root=str(tmp_path / "one"), trainer_factory=_StubTrainer,
                            checkpoint=False)
    for rank in range(world):
        path, trial, ev, rows = res[rank]
        np.testing.assert_array_equal(np.array(trial, np.float32)[..., 1:], ref.trial[..., 1:])
        np.testing.assert_array_equal(np.array(ev, np.float32)[..., 1:], ref.eval[..., 1:])
        assert rows == ref.rows.tolist() == [8] * 5  # 4 drains x 2 episodes
    # eval reward of episode 0 at step 20 / 40 is 1 + 0.001 (100 seed + step), seed = 3 + trial
    assert np.array(res[0][2])[4, 1, 0, 1] == np.float32(1 + 0.001 * (100 * 7 + 40))  # trial 4 (rank 0)
    assert np.array(res[1][2])[3, 0, 0, 1] == np.float32(1 + 0.001 * (100 * 6 + 20))  # trial 3 came from rank 1
    assert os.path.exists(res[0][0] + "_trial.npy")
    saved = np.load(res[0][0] + "_eval.npy")
    np.testing.assert_array_equal(saved[..., 1:], ref.eval[..., 1:])
