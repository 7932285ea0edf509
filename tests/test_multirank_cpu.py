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
