"""Which of this process's first library-created HIP streams run T C2 seeds
concurrently: creates 9 streams (rlmd_stream_create) in order,
then times a SeedGroup on each listed set of stream numbers (1-based creation
order).  One JSON line per set.

    python tools/probe/seeds_stream_sets.py "1,2,3,4" "1,2,3,5" "6,7,8,9"
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from rlmd_amd.trainer import SeedGroup, VecTrainer, _hip_streams

    dev = "cuda:0"
    kw = dict(env="gbm", investor="A", n_lanes=65536, algo="SAC", k_updates=8, replay_capacity=1 << 20,
              warmup_steps=0, smoothing_window=0, precision="bf16")
    streams = _hip_streams(torch.device(dev), 9)
    solo = VecTrainer(seed=7, init_seed=7, device=dev, **kw)
    for _ in range(5):
        solo.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        solo.step()
    torch.cuda.synchronize()
    one = 65536 * 20 / (time.perf_counter() - t0)
    del solo
    for spec in sys.argv[1:]:
        ids = [int(v) for v in spec.split(",")]
        grp = SeedGroup([420 + 1000 * i for i in range(len(ids))], device=dev, streams=[streams[i - 1] for i in ids],
                        **kw)
        for _ in range(5):
            grp.step()
        grp.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            grp.step()
        grp.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"streams": ids, "vs_one_seed": len(ids) * 65536 * 20 / dt / one,
                          "ms_per_group_step": 1e3 * dt / 20}), flush=True)
        del grp
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
