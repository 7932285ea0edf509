"""Probe (GPU): two C2 seeds on one MI355X — does a stream priority split, or the
full CU budget for both, raise the pair's throughput over SeedGroup's default
(CU-masked streams, each seed's learner on half the CUs)?

    python tools/probe/seeds_priority.py [steps]

Prints, per variant, the group's ms per vector step and the ratio to one seed."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from rlmd_amd.trainer import SeedGroup, VecTrainer

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    kw = dict(env="gbm", investor="A", n_lanes=65536, algo="SAC", precision="bf16", warmup_steps=0,
              smoothing_window=0, replay_capacity=1 << 20, k_updates=8)
    dev = "cuda:0"

    def timed(step, sync):
        for _ in range(5):
            step()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        return (time.perf_counter() - t0) / steps * 1e3

    one = VecTrainer(seed=7, device=dev, **kw)
    ms1 = timed(one.step, torch.cuda.synchronize)
    del one
    print(f"one seed: {ms1:.4f} ms per step", flush=True)
    variants = [
        ("cu streams, half CU budget (default)", dict(streams="cu")),
        ("cu streams, full CU budget", dict(streams="cu", cu_budget=None)),
        ("torch streams, priorities high / low, half budget",
         dict(streams=[torch.cuda.Stream(device=dev, priority=-1), torch.cuda.Stream(device=dev, priority=0)])),
        ("torch streams, priorities high / low, full budget",
         dict(streams=[torch.cuda.Stream(device=dev, priority=-1), torch.cuda.Stream(device=dev, priority=0)],
              cu_budget=None)),
    ]
    for name, v in variants:
        grp = SeedGroup([420, 1420], device=dev, **v, **kw)
        ms = timed(grp.step, grp.synchronize)
        print(f"{name}: {ms:.4f} ms per group step, {2 * ms1 / ms:.3f} x one seed", flush=True)
        del grp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
