"""Experiment: is the C2 training loop host-bound?  After a device sync (empty
queue), time the host-side enqueue of a few tr.step() calls (no sync in
between), then the device time of the same steps; both per step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from rlmd_amd import _abi
    from rlmd_amd.trainer import VecTrainer

    dev = torch.device("cuda:0")
    tr = VecTrainer(env="gbm", investor="A", n_lanes=65536, algo="SAC", k_updates=8, replay_capacity=1 << 20,
                    seed=420, warmup_steps=0, smoothing_window=0, precision="bf16", device=dev, init_seed=420)
    for _ in range(10):
        tr.step()
    torch.cuda.synchronize()
    for prof in (0, 1):
        tr.profile(prof)
        for n in (1, 3, 10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                tr.step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"profile {prof} steps {n}: host enqueue {1e6 * (t1 - t0) / n:8.1f} us/step, "
                  f"wall {1e6 * (t2 - t0) / n:8.1f} us/step", flush=True)
        tr.profile(0)


if __name__ == "__main__":
    main()
