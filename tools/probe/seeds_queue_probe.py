"""Seeds per GPU vs the placement of their streams on the process's hardware
queues: before a SeedGroup of T C2 trainers, create and use
`offset` extra torch streams, so the group's streams take other pool slots and
(HIP's round-robin) other hardware queues.  Prints one JSON line per (T, offset):
the group's env steps/s over one seed alone.

    python tools/probe/seeds_queue_probe.py [--T 2,3,4] [--offsets 0,1,2,3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from rlmd_amd.trainer import SeedGroup, VecTrainer

    ap = argparse.ArgumentParser()
    ap.add_argument("--T", default="2,3,4")
    ap.add_argument("--offsets", default="0,1,2,3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--streams", default="pool", help="SeedGroup streams: pool (torch) or hip (rlmd_stream_create)")
    args = ap.parse_args()
    dev = "cuda:0"
    kw = dict(env="gbm", investor="A", n_lanes=65536, algo="SAC", k_updates=8, replay_capacity=1 << 20,
              warmup_steps=0, smoothing_window=0, precision="bf16")
    solo = VecTrainer(seed=7, init_seed=7, device=dev, **kw)
    for _ in range(5):
        solo.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solo.step()
    torch.cuda.synchronize()
    one = 65536 * args.steps / (time.perf_counter() - t0)
    del solo
    print(json.dumps({"solo_env_steps_per_s": one}), flush=True)
    keep = []
    for off in [int(v) for v in args.offsets.split(",")]:
        for T in [int(v) for v in args.T.split(",")]:
            extra = [torch.cuda.Stream(device=dev) for _ in range(off)]
            for st in extra:  # bind each extra stream by using it
                with torch.cuda.stream(st):
                    torch.zeros(1, device=dev).add_(1)
            keep += extra
            grp = SeedGroup([420 + 1000 * i for i in range(T)], device=dev, streams=args.streams, **kw)
            for _ in range(5):
                grp.step()
            grp.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                grp.step()
            grp.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"T": T, "offset": off, "streams": args.streams, "vs_one_seed": T * 65536 * args.steps / dt / one,
                              "ms_per_group_step": 1e3 * dt / args.steps}), flush=True)
            del grp
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
