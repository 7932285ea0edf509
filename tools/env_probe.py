"""Env-kernel timing probe (GPU): the C2 fused env step with and without the
episode-statistics accumulator, K = 0 learner updates.  Prints phase times."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from rlmd_amd.trainer import VecTrainer


def run(tr, steps=50):
    torch.cuda.synchronize()
    tr.profile(1)
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    ms, cnt = tr.profile_read()
    tr.profile(0)
    return [ms[i] / max(cnt[i], 1) for i in range(3)]


for fam, inv in [("gbm", "A"), ("dice_sh", "A")]:
    tr = VecTrainer(env=fam, investor=inv, n_lanes=65536, algo="SAC", k_updates=0, replay_capacity=1 << 20,
                    seed=420, warmup_steps=0, smoothing_window=0, device="cuda:0")
    for _ in range(10):
        tr.step()
    print(fam, "with ep_stats  act/env/learn ms", run(tr))
    tr.ep_stats = None
    print(fam, "no ep_stats    act/env/learn ms", run(tr))
