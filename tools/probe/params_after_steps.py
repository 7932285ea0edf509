"""Probe (GPU): run C2 (65,536 GBM lanes, SAC 256/256 bf16, K = 8) for a few vector
steps from a fixed seed and save the agent's parameters, the replay ring's actions
and the lanes' wealth — to compare two library builds bit for bit:

    RLMD_LIB_PATH=<lib> python tools/probe/params_after_steps.py out.npz [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch

    from rlmd_amd.trainer import VecTrainer

    out, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tr = VecTrainer("gbm", "A", 65536, algo="SAC", k_updates=8, replay_capacity=1 << 20, seed=3, init_seed=3,
                    warmup_steps=0, smoothing_window=0, precision="bf16", device="cuda:0")
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    w, t = tr.env.lane_state()
    np.savez(out, params=tr.agent.params.cpu().numpy(), target=tr.agent.target.cpu().numpy(),
             wealth=np.asarray(w), stats=tr.last_stats())
    print("saved", out)


if __name__ == "__main__":
    main()
