"""Deterministic CPU stand-in for rlmd_amd.trainer.VecTrainer (test
infrastructure): seed-determined outputs in the trainer's interface, so the host
logic around it (run_experiment's sharding, logs, checkpoints) runs without a
GPU, and make_golden.aggregate_fixtures can hand its log files to the
reference's readers."""
import numpy as np
import torch


class StubTrainer:
    def __init__(self, seed, init_logtemp=0.0, risk_dim=4):
        self.seed, self.t, self.risk_dim = seed, 0, risk_dim

    def step(self):
        self.t += 1

    def flush_stats(self):
        return torch.tensor([float(self.t), 1.5 * self.t + self.seed, 10.0 * self.t, 0.0])

    def last_stats(self, shadow=False):
        st = np.full(16, self.seed + 0.001 * self.t)
        st[8:10] = 0.5 + 0.01 * self.seed  # tail indices (< 1: shadow means defined)
        st[2:4], st[4:6] = 1.0, 5.0 + self.seed  # critic min / max
        return st

    def episode_log(self, cap):
        pass

    def drain_episodes(self):
        """Two finished episodes per vector step, seed-tagged scores."""
        r = self.risk_dim
        rows = np.array([[self.t, lane, self.seed + 0.01 * lane, 3.0 + lane] + [float(k) for k in range(r)]
                         for lane in (0, 5)])
        return rows, 0

    def evaluate(self, n_eval=100, max_steps=100):
        rew = 1.0 + 0.001 * (np.arange(n_eval, dtype=np.float64) + 100 * self.seed + self.t)
        risk = np.tile(rew[:, None], (1, self.risk_dim))
        risk[:, 3] = 0.25 + 0.001 * np.arange(n_eval)  # leverage column
        return {"reward": rew, "steps": np.full(n_eval, 7), "risk": risk}
