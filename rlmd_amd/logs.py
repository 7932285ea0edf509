"""Experiment logs in the reference's .npy layout.

The reference drivers keep four float32 arrays per (algo, loss, multi-step)
experiment and save them next to each other (scripts/rl_multiplicative.py:
124-152, :437-450; scripts/rl_market.py has the same shapes with the market
risk width), named by tools/utils.py:170-220 (save_directory):

  <dir>_trial.npy       [n_trials, n_rows, 19]    time, score, steps, loss[11], logtemp, loss_params[4]
  <dir>_eval.npy        [n_trials, n_evals, n_eval, 20]   time, reward, steps, loss[11], logtemp,
                                                   loss_params[4], cum_steps   (eval_episodes.py:267-273, :535-543)
  <dir>_trial_risk.npy  [n_trials, n_rows, risk_dim]
  <dir>_eval_risk.npy   [n_trials, n_evals, n_eval, risk_dim]  (market: [gap, risk...])

so tools/aggregate_data.py and the plotting scripts read this build's output
unchanged.  Trial rows are per finished episode as in the reference (the
device episode log of the fused train step: final reward, length, last risk
vector; the learner statistics of the vector step the episode ended in; time =
length x that interval's wall time per vector step).  ``log_row`` keeps the
older aggregate mode (one row per logging interval: mean final reward and
length of the episodes that ended in it, risk = NaN).  Evaluation rows are per
episode, exactly as the reference's.
"""
import os

import numpy as np


def save_directory(inputs, results=True):
    """tools/utils.py:170-220: the experiment's file stem."""
    step_exp = int(len(str(int(inputs["n_cumsteps"]))) - 1)
    buff_exp = int(len(str(int(inputs["buffer"]))) - 1)
    dyna = {"A": "additive/", "M": "multiplicative/", "MKT": "market/", "GUD": "guidance/"}[inputs["dynamics"]]
    parts = [
        "./results/", dyna, "data/", inputs["env_id"] + "/", inputs["env_id"] + "--", inputs["dynamics"] + "_",
        inputs["algo"] + "-", inputs["s_dist"], "_" + inputs["loss_fn"], "-" + str(inputs["critic_mean_type"]),
        "_B" + str(int(inputs["buffer"]))[0:2] + "e" + str(buff_exp - 1), "_M" + str(inputs["multi_steps"]),
        "_S" + str(int(inputs["n_cumsteps"]))[0:2] + "e" + str(step_exp - 1), "_N" + str(inputs["n_trials"]),
    ]
    if not results:
        parts[2] = "models/"
        parts.append("t" + str(inputs["trial"]))
    if inputs.get("test_agent"):
        parts[1] = "test_" + parts[1]
    return "".join(parts)


def multi_log_dim(env_id, n_gambles):
    """tools/utils.py:254-281."""
    dim = 4 + (n_gambles if n_gambles > 1 else 0)
    dim += 1 if "_InvB" in env_id else 0
    dim += 2 if "_InvC" in env_id else 0
    return 4 + 2 + 1 if "_SH" in env_id else dim


def market_log_dim(env_id, n_assets):
    """tools/utils.py:284-307."""
    dim = 4 + (n_assets if n_assets > 1 else 0)
    dim += 1 if "_InvB" in env_id else 0
    dim += 2 if "_InvC" in env_id else 0
    return dim


class ExperimentLog:
    """The four arrays of one experiment, filled trial by trial."""

    def __init__(self, n_trials, n_rows, n_evals, n_eval, risk_dim, market=False, max_rows=1 << 22):
        self.trial = np.zeros((n_trials, n_rows, 19), dtype=np.float32)
        self.eval = np.zeros((n_trials, n_evals, n_eval, 20), dtype=np.float32)
        self.trial_risk = np.zeros((n_trials, n_rows, risk_dim), dtype=np.float32)
        # eval_market logs [gap, risk...] (eval_episodes.py:542-543)
        self.eval_risk = np.zeros((n_trials, n_evals, n_eval, risk_dim + (1 if market else 0)), dtype=np.float32)
        self.market = market
        self.rows = np.zeros(n_trials, dtype=np.int64)
        # per-episode rows grow with lanes x steps / episode length (the reference's
        # single stream never sees this): bounded, (19 + risk) x 4 B per row per trial
        self.max_rows = int(max_rows)

    def grow(self, n_rows):
        """Widen the trial arrays to at least n_rows rows per trial (zero rows),
        doubling up to max_rows."""
        cur = self.trial.shape[1]
        if n_rows <= cur:
            return
        if n_rows > self.max_rows:
            raise RuntimeError(f"trial log needs {n_rows} rows per trial > max_rows {self.max_rows} "
                               f"({self.trial.shape[0]} trials x {19 + self.trial_risk.shape[2]} x 4 B per row): "
                               "log one aggregate row per interval (episode_rows=False) or raise the bound")
        t = np.zeros((self.trial.shape[0], n_rows, 19), dtype=np.float32)
        r = np.zeros((self.trial.shape[0], n_rows, self.trial_risk.shape[2]), dtype=np.float32)
        t[:, :cur], r[:, :cur] = self.trial, self.trial_risk
        self.trial, self.trial_risk = t, r

    def log_episodes(self, trial, seconds, score, steps, stats16, risk):
        """One row per finished episode (rl_multiplicative.py:275-283, :400-414):
        [time, score, steps, loss[11], logtemp, loss_params[4]] with the learner
        statistics of the vector step the episodes ended in, and each episode's
        own last risk vector."""
        n = len(score)
        if n == 0:
            return
        i = int(self.rows[trial])
        if i + n > self.trial.shape[1]:
            self.grow(max(min(2 * self.trial.shape[1], self.max_rows), i + n))
        st = np.asarray(stats16, dtype=np.float64)
        t = self.trial[trial, i:i + n]
        t[:, 0], t[:, 1], t[:, 2] = seconds, score, steps
        t[:, 3:14] = st[:11]
        t[:, 14] = st[11]
        t[:, 15:19] = st[12:16]
        self.trial_risk[trial, i:i + n] = np.asarray(risk, dtype=np.float64)[:, :self.trial_risk.shape[2]]
        self.rows[trial] += n

    def log_row(self, trial, seconds, score, steps, stats16, risk=None):
        """One trial row: [time, score, steps, loss[11], logtemp, loss_params[4]] (rl_multiplicative.py:402-413)."""
        i = self.rows[trial]
        if i >= self.trial.shape[1]:
            return
        st = np.asarray(stats16, dtype=np.float64)
        self.trial[trial, i, 0:3] = (seconds, score, steps)
        self.trial[trial, i, 3:14] = st[:11]
        self.trial[trial, i, 14] = st[11]
        self.trial[trial, i, 15:19] = st[12:16]
        self.trial_risk[trial, i] = np.nan if risk is None else risk
        self.rows[trial] += 1

    def log_eval(self, trial, eval_run, ev, seconds, stats16, cum_steps):
        """One evaluation event: per episode [time, reward, steps, loss[11], logtemp,
        loss_params[4], cum_steps] and its risk row (eval_episodes.py:267-273, :535-543).
        ev: VecTrainer.evaluate / evaluate_market output.  The reference stamps each
        episode's own wall time; one launch runs them all, so each gets the event's
        time divided evenly."""
        n = len(ev["reward"])
        st = np.asarray(stats16, dtype=np.float64)
        e = self.eval[trial, eval_run, :n]
        e[:, 0] = seconds / n
        e[:, 1] = ev["reward"]
        e[:, 2] = ev["steps"]
        e[:, 3:14] = st[:11]
        e[:, 14] = st[11]
        e[:, 15:19] = st[12:16]
        e[:, 19] = cum_steps
        self.eval_risk[trial, eval_run, :n] = ev["risk_log"] if self.market else ev["risk"]

    def save(self, directory):
        """Truncate the trial arrays to the longest trial (rl_multiplicative.py:437-445)
        and write the four .npy files."""
        os.makedirs(os.path.dirname(directory), exist_ok=True)
        counts = [int(np.min(np.where(self.trial[t, :, 0] == 0)[0])) if (self.trial[t, :, 0] == 0).any()
                  else self.trial.shape[1] for t in range(self.trial.shape[0])]
        m = max(counts)
        np.save(directory + "_trial.npy", self.trial[:, :m, :])
        np.save(directory + "_eval.npy", self.eval)
        np.save(directory + "_trial_risk.npy", self.trial_risk[:, :m, :])
        np.save(directory + "_eval_risk.npy", self.eval_risk)
        return m


def shadow_equiv(mean, alpha, cmin, cmax, min_mul=1.0, device="cuda:0"):
    """tools/aggregate_data.py:441-447's keqv over whole arrays on the device
    (rlmd_shadow_equiv): the max multiplier equating the shadow and empirical
    means, 1 where the tail index is >= 1.  Inputs broadcast to one shape."""
    import torch

    from . import _abi

    arrs = np.broadcast_arrays(*(np.asarray(x, dtype=np.float64) for x in (mean, alpha, cmin, cmax)))
    shape = arrs[0].shape
    t = [torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(device) for a in arrs]
    out = torch.empty_like(t[0])
    P = _abi.ptr
    _abi.check(_abi.lib().rlmd_shadow_equiv(P(t[0]), P(t[1]), P(t[2]), P(t[3]), float(min_mul), t[0].numel(), P(out),
                                            _abi.stream_ptr()))
    return out.cpu().numpy().reshape(shape)
