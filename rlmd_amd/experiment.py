"""Vectorised counterpart of the reference drivers' trial loop with their logs.

scripts/rl_multiplicative.py:154-450 (and rl_market.py:167-480) run n_trials
independent agents, evaluate every eval_freq steps (100 episodes) with the
critics' shadow means filled in first (loss[6:8] = agent_shadow_mean, :255,
:275), and save the trial / eval logs as .npy under utils.save_directory
(:447-450).  Here one trial is one VecTrainer (its own seed); a "step" is one
vector step over all lanes; trial rows are per finished episode from the
device episode log (rlmd_amd/logs.py), with the trailing-score checkpoints of
:285-293 and the `continue` chain of :172-183; evaluation rows are per episode
as in the reference.

Trials are independent (the reference runs them one after another and shares
nothing but the output arrays), so under torch.distributed they shard over
ranks: trial t runs on rank t % world, each rank on its own GPU, and the only
collective is one all_gather of the four log arrays after the last trial (RCCL
over xGMI on the GPU box, gloo in tests/test_multirank_cpu.py); rank 0 writes
the .npy files.
"""
import os
import time

import numpy as np
import torch

from . import logs

ENV_NAMES = {"coin": "Coin", "dice": "Dice", "gbm": "GBM", "dice_sh": "Dice_SH"}


def env_id(env, investor, n_gambles=1, market_name="SNP", obs_days=1, action_days=1):
    """The reference's inputs["env_id"]: main.py gym_envs name + "_n" + n_gambles
    (rl_multiplicative.py:49-51; Dice_SH_* too), market name + "_D" + obs_days +
    "_T" + action_days (rl_market.py:62-65)."""
    if env == "market":
        return f"{market_name}_Inv{investor}_D{obs_days}_T{action_days}"
    if env == "dice_sh":
        return f"Dice_SH_{investor if investor == 'INSURED' else 'Inv' + investor}_n{n_gambles}"
    return f"{ENV_NAMES[env]}_Inv{investor}_n{n_gambles}"


def _world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def gather_logs(lg, owner, world, device):
    """Two all_gathers: every rank's four log arrays as one flat f32 slab (the
    logs' own dtype: no widening) and the per-trial row counts (int64); trial t
    is taken from rank owner[t].  The trial arrays are first widened to the
    largest row count of any rank (one all_reduce of that count).  The slab is
    n_trials x (rows x (19 + risk) + evals x n_eval x (20 + risk)) x 4 B per
    rank; ExperimentLog.max_rows bounds the rows before the run gets here."""
    import torch.distributed as dist

    width = torch.tensor([lg.trial.shape[1]], dtype=torch.int64, device=device)
    dist.all_reduce(width, op=dist.ReduceOp.MAX)
    lg.grow(int(width.item()))
    parts = [lg.trial, lg.eval, lg.trial_risk, lg.eval_risk]
    flat = torch.from_numpy(np.concatenate([np.asarray(p, np.float32).ravel() for p in parts])).to(device)
    out = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(out, flat)
    rows = torch.from_numpy(lg.rows.astype(np.int64)).to(device)
    rows_out = [torch.empty_like(rows) for _ in range(world)]
    dist.all_gather(rows_out, rows)
    got = [o.cpu().numpy() for o in out]
    got_rows = [o.cpu().numpy() for o in rows_out]
    sizes = [p.size for p in parts]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    for t, r in enumerate(owner):
        src = [got[r][offs[i]:offs[i + 1]].reshape(parts[i].shape) for i in range(len(parts))]
        lg.trial[t], lg.eval[t], lg.trial_risk[t], lg.eval_risk[t] = src[0][t], src[1][t], src[2][t], src[3][t]
        lg.rows[t] = int(got_rows[r][t])
    return lg


class _Checkpoint:
    """rl_multiplicative.py:285-293: save the actor / critics at every new high of
    the trailing mean of the last `trail` episode scores (checked after every
    episode, in episode order; one save per logging interval at most, as all its
    episodes end with the same parameters)."""

    def __init__(self, trail, prefix, floor):
        self.trail, self.prefix, self.best = int(trail), prefix, floor
        self.scores = np.zeros(0)
        self.saves = 0

    def update(self, trainer, scores):
        if len(scores) == 0 or self.prefix is None:
            return False
        allv = np.concatenate([self.scores[-(self.trail - 1):] if self.trail > 1 else self.scores[:0], scores])
        c = np.concatenate([[0.0], np.cumsum(allv)])
        k = len(allv) - len(scores)
        ends = np.arange(k + 1, len(allv) + 1)
        lo = np.maximum(ends - self.trail, 0)
        trail = (c[ends] - c[lo]) / (ends - lo)
        self.scores = allv[-self.trail:]
        if trail.max() > self.best:
            self.best = float(trail.max())
            os.makedirs(os.path.dirname(self.prefix) or ".", exist_ok=True)
            trainer.agent.save(self.prefix)
            self.saves += 1
            return True
        return False


def run_experiment(env="gbm", investor="A", n_gambles=1, algo="SAC", loss="MSE", n_lanes=4096, n_cumsteps=2000,
                   eval_freq=1000, n_eval=100, max_eval_steps=100, n_trials=1, k_updates=1, log_every=1,
                   warmup_steps=1000, smoothing_window=2000, buffer=1_000_000, multi_steps=1, precision="bf16",
                   seed=0, results_root=".", test_agent=True, device="cuda:0", test_days=250,
                   trainer_factory=None, gather_device=None, episode_rows=True, episode_cap=None, trail=50,
                   checkpoint=True, continue_trials=False, max_episode_rows=1 << 22, schedule="updates",
                   **trainer_kw):
    """Train n_trials independent vectorised agents (sharded over the ranks of an
    initialised process group, trial t on rank t % world) and save the
    reference's four log arrays on rank 0; returns (file stem, ExperimentLog),
    the log complete on every rank.

    episode_rows: one trial row per finished episode from the device episode log;
    False: one aggregate row per interval.  A lane finishes at most one episode
    per vector step, so a wave's log slots (episode_cap rows per 64 lanes per
    drain) never overflow when episode_cap >= 64 x the steps between drains:
    the default drains every `log_every` steps with 64 x log_every slots per
    wave up to log_every 64, and beyond that drains every step (64 slots) into a
    host list folded into the row at the log step.  A drain that reports
    dropped rows raises (a lossy log would bias the trial rows and the
    trailing-score checkpoints towards low lanes).  max_episode_rows bounds the
    per-episode trial rows of one trial (host memory and the logging gather:
    (19 + risk) x 4 B per row); a run that exceeds it raises, pointing at
    episode_rows=False (one aggregate row per logging interval).
    warmup_steps / smoothing_window: UNITS depend on `schedule`.  With the
    default schedule="updates" they are the reference's lengths in its env steps
    (one learner update per env step, main.py:256-257) and are converted to the
    same number of learner updates: ceil(steps / k_updates) vector steps
    (trainer.schedule_steps).  With schedule="vector" they are vector steps per
    lane, the unit VecTrainer itself takes (rounds 1-3's behaviour).  Callers
    that passed per-lane vector-step counts before round 4 must pass
    schedule="vector" or their warm-up becomes k_updates times shorter
    ("Units of the warm-up / smoothing arguments").
    checkpoint: trailing-`trail` checkpoints under the reference's models/ path.  continue_trials: inputs["continue"] — trial t starts from
    trial t-1's last checkpoint and final log temperature (run on one rank, as
    the chain is sequential).  trainer_factory(seed, init_logtemp) replaces the
    VecTrainer construction (tests)."""
    world, rank = _world()
    market = env == "market"
    dyn = "MKT" if market else "M"
    eid = env_id(env, investor, n_gambles, obs_days=trainer_kw.get("obs_days", 1))
    inputs = {"env_id": eid, "dynamics": dyn, "algo": algo, "s_dist": trainer_kw.get("s_dist", "N"),
              "loss_fn": loss, "critic_mean_type": "E", "buffer": buffer, "multi_steps": multi_steps,
              "n_cumsteps": n_cumsteps, "n_trials": n_trials, "test_agent": test_agent}
    n_rows = (n_cumsteps + log_every - 1) // log_every
    n_evals = n_cumsteps // eval_freq
    rdim = (logs.market_log_dim(eid, n_gambles) if market else logs.multi_log_dim(eid, n_gambles))
    lg = logs.ExperimentLog(n_trials, n_rows, n_evals, n_eval, rdim, market=market, max_rows=max_episode_rows)
    if trainer_factory is None:
        from .trainer import VecTrainer, schedule_steps

        warmup_steps = schedule_steps(warmup_steps, k_updates, schedule)
        smoothing_window = schedule_steps(smoothing_window, k_updates, schedule)

        def trainer_factory(sd, init_logtemp=0.0):
            return VecTrainer(env, investor, n_lanes, n_gambles, algo=algo, loss=loss, k_updates=k_updates,
                              replay_capacity=(buffer // n_lanes) * n_lanes if multi_steps > 1 else buffer,
                              seed=sd, warmup_steps=warmup_steps, smoothing_window=smoothing_window,
                              precision=precision, device=device, multi_steps=multi_steps,
                              initial_logtemp=init_logtemp, **trainer_kw)
    # a `continue` chain is sequential: rank 0 runs every trial
    owner = [0 if continue_trials else t % world for t in range(n_trials)]
    prev_prefix, prev_logtemp = None, 0.0
    floor = 1e-6 if env == "dice_sh" else 1e-3  # env.reward_range[0] (MIN_REWARD)
    for trial in range(n_trials):
        if owner[trial] != rank:
            continue
        cont = continue_trials and trial > 0 and prev_prefix is not None
        tr = trainer_factory(seed + trial, prev_logtemp if cont else 0.0)
        if cont and os.path.exists(prev_prefix + "_actor.pt"):
            tr.agent.load(prev_prefix)
        prefix = None
        if checkpoint:
            st = logs.save_directory(dict(inputs, trial=trial + 1), results=False)
            prefix = os.path.join(results_root, st[2:] if st.startswith("./") else st)
        ck = _Checkpoint(trail, prefix, floor)
        drain_every = log_every
        if episode_rows:
            cap = episode_cap
            if cap is None:
                drain_every = log_every if log_every <= 64 else 1
                cap = 64 * drain_every
            tr.episode_log(cap)
        pending = []
        prev = np.zeros(3)
        t_row, steps_in_row = time.perf_counter(), 0
        eval_run = 0
        for step in range(1, n_cumsteps + 1):
            tr.step()
            steps_in_row += 1
            log_now = step % log_every == 0 or step == n_cumsteps
            if episode_rows and (log_now or step % drain_every == 0):
                got, dropped = tr.drain_episodes()
                if dropped:
                    raise RuntimeError(f"episode log dropped {dropped} rows at step {step}: episode_cap "
                                       f"{episode_cap} < 64 x steps between drains")
                pending.append(got)
            if log_now:
                now = time.perf_counter()
                stats = tr.last_stats(shadow=True)
                if episode_rows:
                    rows = np.concatenate(pending) if len(pending) > 1 else pending[0]
                    pending = []
                    per_step = (now - t_row) / steps_in_row
                    lg.log_episodes(trial, rows[:, 3] * per_step, rows[:, 2], rows[:, 3], stats, rows[:, 4:])
                    ck.update(tr, rows[:, 2])
                else:
                    n, rs, ls, _ = tr.flush_stats().cpu().numpy()
                    dn, dr, dl = n - prev[0], rs - prev[1], ls - prev[2]
                    prev = np.array([n, rs, ls])
                    lg.log_row(trial, now - t_row, dr / dn if dn else np.nan, dl / dn if dn else np.nan, stats)
                t_row, steps_in_row = now, 0
            if step % eval_freq == 0 and eval_run < n_evals:
                st = tr.last_stats(shadow=True)  # loss[6:8] = agent_shadow_mean(...) first
                t0 = time.perf_counter()
                ev = (tr.evaluate_market(n_eval=n_eval, test_days=test_days) if market
                      else tr.evaluate(n_eval=n_eval, max_steps=max_eval_steps))
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                lg.log_eval(trial, eval_run, ev, time.perf_counter() - t0, st, step)
                eval_run += 1
        prev_logtemp = float(tr.last_stats()[11]) if algo == "SAC" else 0.0
        prev_prefix = prefix if ck.saves else None
        del tr
    if world > 1:
        import torch.distributed as dist

        dev = gather_device or (torch.device("cuda", torch.cuda.current_device())
                                if dist.get_backend() == "nccl" else torch.device("cpu"))
        gather_logs(lg, owner, world, dev)
    stem = logs.save_directory(inputs, results=True)
    path = os.path.join(results_root, stem[2:] if stem.startswith("./") else stem)
    if rank == 0:
        lg.save(path)
    return path, lg
