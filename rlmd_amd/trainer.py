"""Vectorised training loop: N lanes of one env class + one shared learner.

One ``step()`` is one fused vector step of scripts/rl_multiplicative.py:190-227
(and scripts/rl_market.py:217-270) over all lanes, in librlmd_amd.so
(rlmd_train_step): actions (random warm-up draws, or the policy), the
action_window clip, the env step, the replay insert of (s, a, r, s',
learn_done), auto-reset of finished lanes, then K learn() updates.

Semantics decisions versus the reference's single stream: the
warm-up and smoothing counters of this class are vector steps per lane (the
vectorised drivers pass the reference's lengths through schedule_steps, which
converts them to the same number of learner updates); K updates of batch B per
vector step (UTD = K / N per env step, reported with every metric); one agent
shared by all lanes; uniform sampling over all lanes' transitions.
"""
import ctypes

import numpy as np
import torch

from . import _abi
from ._abi import check, ptr, stream_ptr
from .agent import DeviceAgent, ReplayMemory
from .envs import VecEnv

# reference defaults (main.py:144-259, rl_multiplicative.py:108-113)
DEFAULTS = {
    "SAC": dict(h1=256, h2=256, batch=512, topk=256),
    "TD3": dict(h1=400, h2=300, batch=200, topk=100),
}


def schedule_steps(steps, k_updates, schedule="updates"):
    """The reference's warm-up / smoothing lengths (env steps of its single stream,
    where one env step is one learner update: main.py:256-257) as vector steps.

    "updates": the schedule ends after the same number of LEARNER UPDATES as in the
    reference, ceil(steps / K) vector steps at K updates per vector step.  This is
    the default of the vectorised drivers (tools/converge.py, run_experiment):
    counted per lane in vector steps ("vector"), a 1e3-step warm-up at K = 8 is
    8,000 updates on random-action data — measured: TD3 on Dice_SH_InvA then
    saturates both actions at the tanh bounds (lev 1.98, no safe haven, -57 %/step)
    and never recovers, where the reference's 800 warm-up updates leave it at
    +0.4 %/step."""
    if schedule == "vector" or k_updates <= 1:
        return int(steps)
    return -(-int(steps) // int(k_updates))


class VecTrainer:
    def __init__(self, env="gbm", investor="A", n_lanes=65536, n_gambles=1, algo="SAC", loss="MSE",
                 k_updates=1, replay_capacity=1 << 20, seed=0, warmup_steps=1000,
                 smoothing_window=2000, precision="bf16", hidden=None, batch=None, topk=None,
                 prices=None, obs_days=1, time_length=0, shuffle_days=5, sample_days=0,
                 device="cuda:0", init_seed=None, multi_steps=1, dynamics="A", gamma=0.99, s_dist="N",
                 initial_logtemp=0.0, agent_kw=None, slice_groups=0, cu_budget=None, stored_state="reference"):
        """warmup_steps / smoothing_window: vector steps per lane (the ABI's counters;
        schedule_steps converts the reference's lengths).  agent_kw: further
        DeviceAgent settings (update intervals, learning rates, ...).  cu_budget:
        the CUs this trainer's learner may count on (rlmd_agent_set_cu_budget;
        None = the device's).  stored_state: see set_stored_state."""
        self.device = torch.device(device)
        self.env = VecEnv(env, investor, n_lanes, n_gambles, seed=seed, prices=prices, obs_days=obs_days,
                          time_length=time_length, shuffle_days=shuffle_days, sample_days=sample_days,
                          device=device, slice_groups=slice_groups)
        d = DEFAULTS[algo]
        h1, h2 = hidden or (d["h1"], d["h2"])
        self.batch = batch or d["batch"]
        self.topk = topk or d["topk"]
        S, A = self.env.state_dim, self.env.action_dim
        self.agent = DeviceAgent(algo, S, A, h1, h2, self.batch, self.topk, loss=loss, precision=precision,
                                 seed=seed, init_seed=init_seed, policy_dist=s_dist, device=device,
                                 initial_logtemp=initial_logtemp, **(agent_kw or {}))
        if cu_budget is not None:
            check(_abi.lib().rlmd_agent_set_cu_budget(self.agent.h, int(cu_budget)))
        self.replay = ReplayMemory(replay_capacity, S, A, device=device, multi_steps=multi_steps, lanes=n_lanes,
                                   dynamics=dynamics, gamma=gamma)
        self.n_lanes, self.k_updates = n_lanes, k_updates
        self.cfg = _abi.TrainCfg()
        self.cfg.cum_step = 0
        self.cfg.warmup_steps = warmup_steps
        self.cfg.smoothing_window = smoothing_window
        self.cfg.abs_warmup = 0 if self.env.family == _abi.GBM or self.env.family == _abi.MARKET else 1
        self.cfg.k_updates = k_updates
        self.obs = torch.empty(n_lanes, S, dtype=torch.float32, device=self.device)
        self.actions = torch.zeros(n_lanes, A, dtype=torch.float32, device=self.device)
        self.ep_stats = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.stats = torch.full((max(k_updates, 1), 16), float("nan"), dtype=torch.float32, device=self.device)
        check(_abi.lib().rlmd_train_reset(self.env.h, ptr(self.obs), stream_ptr()))
        if stored_state != "reference":
            self.set_stored_state(stored_state)

    @property
    def cum_step(self):
        return self.cfg.cum_step

    def step(self, k_updates=None):
        if k_updates is not None:
            self.cfg.k_updates = k_updates
        self.agent.sync_written()
        check(_abi.lib().rlmd_train_step(self.env.h, self.replay.h, self.agent.h, self.cfg, ptr(self.obs),
                                         ptr(self.actions), ptr(self.ep_stats), ptr(self.stats), stream_ptr()))
        self.cfg.cum_step += 1

    def run(self, n_steps):
        for _ in range(n_steps):
            self.step()

    # per-handle switches (several trainers may share a process, each on its stream)
    def set_fused(self, on):
        """The acting + env fusion of this trainer's env (rlmd_train_set_fused)."""
        check(_abi.lib().rlmd_train_set_fused(self.env.h, 1 if on else 0))

    def last_fused(self):
        return bool(_abi.lib().rlmd_train_last_fused(self.env.h))

    def set_stored_state(self, mode):
        """What replay rows store as `s` (rlmd_train_set_stored_state):
        "reference" (default) = the reference loop's aliased post-step state from
        an episode's second step on (coin / dice / GBM / market; Dice_SH keeps the
        pre-step state), "prestep" = the true pre-step state (a diagnostic)."""
        code = {"reference": 0, "prestep": 1}[mode]
        check(_abi.lib().rlmd_train_set_stored_state(self.env.h, code))

    def stored_state(self):
        return ("reference", "prestep")[_abi.lib().rlmd_train_stored_state(self.env.h)]

    def profile(self, mode):
        """rlmd_profile_enable on this trainer's agent: 0 off, 1 every phase, 2 the
        env kernel's dispatch only, 3 kernel-attached pairs on the env kernel and
        (unfused steps) the acting kernel."""
        check(_abi.lib().rlmd_profile_enable(self.agent.h, int(mode)))

    def profile_stride(self, stride):
        """Time only every stride-th launch of each phase (rlmd_profile_stride)."""
        check(_abi.lib().rlmd_profile_stride(self.agent.h, int(stride)))

    def profile_read(self):
        """(summed ms, launch count) per phase: 0 acting, 1 env kernel, 2 learn."""
        import ctypes as C

        ms, cnt = (C.c_double * 3)(), (C.c_int64 * 3)()
        check(_abi.lib().rlmd_profile_read(self.agent.h, ms, cnt))
        return list(ms), list(cnt)

    def profile_samples(self, phase):
        """The individual timed launches of one phase (ms), rlmd_profile_samples."""
        import ctypes as C

        n = C.c_int64()
        check(_abi.lib().rlmd_profile_samples(self.agent.h, int(phase), None, 0, C.byref(n)))
        buf = (C.c_double * max(n.value, 1))()
        check(_abi.lib().rlmd_profile_samples(self.agent.h, int(phase), buf, n.value, C.byref(n)))
        return list(buf[:n.value])

    def last_stats(self, shadow=False, low_mul=1.0, high_mul=10.0):
        """loss[11] | logtemp | loss_params[4] of the last update (numpy f64).
        shadow: first fill loss[6:8] with the critics' power-law shadow means on
        the device, as the reference's loss[6:8] = agent_shadow_mean(inputs, loss)
        does at every evaluation and episode end (tools/utils.py:441-471;
        shadow_low_mul 1e0 / shadow_high_mul 1e1, main.py:216-217)."""
        k = max(self.cfg.k_updates, 1) - 1
        if shadow:
            row = self.stats[k]
            check(_abi.lib().rlmd_shadow_means(ptr(row), 1, 16, float(low_mul), float(high_mul),
                                               row.data_ptr() + 6 * row.element_size(), 16, stream_ptr()))
        return self.stats[k].double().cpu().numpy()

    def evaluate(self, n_eval=100, max_steps=100, with_stats=True):
        """eval_multiplicative (tools/eval_episodes.py:176-399) on the device: n_eval
        episodes of a separate env (its own seed), each from the reset state with
        the deterministic policy action held constant, the action window applied
        as the reference does at this cum_step; returns the per-episode last
        reward / steps / risk and the 17-entry summary (rlmd_eval_stats)."""
        env = getattr(self, "_eval_env", None)
        if env is None or env.n_lanes != n_eval:
            kw = dict(self.env.make_kw, shuffle_days=3)  # eval shuffles market rows in blocks of 3 (E8)
            env = VecEnv(self.env.family, self.env.investor, n_eval, self.env.n_gambles, seed=self.env.seed + 10007,
                         device=self.device, **kw)
            self._eval_env = env
        obs = env.reset().float()
        actions = self.agent.act(obs, mode=1)
        dev = self.device
        reward = torch.empty(n_eval, dtype=torch.float64, device=dev)
        steps = torch.empty(n_eval, dtype=torch.int32, device=dev)
        risk = torch.empty(n_eval, env.risk_dim, dtype=torch.float64, device=dev)
        stats = torch.empty(17, dtype=torch.float64, device=dev)
        lib = _abi.lib()
        check(lib.rlmd_eval_rollout(env.h, ptr(actions), int(max_steps), int(self.cfg.cum_step),
                                    int(self.cfg.warmup_steps), int(self.cfg.smoothing_window), None, ptr(reward),
                                    ptr(steps), ptr(risk), stream_ptr()))
        if with_stats:  # the NumPy-exact summary (rlmd_eval_stats) covers 1..1024 episodes
            check(lib.rlmd_eval_stats(ptr(reward), ptr(steps), ptr(risk), n_eval, env.risk_dim, env.investor,
                                      ptr(stats), stream_ptr()))
        return {"reward": reward.cpu().numpy(), "steps": steps.cpu().numpy(), "risk": risk.cpu().numpy(),
                "stats": stats.cpu().numpy() if with_stats else None}

    def evaluate_market(self, n_eval=100, test_days=250, gap_days=(5, 20), test_shuffle_days=3, rng=None):
        """eval_market (tools/eval_episodes.py:402-611) for a market trainer: the
        reference evaluates from eval_start_idx = start_idx + step of its one
        training stream (rl_market.py:283-284); here episode i starts from lane
        (i mod N)'s current position plus a gap drawn in [gap_min, gap_max]
        (host draw, as the reference's np.random.randint).  The gap must keep the
        test slice inside the price table (the reference's sample_length
        reserves it: rl_market.py:58-60)."""
        assert self.env.family == _abi.MARKET, "evaluate_market needs a market trainer"
        rng = rng if rng is not None else np.random.default_rng(self.env.seed + self.cfg.cum_step)
        _, t = self.env.lane_state()
        eval_start = (self.env.lane_start() + t - 1)[np.arange(n_eval) % self.n_lanes]
        starts = eval_start + rng.integers(gap_days[0], gap_days[1] + 1, size=n_eval)
        kw = self.env.make_kw
        # one evaluation env per shape, kept across events (its construction —
        # allocations, the price upload, a synchronising reset — was ~1.3 ms of
        # each C4 event); its Philox episode counters advance per event
        key = (n_eval, test_days, test_shuffle_days)
        if getattr(self, "_mkt_eval", (None,))[0] != key:
            tl = test_days + kw["obs_days"] - 1
            ad = kw.get("action_days", 1)
            self._mkt_eval = (key, VecEnv(_abi.MARKET, self.env.investor, n_eval, np.asarray(kw["prices"]).shape[1],
                                          seed=self.env.seed + 20011, prices=kw["prices"], obs_days=kw["obs_days"],
                                          time_length=tl, action_days=ad, shuffle_days=test_shuffle_days,
                                          sample_days=tl * ad + 1, device=self.device))
        return market_evaluate(self.agent, kw["prices"], self.env.investor, kw["obs_days"], test_days, starts,
                               self.cfg.cum_step, self.cfg.warmup_steps, self.cfg.smoothing_window,
                               shuffle_days=test_shuffle_days, device=self.device, env=self._mkt_eval[1])

    def episode_log(self, cap_per_wave=256):
        """Log every finished episode on the device (rlmd_train_episode_log): rows
        [env step, lane, final reward, length, risk...]; 0 disables."""
        check(_abi.lib().rlmd_train_episode_log(self.env.h, int(cap_per_wave)))
        self._ep_cap = int(cap_per_wave)
        self._ep_out = None

    def drain_episodes(self):
        """The episodes logged since the last drain as f64 rows [env step, lane,
        final reward, length, risk...] ordered by (step, lane), and the number of
        rows the per-wave caps dropped."""
        w = 4 + self.env.risk_dim
        cap = ((self.n_lanes + 63) // 64) * self._ep_cap
        if self._ep_out is None:
            self._ep_out = torch.empty(cap, w, dtype=torch.float32, device=self.device)
        import ctypes as C

        n, seen = C.c_int64(), C.c_int64()
        check(_abi.lib().rlmd_train_episode_drain(self.env.h, ptr(self._ep_out), cap, C.byref(n), C.byref(seen),
                                                  stream_ptr()))
        rows = self._ep_out[:n.value].double().cpu().numpy()
        rows = rows[np.lexsort((rows[:, 1], rows[:, 0]))]
        return rows, int(seen.value) - int(n.value)

    def flush_stats(self):
        """Fold the last step's pending episode statistics into ep_stats."""
        check(_abi.lib().rlmd_train_flush_stats(self.env.h, stream_ptr()))
        return self.ep_stats

    def episode_stats(self):
        n, rsum, lsum, _ = self.flush_stats().cpu().numpy()
        return {"episodes": int(n), "mean_final_reward": rsum / max(n, 1), "mean_length": lsum / max(n, 1)}


def market_evaluate(agent, prices, investor, obs_days, test_days, starts, cum_step, warmup_steps,
                    smoothing_window, shuffle_days=3, seed=0, action_days=1, device="cuda:0", env=None, fused=None):
    """eval_market (tools/eval_episodes.py:402-611) on the device, one lane per
    episode: a Market_Inv?_D1/Dx env of time_length test_days + obs_days - 1
    starting at price row starts[i] (gap + eval_start_idx), its extract shuffled
    in blocks of shuffle_days; the deterministic policy acts on every state.
    Returns per-episode last reward / steps / risk, the risk-log rows
    [start, risk...] of eval_risk_log, and the 14 summary statistics of
    :545-585 (rlmd_eval_stats on those rows, NumPy-exact)."""
    dev = torch.device(device)
    starts = np.asarray(starts, dtype=np.int32)
    n = len(starts)
    tl = test_days + obs_days - 1
    if env is None:
        env = VecEnv(_abi.MARKET, investor, n, np.asarray(prices).shape[1], seed=seed, prices=prices,
                     obs_days=obs_days, time_length=tl, action_days=action_days, shuffle_days=shuffle_days,
                     sample_days=tl * action_days + 1, device=dev)
    assert env.n_lanes == n
    assert agent.S == env.state_dim and agent.A == env.action_dim, "agent / env dims differ"
    if fused is not None:  # the env handle's one-launch switch (rlmd_train_set_fused)
        check(_abi.lib().rlmd_train_set_fused(env.h, 1 if fused else 0))
    n_days = np.asarray(prices).shape[0]
    if starts.min() < 0 or starts.max() + tl * action_days + 1 > n_days:
        raise ValueError("an evaluation slice leaves the price table")
    st = torch.from_numpy(starts).to(dev)
    obs = torch.empty(n, env.state_dim, dtype=torch.float32, device=dev)
    act = torch.empty(n, env.action_dim, dtype=torch.float32, device=dev)
    live = torch.empty(n, dtype=torch.uint8, device=dev)
    reward = torch.empty(n, dtype=torch.float64, device=dev)
    steps = torch.empty(n, dtype=torch.int32, device=dev)
    risk = torch.empty(n, env.risk_dim, dtype=torch.float64, device=dev)
    lib = _abi.lib()
    agent.sync_written()
    check(lib.rlmd_eval_market(env.h, agent.h, ptr(st), int(cum_step), int(warmup_steps), int(smoothing_window),
                               ptr(obs), ptr(act), ptr(live), ptr(reward), ptr(steps), ptr(risk), stream_ptr()))
    risk_log = torch.cat([st.double()[:, None], risk], 1).contiguous()
    stats = torch.empty(17, dtype=torch.float64, device=dev)
    check(lib.rlmd_eval_stats(ptr(reward), ptr(steps), ptr(risk_log), n, env.risk_dim + 1, _abi.INV_A, ptr(stats),
                              stream_ptr()))
    return {"reward": reward.cpu().numpy(), "steps": steps.cpu().numpy(), "risk": risk.cpu().numpy(),
            "risk_log": risk_log.cpu().numpy(), "stats": stats[1:15].cpu().numpy()}


_HIP_STREAMS = {}


def _hip_streams(device, n):
    """The first n of this process's group streams on `device`, created on first
    use by the library's HIP runtime and kept for the process (the trainers'
    tensors were allocated on them; torch's caching allocator keys its blocks by
    stream).  HIP places each new stream on one of the process's hardware queues
    as it is created, so every group reuses the same placement: seed i of any
    group runs on the i-th stream created.  Round 5 measured torch pool streams
    taken by consecutive groups at 1.36 - 1.96 x one seed for T = 3 depending on
    which pool slots they got (tools/probe/seeds_queue_probe.py)."""
    lst = _HIP_STREAMS.setdefault(str(device), [])
    with torch.cuda.device(device):
        while len(lst) < n:
            h = ctypes.c_void_p()
            check(_abi.lib().rlmd_stream_create(ctypes.byref(h)))
            lst.append(torch.cuda.ExternalStream(h.value, device=device))
    return lst[:n]


_CU_STREAMS = {}


def _cu_streams(device, n, layout):
    """n CU-masked streams (rlmd_stream_create_cu), kept for the process like
    _hip_streams.  The HIP runtime gives a CU-masked stream a hardware queue of its
    own, so no two seeds share a queue whatever the order of creation.  layout
    "all": every stream may use every CU; "split": stream i gets the CUs c with
    c % n == i (interleaved, so every XCD serves every seed)."""
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    words = (ncu + 31) // 32
    out = []
    with torch.cuda.device(device):
        for i in range(n):
            key = (str(device), layout, n if layout == "split" else 0, i)
            if key not in _CU_STREAMS:
                bits = np.zeros(words * 32, dtype=np.uint8)
                bits[[c for c in range(ncu) if layout == "all" or c % n == i]] = 1
                mask = np.packbits(bits.reshape(words, 32)[:, ::-1], axis=1).view(">u4").astype(np.uint32).ravel()
                h = ctypes.c_void_p()
                check(_abi.lib().rlmd_stream_create_cu(mask.ctypes.data_as(ctypes.c_void_p), words, ctypes.byref(h)))
                _CU_STREAMS[key] = torch.cuda.ExternalStream(h.value, device=device)
            out.append(_CU_STREAMS[key])
    return out


class SeedGroup:
    """Several independent seeds of one workload on one GPU (GPU g runs
    seeds {g, g + G, ...}; the reference's trial loop, rl_multiplicative.py:154-183,
    rl_market.py:167-196, runs them one after another).

    Each seed is a whole VecTrainer — its own lanes, replay ring, learner and
    per-handle switches — launched on its own HIP stream, so the seeds' kernel
    chains run concurrently on the chip (one learner's latency-bound update chain
    leaves most CUs idle).  Nothing is shared between seeds: every seed computes
    exactly what it computes alone with the same CU budget (tests/test_seeds_gpu.py
    checks bit-equality).

    cu_budget ("auto"): each seed's learner counts on 1/T of the device's CUs, so
    the layer-2 column split (twice the workgroups of a row kernel) is not taken
    where T learners' grids would queue for the same CUs (round-5 measurement at
    C2: T = 2 1.60 x one seed with the split, 1.71 x without)."""

    def __init__(self, seeds, device="cuda:0", cu_budget="auto", streams="cu", **kw):
        """streams: "cu" (default) — CU-masked streams over every CU, one hardware
        queue each (round 6, C2: T = 2 / 3 / 4 at 1.64 / 2.04 / 2.17 x one seed,
        against 1.67 / 1.37 / 2.16 x on torch's pool, whose T = 3 placement put two
        seeds on one queue); "pool" — torch's stream pool; a list — the caller's streams, one
        per seed; "hip" — streams created for the
        group by the library's HIP runtime (rlmd_stream_create), wrapped as torch
        external streams: one process-wide list per device, seed i of every group
        on its i-th stream (see _hip_streams); "cu_split" — CU-masked streams
        with a 1/T interleaved share of the CUs per seed (see _cu_streams)."""
        import torch

        self.device = torch.device(device)
        self.seeds = list(seeds)
        if cu_budget == "auto":
            cu_budget = None
            if len(self.seeds) > 1:
                ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
                cu_budget = max(1, ncu // len(self.seeds))
        self.cu_budget = cu_budget
        if streams == "hip":
            self.streams = _hip_streams(self.device, len(self.seeds))
        elif streams in ("cu", "cu_split"):
            self.streams = _cu_streams(self.device, len(self.seeds), "all" if streams == "cu" else "split")
        elif isinstance(streams, (list, tuple)):
            assert len(streams) == len(self.seeds), "one stream per seed"
            self.streams = list(streams)
        else:
            self.streams = [torch.cuda.Stream(device=self.device) for _ in self.seeds]
        self.trainers = []
        for s, st in zip(self.seeds, self.streams):
            with torch.cuda.stream(st):
                kws = dict(kw)
                kws.setdefault("init_seed", s)
                self.trainers.append(VecTrainer(seed=s, device=device, cu_budget=cu_budget, **kws))
        self.synchronize()

    def step(self, k_updates=None):
        """One vector step of every seed, each enqueued on its own stream."""
        import torch

        for tr, st in zip(self.trainers, self.streams):
            with torch.cuda.stream(st):
                tr.step(k_updates)

    def synchronize(self):
        for st in self.streams:
            st.synchronize()

    def __len__(self):
        return len(self.trainers)
