"""Generate golden vectors from the reference (majidsina/rlmd) itself.

Runs ONLY in the build container, where /root/reference exists, via the import
shims of ``_refshim.py``.  The outputs are small ``.npz``
fixtures committed under ``tests/golden/``; the reference never travels.

Every fixture is data: inputs we chose (actions, injected random draws, batch
indices, network initial parameters) and the outputs the REFERENCE computed on
them.  Random draws are injected by replacing the ``np`` / distribution
attributes the reference calls with proxies that hand out our draws through
the same formulae the reference's libraries use (verified against a real
``numpy.random.RandomState`` in ``rng_choice_kat``).

Usage (from anywhere):  python tests/golden/make_golden.py
"""
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refshim  # noqa: E402

_refshim.install()

import torch as T  # noqa: E402

np.set_printoptions(precision=17)


# ----------------------------------------------------------------------------
# draw-injection proxies
# ----------------------------------------------------------------------------
class _InjectedRandom:
    """Stand-in for ``np.random`` inside a reference module.

    ``normal(loc, scale, size)`` returns ``loc + scale * z`` with z injected
    (NumPy's legacy ``normal`` is ``loc + scale * gauss``); ``choice(a, p=p)``
    returns ``a[searchsorted(cumsum(p)/cumsum(p)[-1], u, 'right')]`` with u
    injected (NumPy legacy ``RandomState.choice``; pinned by rng_choice_kat).
    """

    def __init__(self):
        self.queue = []
        self.log = []

    def push(self, vals):
        self.queue.extend(list(np.atleast_1d(vals)))

    def _take(self, size):
        n = 1 if size is None else int(np.prod(size))
        out = np.array(self.queue[:n], dtype=np.float64)
        assert out.size == n, "ran out of injected draws"
        del self.queue[:n]
        self.log.extend(out.tolist())
        return out if size is not None else out[0]

    def normal(self, loc=0.0, scale=1.0, size=None):
        z = self._take(size)
        return loc + scale * z

    def choice(self, a, size=None, replace=True, p=None):
        u = self._take(size)
        p = np.asarray(p, dtype=np.float64)
        cdf = p.cumsum()
        cdf /= cdf[-1]
        idx = cdf.searchsorted(u, side="right")
        return np.asarray(a)[idx]

    def randint(self, low, high=None, size=None):
        v = self._take(size)
        return v.astype(np.int64) if size is not None else int(v)

    def permutation(self, x):
        raise NotImplementedError


class _NpProxy(types.ModuleType):
    """``np`` replacement: numpy everywhere except ``random`` (+ ``array`` fix)."""

    def __init__(self, rnd, flatten_array=False):
        super().__init__("np_proxy")
        self.random = rnd
        self._flatten = flatten_array

    def __getattr__(self, name):
        return getattr(np, name)

    def array(self, obj, *args, **kw):
        # Dice_SH_INSURED builds a risk list holding a size-1 ndarray, which
        # NumPy 2 rejects; flatten size-1 elements as NumPy 1.22 did.
        if self._flatten and isinstance(obj, list):
            obj = [o.reshape(()) if isinstance(o, np.ndarray) and o.size == 1 else o for o in obj]
        return np.array(obj, *args, **kw)


# ----------------------------------------------------------------------------
# F0: RNG known-answer pins for the restatement's draw conventions
# ----------------------------------------------------------------------------
def rng_choice_kat():
    """Pin legacy ``choice(a, p)`` == a[searchsorted(cumsum(p), random_sample(), 'right')]."""
    out = {}
    for name, a, p in (
        ("coin", [0.5, -0.4], [0.5, 0.5]),
        ("dice", [0.5, -0.5, 0.05], [1 / 6, 1 / 6, 1 - 2 / 6]),
    ):
        rs = np.random.RandomState(1234)
        u = rs.random_sample(4096)
        rs = np.random.RandomState(1234)
        ch = np.array([rs.choice(a, p=p) for _ in range(4096)])
        out[name + "_u"] = u
        out[name + "_choice"] = ch
    return out


# ----------------------------------------------------------------------------
# F1: env step traces
# ----------------------------------------------------------------------------
ENV_SPECS = []
for fam, mod in (("coin", "coin_flip_envs"), ("dice", "dice_roll_envs"), ("gbm", "gbm_envs")):
    pref = {"coin": "Coin", "dice": "Dice", "gbm": "GBM"}[fam]
    for inv in ("A", "B", "C"):
        for n in (1, 5):
            ENV_SPECS.append((fam, mod, f"{pref}_Inv{inv}", inv, n))
for inv in ("INSURED", "InvA", "InvB", "InvC"):
    ENV_SPECS.append(("sh", "dice_roll_sh_envs", f"Dice_SH_{inv}", inv, 1))


def _action_schedule(rng, n_steps, a_dim):
    """f32 actions in [-0.99, 0.99] with the edge cases the done logic keys on."""
    acts = rng.uniform(-0.99, 0.99, size=(n_steps, a_dim)).astype(np.float32)
    # sprinkle edges: exact +-0.99 (lev_max), 0 (lev_min), tiny, and long runs of
    # large leverage so wealth walks to its floor / ceiling.
    for t in range(n_steps):
        k = t % 37
        if k == 5:
            acts[t, :] = np.float32(0.99)
        elif k == 11:
            acts[t, :] = np.float32(-0.99)
        elif k == 17:
            acts[t, :] = 0.0
        elif k == 23:
            acts[t, :] = np.float32(1e-6)
        elif 25 <= k <= 33:
            acts[t, :] = np.float32(0.9) * np.sign(acts[t, :] + 1e-3)
    return acts


EDGE_SPECS = [  # all-favourable draws so wealth reaches MAX_VALUE (done_state)
    ("gbm", "gbm_envs", "GBM_InvA", "A", 1),
    ("gbm", "gbm_envs", "GBM_InvC", "C", 2),
    ("coin", "coin_flip_envs", "Coin_InvA", "A", 1),
    ("coin", "coin_flip_envs", "Coin_InvC", "C", 1),
    ("dice", "dice_roll_envs", "Dice_InvB", "B", 1),
    ("sh", "dice_roll_sh_envs", "Dice_SH_InvA", "InvA", 1),
]


def _window_actions(acts, t0=1000, sw=2000):
    """The smoothing-window clip of scripts/rl_multiplicative.py:203-211 applied as
    the reference applies it (tools/utils.py:345-373): np.clip with np.float64
    bounds, so the env receives FLOAT64 actions (NumPy 2 promotion)."""
    import tools.utils as ut

    return np.stack([ut.action_window(acts[t], 0.99, -0.99, t0 + 1 + 7 * t, sw, t0) for t in range(len(acts))])


def env_traces(n_steps=240, seed=7):
    import importlib

    out = {}
    rng = np.random.default_rng(seed)
    rng_w = np.random.default_rng(seed + 1000)
    specs = ([(s, False, False) for s in ENV_SPECS] + [(s, True, False) for s in EDGE_SPECS]
             + [(s, False, True) for s in ENV_SPECS])
    for (fam, modname, cls, inv, n), edge, win in specs:
        r_ = rng_w if win else rng
        mod = importlib.import_module("envs." + modname)
        rnd = _InjectedRandom()
        saved = mod.np
        mod.np = _NpProxy(rnd, flatten_array=True)
        try:
            env = getattr(mod, cls)() if fam == "sh" else getattr(mod, cls)(n)
            a_dim = env.action_space.shape[0]
            s_dim = env.observation_space.shape[0]
            acts = _action_schedule(r_, n_steps, a_dim)
            n_draw = 1 if fam == "sh" else n
            if fam == "gbm":
                draws = r_.standard_normal((n_steps, n_draw))
                # fat left tail occasionally so MIN_RETURN clipping is exercised
                draws[::29] -= 8.0
            else:
                draws = r_.random((n_steps, n_draw))
            if win:
                acts = _window_actions(acts)
                assert acts.dtype == np.float64
            if edge:
                acts = np.full((n_steps, a_dim), np.float32(0.7), dtype=np.float32)
                if fam == "sh":
                    acts[:, 1:] = np.float32(-0.99)  # no safe haven: pure up-moves
                draws = np.full((n_steps, n_draw), 3.0 if fam == "gbm" else 0.01)
            S = np.zeros((n_steps, s_dim))  # state before the step
            S2 = np.zeros((n_steps, s_dim))
            R = np.zeros(n_steps)
            D = np.zeros((n_steps, 2), dtype=np.bool_)
            risk_dim = None
            RISK = []
            state = env.reset().copy()
            for t in range(n_steps):
                S[t] = state
                rnd.push(draws[t])
                s2, rew, done, risk = env.step(acts[t])
                S2[t] = s2
                R[t] = rew
                D[t] = done
                RISK.append(np.array(risk, dtype=np.float64).ravel().copy())
                state = s2.copy()
                if done[0]:
                    state = env.reset().copy()
            risk_dim = RISK[0].size
            key = f"{cls}_n{n}" + ("_edge" if edge else "") + ("_win" if win else "")
            out[key + "/actions"] = acts
            out[key + "/draws"] = draws
            out[key + "/state"] = S
            out[key + "/next_state"] = S2
            out[key + "/reward"] = R
            out[key + "/done"] = D
            out[key + "/risk"] = np.stack(RISK).reshape(n_steps, risk_dim)
        finally:
            mod.np = saved
    return out


# ----------------------------------------------------------------------------
# F2: market slicing / shuffling / observation
# ----------------------------------------------------------------------------
def market_fixtures(seed=11):
    import tools.env_resources as er

    rng = np.random.default_rng(seed)
    prices = np.load("/root/reference/tools/market_data/stooq_usei.npy")[:600]
    out = {"prices": prices}
    # time_slice with injected randint
    rnd = _InjectedRandom()
    saved = er.np
    er.np = _NpProxy(rnd)
    try:
        starts = rng.integers(0, 600 - 130, size=4)
        for i, st in enumerate(starts):
            rnd.push([st])
            ext, s_idx = er.time_slice(prices, 100, 1, 130)
            out[f"slice{i}/start"] = np.int64(s_idx)
            out[f"slice{i}/extract"] = ext
    finally:
        er.np = saved

    # shuffle_data with injected permutations: record the permutation of row
    # indices each block received (the reference permutes row blocks).
    perms = []

    class _PermRandom:
        def permutation(self, x):
            p = rng.permutation(len(x))
            perms.append(p)
            return np.asarray(x)[p]

    er.np = _NpProxy(_PermRandom())
    try:
        for i, (L, d) in enumerate(((101, 5), (103, 5), (250, 3), (251, 3))):
            perms.clear()
            block = prices[17 : 17 + L]
            sh = er.shuffle_data(block, d)
            out[f"shuffle{i}/input"] = block
            out[f"shuffle{i}/interval"] = np.int64(d)
            out[f"shuffle{i}/perms"] = np.concatenate(perms).astype(np.int64)
            out[f"shuffle{i}/output"] = sh
    finally:
        er.np = saved

    # observed_market_state
    ext = prices[40:140]
    for d in (1, 5):
        obs = np.stack([er.observed_market_state(ext, t, 1, d) for t in range(0, 90)])
        out[f"obs_d{d}"] = obs
    out["obs_extract"] = ext
    return out


def market_env_traces(seed=13):
    """One D1 and one Dx episode per investor on stooq_usei (3 assets)."""
    import envs.market_envs as me

    rng = np.random.default_rng(seed)
    prices = np.load("/root/reference/tools/market_data/stooq_usei.npy")
    out = {}
    T_len = 60
    for dname, d in (("D1", 1), ("Dx", 4)):
        for inv in ("A", "B", "C"):
            cls = getattr(me, f"Market_Inv{inv}_{dname}")
            n = prices.shape[1]
            env = cls(n, T_len + d - 1, d)
            a_dim = env.action_space.shape[0]
            st = int(rng.integers(0, prices.shape[0] - 200))
            ext = prices[st : st + T_len + d + 5]
            import tools.env_resources as er

            obs0 = er.observed_market_state(ext, 0, 1, d)
            state = env.reset(obs0).copy()
            acts = rng.uniform(-0.99, 0.99, size=(T_len + 5, a_dim)).astype(np.float32)
            S, S2, R, D, RK = [], [], [], [], []
            t = 0
            done = False
            while not done:
                t += 1
                o = er.observed_market_state(ext, t, 1, d)
                s2, r, dn, risk = env.step(acts[t - 1], o)
                S.append(state)
                S2.append(s2.copy())
                R.append(r)
                D.append(dn)
                RK.append(np.array(risk).copy())
                state = s2.copy()
                done = dn[0]
            key = f"Market_Inv{inv}_{dname}"
            out[key + "/extract"] = ext
            out[key + "/obs_days"] = np.int64(d)
            out[key + "/time_length"] = np.int64(T_len + d - 1)
            out[key + "/actions"] = acts[: len(R)]
            out[key + "/state"] = np.stack(S)
            out[key + "/next_state"] = np.stack(S2)
            out[key + "/reward"] = np.array(R)
            out[key + "/done"] = np.array(D)
            out[key + "/risk"] = np.stack(RK)
    return out


# ----------------------------------------------------------------------------
# F3: critic losses, tail index, side estimators
# ----------------------------------------------------------------------------
LOSSES = ["MSE", "HUB", "MAE", "HSC", "CAU", "TCAU", "CIM", "MSE2", "MSE4", "MSE6"]


def _zipf(k):
    zx = (T.ones((k,)) + k).view(-1)
    for x in range(k):
        zx[x] = zx[x] / (x + 1)
    zx = T.log(zx)
    zx = zx - T.mean(zx)
    return zx, T.sum(zx**2)


def critic_loss_fixtures(seed=3):
    import tools.critic_loss as cl

    g = T.Generator().manual_seed(seed)
    out = {}
    for B, k in ((512, 256), (200, 100)):
        # fat-tailed targets (Student-t nu=2 via normal/sqrt(chi2/2))
        base = T.randn(B, 1, generator=g)
        chi = (T.randn(B, 2, generator=g) ** 2).sum(1, keepdim=True) / 2
        target = (base / T.sqrt(chi + 1e-3)).float()
        q1 = (target + 0.3 * T.randn(B, 1, generator=g)).float()
        q2 = (target + 0.5 * T.randn(B, 1, generator=g)).float()
        zx, zx2 = _zipf(k)
        log_noise = T.tensor(1e-6)
        kern1 = cl.cim_size(q1, target).numpy()
        kern2 = cl.cim_size(q2, target).numpy()
        key0 = f"B{B}"
        out[key0 + "/q1"] = q1.numpy()
        out[key0 + "/q2"] = q2.numpy()
        out[key0 + "/target"] = target.numpy()
        out[key0 + "/k"] = np.int64(k)
        out[key0 + "/cim1"] = kern1
        out[key0 + "/cim2"] = kern2
        for sc in (1.0, 0.37):
            out[key0 + f"/nagy_s{sc}_1"] = cl.nagy_algo(q1, target, sc).numpy()
            out[key0 + f"/nagy_s{sc}_2"] = cl.nagy_algo(q2, target, sc).numpy()
        scale1, scale2 = 0.8, 1.3
        out[key0 + "/scale1"] = np.float64(scale1)
        out[key0 + "/scale2"] = np.float64(scale2)
        for lt in LOSSES:
            a = q1.clone().requires_grad_(True)
            b = q2.clone().requires_grad_(True)
            res = cl.loss_function(a, scale1, float(kern1), b, scale2, float(kern2),
                                   target, B, k, log_noise, zx, zx2, lt)
            m1, mn1, mx1, _, al1, m2, mn2, mx2, _, al2 = res
            (m1 + m2).backward()
            key = f"{key0}/{lt}"
            out[key + "/stats"] = np.array(
                [m1.item(), m2.item(), mn1.item(), mn2.item(), mx1.item(), mx2.item(),
                 al1.item(), al2.item()], dtype=np.float64)
            out[key + "/grad1"] = a.grad.numpy().copy()
            out[key + "/grad2"] = b.grad.numpy().copy()
    return out


def shadow_fixtures():
    import tools.utils as ut

    alphas = np.linspace(0.05, 0.95, 19)
    mins = np.linspace(0.01, 2.0, 19)
    maxs = np.linspace(3.0, 50.0, 19)
    sh = np.array([ut.shadow_means(a, lo, hi, 1.0, 10.0) for a, lo, hi in zip(alphas, mins, maxs)])
    # action window
    acts = np.linspace(-0.99, 0.99, 11)
    steps = np.array([0, 500, 1000, 1001, 1200, 1500, 1999, 2000])
    win = np.stack([ut.action_window(acts.copy(), 0.99, -0.99, s, 2000, 1000) for s in steps])
    # agent_shadow_mean on float32 loss rows, as learn() returns them (0-d float32
    # arrays): tail indices below / above 1, negative, tiny and huge maxima
    rng = np.random.default_rng(17)
    rows = []
    for i in range(64):
        l = np.full(11, np.nan, dtype=np.float32)
        l[0:2] = rng.uniform(0.1, 5.0, 2)
        l[2:4] = rng.uniform(1e-4, 0.1, 2)
        l[4:6] = 10 ** rng.uniform(-3, 3, 2)
        l[8:10] = rng.uniform(-2.0, 1.5, 2)
        rows.append(l)
    rows[0][8:10] = [0.999, 1.0]
    rows[1][4:6] = [1e-5, 1e-7]  # alpha / high large: exp overflows (the reference's inf / nan)
    rows[2][8:10] = [np.nan, 0.5]
    rows = np.stack(rows)
    loss32 = [[np.float32(v) for v in r] for r in rows]
    agent = []
    with np.errstate(all="ignore"):
        for r in loss32:
            sh1, sh2 = ut.agent_shadow_mean({"shadow_low_mul": 1e0, "shadow_high_mul": 1e1}, r)
            agent.append([sh1, sh2])
    agent = np.array(agent)
    assert agent.dtype == np.float32
    # shadow_equiv as tools/aggregate_data.py:441-447 calls it: (mean, tail, cmin,
    # mean, 1) on float64 aggregates; tail indices on both sides of 1
    rng = np.random.default_rng(23)
    eq_mean = 10 ** rng.uniform(-3, 2, 64)
    eq_alpha = rng.uniform(0.05, 1.3, 64)
    eq_min = eq_mean * 10 ** rng.uniform(-4, -0.1, 64)
    with np.errstate(all="ignore"):
        eq = np.array([float(np.atleast_1d(ut.shadow_equiv(m, a, lo, m, 1))[0])
                       for m, a, lo in zip(eq_mean, eq_alpha, eq_min)])
    return {"alpha": alphas, "min": mins, "max": maxs, "shadow": sh,
            "aw_actions": acts, "aw_steps": steps, "aw_out": win,
            "loss_rows": rows, "agent_shadow": agent,
            "eq_mean": eq_mean, "eq_alpha": eq_alpha, "eq_min": eq_min, "eq_out": eq}


# ----------------------------------------------------------------------------
# F4: multi-step replay histories (tools/replay.py:93-332)
# ----------------------------------------------------------------------------
MS_STREAMS = {"a": (30, [4, 9, 13, 22]), "b": (26, [12, 14, 15, 20]), "c": (16, [0, 1, 5, 6, 7])}
MS_CHECKPOINTS = (1, 2, 3, 5, 6, 8, 11, 13, 14, 16, 20, 23, 26, 30)


def multistep_fixtures():
    """Scripted single-stream transitions stored with the reference ReplayBuffer
    (NumPy, the default buffer_gpu=False); after every checkpoint prefix, the
    multi-step (reward, initial state, initial action, eff) of EVERY stored step
    from its own history logic (_episode_rewards_states_actions +
    _multi_step_batch, i.e. sample_exp without the random index draw).
    terminal_memory is zero-filled after construction, as the reference's 1e6-row
    np.empty is in practice (fresh zero pages); the store sequence is learn_done
    as a Python bool, as scripts/rl_multiplicative.py:218-220 passes it."""
    from tools.replay import ReplayBuffer

    S, A = 2, 1
    out = {}
    for name, (L, dones) in MS_STREAMS.items():
        idx = np.arange(L)
        st = np.stack([idx - 1.0, 0.5 - idx], 1)
        s2 = np.stack([idx * 1.0, -0.5 - idx], 1)
        act = (0.05 * idx - 0.5)[:, None].astype(np.float32)
        rew = 1.0 + 0.013 * idx + 0.001 * (idx % 3)
        done = np.isin(idx, dones)
        out.update({f"{name}/state": st, f"{name}/action": act, f"{name}/reward": rew,
                    f"{name}/next_state": s2, f"{name}/done": done})
        for n in (3, 5, 7):
            for dyn in ("A", "M"):
                inputs = {"input_dims": [S], "num_actions": A, "mini_batch_size": 1, "discount": 0.99,
                          "multi_steps": n, "r_abs_zero": None, "dynamics": dyn, "buffer": 4096,
                          "n_cumsteps": 4096}
                rb = ReplayBuffer(inputs)
                rb.terminal_memory[:] = False
                for t in range(L):
                    rb.store_exp(st[t], act[t], rew[t], s2[t], bool(done[t]))
                    T = t + 1
                    if T in MS_CHECKPOINTS:
                        rb.batch_size = T
                        hist = rb._episode_rewards_states_actions(list(range(T)))
                        R, Sx, Ax, eff = rb._multi_step_batch(*hist)
                        key = f"{name}/n{n}{dyn}/T{T}"
                        out[key + "/reward"] = np.asarray(R, dtype=np.float64)
                        out[key + "/state"] = np.asarray(Sx, dtype=np.float64)
                        out[key + "/action"] = np.asarray(Ax, dtype=np.float64)
                        out[key + "/eff"] = np.asarray(eff, dtype=np.int64)
    return out


# ----------------------------------------------------------------------------
# F7: evaluation episodes (tools/eval_episodes.py:176-399)
# ----------------------------------------------------------------------------
EVAL_CASES = [  # (module, class, n_gambles, action, cum_steps, warmup, smoothing)
    ("gbm_envs", "GBM_InvA", 1, [0.35], 5000, 1000, 2000),
    ("gbm_envs", "GBM_InvA", 1, [0.35], 1500, 1000, 2000),  # inside the smoothing window
    ("gbm_envs", "GBM_InvB", 1, [0.2, 0.6], 800, 1000, 2000),  # before warm-up ends: no window
    ("coin_flip_envs", "Coin_InvA", 1, [0.125], 5000, 1000, 2000),
    ("coin_flip_envs", "Coin_InvC", 2, [0.5, 0.3, 0.2, -0.1], 1700, 1000, 2000),
    ("dice_roll_envs", "Dice_InvB", 1, [0.1, 0.19], 5000, 1000, 2000),
    ("dice_roll_sh_envs", "Dice_SH_InvA", 1, [0.9, -0.6], 5000, 1000, 2000),
    ("dice_roll_sh_envs", "Dice_SH_INSURED", 1, [0.83], 1200, 1000, 2000),
    ("gbm_envs", "GBM_InvA", 3, [0.97, -0.95, 0.9], 5000, 1000, 2000),  # high leverage: early dones
    ("coin_flip_envs", "Coin_InvB", 1, [0.4, 0.98], 5000, 1000, 2000),
]


class _FixedAgent:
    """eval_next_action stub: the deterministic policy output (f32, as the
    reference agent's torch->numpy action) for the episode's reset state."""

    def __init__(self, action):
        self.action = np.asarray(action, dtype=np.float32)

    def eval_next_action(self, state):
        return self.action.copy()


def eval_fixtures(seed=21, n_eval=24, max_steps=100):
    import importlib

    import tools.eval_episodes as ev

    out = {}
    rng = np.random.default_rng(seed)
    for ci, (modname, cls, n, action, cum, warm, sw) in enumerate(EVAL_CASES):
        mod = importlib.import_module("envs." + modname)
        rnd = _InjectedRandom()
        saved = mod.np
        mod.np = _NpProxy(rnd, flatten_array=True)
        try:
            sh = modname == "dice_roll_sh_envs"
            D = 1 if sh else n
            if modname == "gbm_envs":
                pool = rng.standard_normal(n_eval * max_steps * D)
            else:
                pool = rng.random(n_eval * max_steps * D)
            rnd.queue, rnd.log = list(pool), []
            inputs = {"ENV_KEY": 0, "algo": "SAC", "s_dist": "N", "loss_fn": "MSE", "n_eval": n_eval,
                      "smoothing_window": sw, "max_action": np.float64(0.99), "min_action": np.float64(-0.99),
                      "random": warm, "max_eval_steps": max_steps,
                      "env_gym": f"{modname}.{cls}()" if sh else f"{modname}.{cls}(n_gambles)", "env_id": cls}
            eval_log = np.zeros((1, 1, n_eval, 20))
            risk_w = 7 if sh else (4 + (1 if cls.endswith("InvB") else 2 if cls.endswith("InvC") else 0)
                                   + (n if n > 1 else 0))
            eval_risk = np.zeros((1, 1, n_eval, risk_w))
            ev.eval_multiplicative(n, _FixedAgent(action), inputs, eval_log, eval_risk, 1, cum, 0, 0,
                                   [0.0] * 11, 0.0, [0.0] * 4)
            steps = eval_log[0, 0, :, 2].astype(np.int64)
            used = np.array(rnd.log)
            assert used.size == steps.sum() * D
            draws = np.zeros((n_eval, max_steps, D))
            pos = 0
            for e in range(n_eval):
                k = steps[e] * D
                draws[e, : steps[e]] = used[pos: pos + k].reshape(steps[e], D)
                pos += k
            key = f"case{ci}"
            out[key + "/spec"] = np.array([modname, cls])
            out[key + "/params"] = np.array([n, cum, warm, sw, n_eval, max_steps], dtype=np.int64)
            out[key + "/action"] = np.asarray(action, np.float32)
            out[key + "/draws"] = draws
            out[key + "/reward"] = eval_log[0, 0, :, 1]
            out[key + "/steps"] = steps
            out[key + "/risk"] = eval_risk[0, 0]
        finally:
            mod.np = saved
    return out


# (algo, investor, obs_days, prices file, cum_steps, warm-up, smoothing window);
# the policy is a real reference agent whose deterministic policy acts on every
# state (eval_next_action).  test_shuffle_days = 1 keeps the extract unshuffled
# (the GPU's in-block shuffle is Philox and is checked against the oracle).
EVAL_MARKET_CASES = [
    ("SAC", "A", 1, "stooq_snp", 5000, 1000, 2000),
    ("TD3", "B", 3, "stooq_usei", 1500, 1000, 2000),
    ("SAC", "C", 1, "stooq_usei", 500, 1000, 2000),
    ("TD3", "A", 4, "stooq_snp", 3000, 1000, 2000),
]


# the production widths (SAC 256/256, TD3 400/300): the shapes the one-launch
# evaluation kernel (env.hip eval_market_loop_kernel) is instantiated for
EVAL_MARKET_FULL_CASES = [
    ("SAC", "A", 1, "stooq_snp", 5000, 1000, 2000, (256, 256)),
    ("TD3", "B", 1, "stooq_snp", 1500, 1000, 2000, (400, 300)),
    ("SAC", "C", 3, "stooq_usei", 3000, 1000, 2000, (256, 256)),
    ("TD3", "A", 5, "stooq_snp", 6000, 1000, 2000, (400, 300)),
]


def eval_market_full_fixtures():
    out = eval_market_fixtures(seed=37, n_eval=32, test_days=60, cases=EVAL_MARKET_FULL_CASES)
    return {k: v for k, v in out.items() if "/init/" not in k or "/init/actor." in k}  # evaluation reads the actor


def eval_market_fixtures(seed=31, n_eval=12, test_days=40, cases=None):
    import algos.algo_sac as asac
    import algos.algo_td3 as atd3
    import envs.market_envs as me
    import tools.eval_episodes as ev

    out = {}
    rng = np.random.default_rng(seed)
    cases = cases or [c + ((32, 24),) for c in EVAL_MARKET_CASES]
    for ci, (algo, inv, d, pfile, cum, warm, sw, hid) in enumerate(cases):
        prices = np.load(f"/root/reference/tools/market_data/{pfile}.npy")
        n = prices.shape[1]
        test_length = test_days + d - 1
        cls = getattr(me, f"Market_Inv{inv}_{'D1' if d == 1 else 'Dx'}")
        probe = cls(n, test_length, d)
        S, A = probe.observation_space.shape[0], probe.action_space.shape[0]
        T.manual_seed(seed + ci)
        agent = (asac.Agent_sac if algo == "SAC" else atd3.Agent_td3)(_inputs(algo, S, A, hid, "MSE", 16, 8))
        init = {}
        for nm in _net_names(algo):
            for pn, p in getattr(agent, nm).named_parameters():
                init[f"{nm}.{pn}"] = p.detach().numpy().copy()
        eval_start = int(rng.integers(0, prices.shape[0] - test_length - 40))
        gaps = rng.integers(5, 21, size=n_eval)
        rnd = _InjectedRandom()
        rnd.push(gaps)
        inputs = {"ENV_KEY": 0, "algo": algo, "s_dist": "N", "loss_fn": "MSE", "n_eval": n_eval,
                  "env_id": f"X_Inv{inv}_D{d}_T1", "action_days": 1, "test_days": test_days,
                  "gap_days_min": 5, "gap_days_max": 20, "test_shuffle_days": 1, "smoothing_window": sw,
                  "max_action": np.float64(0.99), "min_action": np.float64(-0.99), "random": warm}
        R = len(np.atleast_1d(probe.risk)) if hasattr(probe, "risk") else 0
        eval_log = np.zeros((1, 1, n_eval, 20))
        eval_risk = np.zeros((1, 1, n_eval, 1 + R))
        saved = ev.np
        ev.np = _NpProxy(rnd)
        try:
            ev.eval_market(prices, d, eval_start, agent, inputs, eval_log, eval_risk, 1, cum, 0, 0,
                           [0.0] * 11, 0.0, [0.0] * 4)
        finally:
            ev.np = saved
        assert not rnd.queue
        key = f"case{ci}"
        out[key + "/spec"] = np.array([algo, inv, pfile])
        out[key + "/params"] = np.array([d, n, test_days, cum, warm, sw, n_eval, eval_start, hid[0], hid[1]],
                                        dtype=np.int64)
        out[key + "/gaps"] = gaps.astype(np.int64)
        # the rows any episode can touch; episode i starts at row gaps[i] of this slice
        out[key + "/prices"] = prices[eval_start: eval_start + 21 + test_length + 1]
        out[key + "/reward"] = eval_log[0, 0, :, 1]
        out[key + "/steps"] = eval_log[0, 0, :, 2].astype(np.int64)
        out[key + "/risk_log"] = eval_risk[0, 0]  # [gap + eval_start_idx, risk...]
        for kk, v in init.items():
            out[f"{key}/init/{kk}"] = v
    return out


# ----------------------------------------------------------------------------
# §8f-2: experiment file naming and risk-log widths (tools/utils.py:170-307)
# ----------------------------------------------------------------------------
LOG_CASES = [  # (env_id, dynamics, algo, s_dist, loss, buffer, multi_steps, n_cumsteps, n_trials, test, n)
    ("Coin_InvA_n1", "M", "SAC", "N", "MSE", 1e6, 1, 5e4, 10, False, 1),
    ("GBM_InvC_n5", "M", "TD3", "N", "HUB", 1e6, 3, 4e5, 5, True, 5),
    ("Dice_SH_InvB", "M", "SAC", "L", "HSC", 2e5, 5, 1e5, 1, False, 1),
    ("SNP_InvB_D1_T1", "MKT", "TD3", "N", "MAE", 1e6, 1, 3e5, 8, False, 1),
    ("USEI_InvC_D5_T1", "MKT", "SAC", "MVN", "CAU", 1e7, 7, 1e6, 3, True, 3),
]


def log_fixtures():
    import tools.utils as ut

    names, models, dims = [], [], []
    for env_id, dyn, algo, sd, lf, buf, ms, ncs, nt, test, n in LOG_CASES:
        inputs = {"env_id": env_id, "dynamics": dyn, "algo": algo, "s_dist": sd, "loss_fn": lf,
                  "critic_mean_type": "E", "buffer": buf, "multi_steps": ms, "n_cumsteps": ncs, "n_trials": nt,
                  "test_agent": test, "trial": 2}
        names.append(ut.save_directory(inputs, results=True))
        models.append(ut.save_directory(inputs, results=False))
        dims.append(ut.market_log_dim(inputs, n) if dyn == "MKT" else ut.multi_log_dim(inputs, n))
    cases = np.array([[str(x) for x in c] for c in LOG_CASES])
    return {"cases": cases, "results": np.array(names), "models": np.array(models), "risk_dim": np.array(dims)}


# ----------------------------------------------------------------------------
# F5: learn() steps for SAC and TD3
# ----------------------------------------------------------------------------
def _inputs(algo, S, A, hidden, loss_fn="MSE", B=None, k=None, s_dist="N"):
    inputs = {
        "test_agent": True, "ENV_KEY": 14, "env_id": "GOLDEN_n1", "dynamics": "M",
        "input_dims": (S,), "num_actions": A, "max_action": 0.99, "min_action": -0.99,
        "algo": algo, "s_dist": s_dist, "loss_fn": loss_fn, "multi_steps": 1,
        "n_trials": 1, "trial": 1, "n_cumsteps": 5e4, "buffer": 1e6,
        "mini_batch_size": B, "actor_percentile": 50, "critic_percentile": 50,
        "batch_size": {"SAC": k, "TD3": k}, "discount": 0.99, "r_abs_zero": None,
        "cauchy_scale": 1, "critic_mean_type": "E", "log_noise": 1e-6, "gpu": "cpu",
        "buffer_gpu": False, "continue": False,
        "sac_actor_learn_rate": 3e-4, "sac_critic_learn_rate": 3e-4,
        "sac_temp_learn_rate": 3e-4, "sac_layer_1_units": hidden[0],
        "sac_layer_2_units": hidden[1], "sac_actor_step_update": 1,
        "sac_temp_step_update": 1, "sac_target_critic_update": 1,
        "sac_target_update_rate": 5e-3, "initial_logtemp": 0, "reward_scale": 1,
        "log_scale_min": -20, "log_scale_max": 2, "reparam_noise": 1e-6,
        "td3_actor_learn_rate": 1e-3, "td3_critic_learn_rate": 1e-3,
        "td3_layer_1_units": hidden[0], "td3_layer_2_units": hidden[1],
        "td3_actor_step_update": 2, "td3_target_actor_update": 2,
        "td3_target_critic_update": 2, "td3_target_update_rate": 5e-3,
        "policy_noise": 0.1, "target_policy_noise": 0.2, "target_policy_clip": 0.5,
    }
    return inputs


def _net_names(algo):
    return ["actor", "target_actor", "critic_1", "target_critic_1", "critic_2", "target_critic_2"]


def learn_fixtures(seed=5):
    import algos.algo_sac as asac
    import algos.algo_td3 as atd3
    import tools.replay as rp

    out = {}
    # (algo, S, A, hidden, B, k, loss, s_dist): cases 4-6 cover the Laplace and
    # MVN samplers (networks_sac.py:180-258); their noise is injected as the
    # uniform w of Laplace.rsample / the eps of MultivariateNormal.rsample
    cases = [
        ("SAC", 5, 1, (64, 64), 512, 256, "MSE", "N"),
        ("SAC", 6, 2, (64, 48), 512, 256, "HUB", "N"),
        ("TD3", 6, 2, (64, 48), 200, 100, "MSE", "N"),
        ("TD3", 5, 1, (40, 32), 200, 100, "HSC", "N"),
        ("SAC", 5, 1, (64, 64), 512, 256, "MSE", "L"),
        ("SAC", 6, 3, (64, 48), 512, 256, "HUB", "L"),
        ("SAC", 6, 3, (64, 48), 512, 256, "MSE", "MVN"),
    ]
    n_steps = 4
    for ci, (algo, S, A, hid, B, k, lt, sd) in enumerate(cases):
        T.manual_seed(seed + ci)
        rng = np.random.default_rng(seed + ci)
        inputs = _inputs(algo, S, A, hid, lt, B, k, sd)
        agent = asac.Agent_sac(inputs) if algo == "SAC" else atd3.Agent_td3(inputs)
        nets = _net_names(algo)
        init = {}
        for nm in nets:
            for pn, p in getattr(agent, nm).named_parameters():
                init[f"{nm}.{pn}"] = p.detach().numpy().copy()
        # replay contents: small (MAX_VALUE-normalised) states like the envs make
        M = B + 37
        st = (rng.random((M, S)) * 3e-14).astype(np.float64)
        ac = rng.uniform(-0.99, 0.99, (M, A)).astype(np.float32)
        rw = rng.uniform(0.5, 1.5, M)
        st2 = (rng.random((M, S)) * 3e-14).astype(np.float64)
        dn = rng.random(M) < 0.1
        for i in range(M):
            agent.store_transistion(st[i], ac[i], rw[i], st2[i], bool(dn[i]))
        # inject replay indices, and policy noise
        idx_q = []
        rnd = _InjectedRandom()

        class _IdxRandom:
            def choice(self, a, size=None, replace=True, p=None):
                return idx_q.pop(0)

        saved_np = rp.np
        rp.np = _NpProxy(_IdxRandom())
        eps_q = []
        from torch.distributions import Normal

        saved_rs = Normal.rsample

        def _rsample(self, sample_shape=T.Size()):
            e = eps_q.pop(0)
            assert tuple(e.shape) == tuple(self.loc.shape)
            return self.loc + e * self.scale

        Normal.rsample = _rsample
        from torch.distributions import Laplace, MultivariateNormal
        from torch.distributions.multivariate_normal import _batch_mv

        saved_lrs, saved_mrs = Laplace.rsample, MultivariateNormal.rsample

        def _lrsample(self, sample_shape=T.Size()):  # torch's formula with the uniform injected
            w = eps_q.pop(0)
            assert tuple(w.shape) == tuple(self.loc.shape)
            return self.loc - self.scale * w.sign() * T.log1p(-w.abs())

        def _mrsample(self, sample_shape=T.Size()):
            e = eps_q.pop(0)
            assert tuple(e.shape) == tuple(self.loc.shape)
            return self.loc + _batch_mv(self._unbroadcasted_scale_tril, e)

        Laplace.rsample = _lrsample
        MultivariateNormal.rsample = _mrsample
        saved_normal_ = T.Tensor.normal_

        def _normal_(self, mean=0.0, std=1.0, generator=None):
            e = eps_q.pop(0)
            assert tuple(e.shape) == tuple(self.shape)
            with T.no_grad():
                self.copy_(mean + std * e)
            return self

        T.Tensor.normal_ = _normal_
        key = f"case{ci}"
        try:
            for s in range(n_steps):
                idx = rng.choice(M, size=B, replace=False)
                idx_q.append(idx)
                if algo == "SAC" and sd == "L":  # U(eps - 1, 1) as Laplace.rsample draws
                    lo = float(np.finfo(np.float32).eps) - 1.0
                    e1 = T.from_numpy(rng.uniform(lo, 1.0, (B, A)).astype(np.float32))
                    e2 = T.from_numpy(rng.uniform(lo, 1.0, (B, A)).astype(np.float32))
                    eps_q.extend([e1, e2])
                    out[f"{key}/step{s}/eps_next"] = e1.numpy()
                    out[f"{key}/step{s}/eps_cur"] = e2.numpy()
                elif algo == "SAC":
                    e1 = T.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
                    e2 = T.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
                    eps_q.extend([e1, e2])
                    out[f"{key}/step{s}/eps_next"] = e1.numpy()
                    out[f"{key}/step{s}/eps_cur"] = e2.numpy()
                else:
                    e1 = T.from_numpy(rng.standard_normal((B, A)).astype(np.float32))
                    eps_q.append(e1)
                    out[f"{key}/step{s}/eps_target"] = e1.numpy()
                out[f"{key}/step{s}/idx"] = idx.astype(np.int64)
                loss, logtemp, lp = agent.learn()
                out[f"{key}/step{s}/loss"] = np.array([float(x) for x in loss])
                out[f"{key}/step{s}/logtemp"] = np.float64(logtemp)
                out[f"{key}/step{s}/loss_params"] = np.array([float(x) for x in lp])
                assert not eps_q and not idx_q
                for nm in nets:
                    for pn, p in getattr(agent, nm).named_parameters():
                        out[f"{key}/step{s}/{nm}.{pn}"] = p.detach().numpy().copy()
        finally:
            rp.np = saved_np
            Normal.rsample = saved_rs
            Laplace.rsample, MultivariateNormal.rsample = saved_lrs, saved_mrs
            T.Tensor.normal_ = saved_normal_
        out[f"{key}/algo"] = np.array(algo)
        out[f"{key}/loss_fn"] = np.array(lt)
        out[f"{key}/s_dist"] = np.array(sd)
        out[f"{key}/dims"] = np.array([S, A, hid[0], hid[1], B, k], dtype=np.int64)
        out[f"{key}/n_steps"] = np.int64(n_steps)
        for kk, v in init.items():
            out[f"{key}/init/{kk}"] = v
        out[f"{key}/replay/state"] = st
        out[f"{key}/replay/action"] = ac
        out[f"{key}/replay/reward"] = rw
        out[f"{key}/replay/next_state"] = st2
        out[f"{key}/replay/done"] = dn
    return out


def lev_fixtures(seed=41):
    """lev/lev_exp.py:128-237 coin_smart_lev on small Bernoulli outcome matrices
    (torch CPU, float32, as lev/coin_flip.py:160-176 calls it): the per-step
    summary table [n_lev, 13, T-1] and the final values [n_lev, I]."""
    import contextlib
    import io

    from lev import lev_exp

    out = {}
    cases = [("pos", 1500, 40, 15, 100.0, 0.5, -0.4, 0.1, 1.0, 0.1),
             ("neg", 1001, 25, 7, 100.0, 0.3, -0.6, 0.25, 1.0, 0.25),
             ("odd", 777, 33, 1, 50.0, 0.5, -0.5, 0.2, 0.6, 0.2)]
    for name, inv, hor, top, v0, up, dn, lo, hi, inc in cases:
        g = T.Generator().manual_seed(seed)
        outc = T.bernoulli(T.full((inv, hor), 0.5), generator=g)
        with contextlib.redirect_stdout(io.StringIO()):
            data, data_T = lev_exp.coin_smart_lev(T.device("cpu"), outc, inv, hor, top, v0, up, dn, lo, hi, inc)
        out[name + "_outcomes"] = outc.numpy().astype(np.uint8)
        out[name + "_args"] = np.array([inv, hor, top, v0, up, dn, lo, hi, inc], dtype=np.float64)
        out[name + "_levs"] = np.array(lev_exp.param_range(lo, hi, inc), dtype=np.float64)
        out[name + "_data"] = data.numpy()
        out[name + "_data_T"] = data_T.numpy()
    # dice / dice_sh: categorical {0 up, 1 down, 2 mid} outcomes with the envs'
    # probabilities (lev/dice_roll.py, lev/dice_roll_sh.py draw them the same way);
    # gbm: N(mu, sigma) log-returns (lev/gbm.py); torch CPU, float32
    for name, inv, hor, top, v0, rets, lo, hi, inc in (
            ("dice", 1200, 36, 12, 100.0, (0.5, -0.5, 0.05), 0.1, 0.9, 0.2),
            ("diceneg", 900, 30, 5, 100.0, (0.3, -0.6, 0.05), 0.25, 1.0, 0.25),
            ("dicesh", 1100, 32, 9, 100.0, (0.5, -0.5, 0.05, -1.0, 5.0, -1.0), 0.1, 0.9, 0.2),
            ("gbm", 1000, 40, 10, 100.0, None, 0.5, 2.5, 0.5)):
        g = T.Generator().manual_seed(seed + inv)
        if name == "gbm":
            outc = 0.0540025395205692 - 0.1897916175617430 ** 2 / 2 + 0.1897916175617430 * T.randn(
                (inv, hor), generator=g)
        else:
            u = T.rand((inv, hor), generator=g)
            outc = T.where(u < 1 / 6, 0.0, T.where(u < 2 / 6, 1.0, 2.0))
        with contextlib.redirect_stdout(io.StringIO()):
            if name == "gbm":
                data, data_T = lev_exp.gbm_smart_lev(T.device("cpu"), outc, inv, hor, top, v0, lo, hi, inc)
            elif name == "dicesh":
                data, data_T = lev_exp.dice_sh_smart_lev(T.device("cpu"), outc.numpy(), inv, hor, top, v0, *rets, lo,
                                                         hi, inc)
            else:
                data, data_T = lev_exp.dice_smart_lev(T.device("cpu"), outc.numpy(), inv, hor, top, v0, *rets, lo, hi,
                                                      inc)
        out[name + "_outcomes"] = outc.numpy().astype(np.float32)
        out[name + "_args"] = np.array([inv, hor, top, v0, lo, hi, inc], dtype=np.float64)
        out[name + "_rets"] = np.array(rets if rets else [], dtype=np.float64)
        out[name + "_data"] = data.numpy()
        out[name + "_data_T"] = data_T.numpy()
    return out


# ----------------------------------------------------------------------------
# F6: the reference's own C1 loop (scripts/rl_multiplicative.py), recorded
# ----------------------------------------------------------------------------
class _RecordingRandom:
    """``np.random`` of coin_flip_envs that draws from the real, seeded global
    generator and records each coin draw u: legacy ``choice(a, p)`` is
    a[searchsorted(cumsum(p)/cumsum(p)[-1], random_sample(), 'right')]
    (pinned by rng_choice_kat), so the stream is consumed exactly as before."""

    def __init__(self, sink):
        self.sink = sink

    def __getattr__(self, name):
        return getattr(np.random, name)

    def choice(self, a, size=None, replace=True, p=None):
        u = np.random.random_sample(size)
        self.sink(np.atleast_1d(u).astype(np.float64))
        cdf = np.asarray(p, dtype=np.float64).cumsum()
        cdf /= cdf[-1]
        return np.asarray(a)[cdf.searchsorted(u, side="right")]

    def normal(self, loc=0.0, scale=1.0, size=None):
        # legacy normal(loc, scale) = loc + scale * gauss(), gauss being the stream
        # standard_normal draws from: bit-identical (checked over 20,000 draws)
        z = np.random.standard_normal(size)
        self.sink(np.atleast_1d(z).astype(np.float64))
        return loc + scale * z


def c1_trace(n_steps=2500, seed=0, key=8):
    """Config C1 as the reference runs it: main.py's tables (key 8 = Coin_InvA;
    key 14 = GBM_InvA, C2's env), SAC, MSE, one trial of n_steps with eval_freq
    1e3, seeded np.random + torch, through
    scripts/rl_multiplicative.multiplicative_env.  n_steps = 2500 covers the
    warm-up (|sample| except GBM, <= 1e3), the smoothing window (f64 clip,
    <= 2e3) and the policy phase.  Recorded for the TRAINING env instance: every
    step's action as the env received it, the env draw (coin: the choice uniform
    u; GBM: the standard normal z of normal(LOG_MEAN, VOL)), the pre-step state /
    next_state / reward / done / risk; what store_transistion RECEIVED, copied
    at call time (stored_state / stored_next_state: the reference's env mutates
    one self.next_state array and the loop stores state after state =
    next_state, rl_multiplicative.py:213-245, so from an episode's second step
    the stored state is the post-step state); every select_next_action output
    (pre-window) and learn() return; the cum_steps of every save_models(); and
    the saved trial / trial_risk logs."""
    import importlib

    import main as ref_main
    from algos import algo_sac
    from tools import utils

    name = ref_main.gym_envs[str(key)][0]
    cf = importlib.import_module({"Coin": "envs.coin_flip_envs", "GBM_": "envs.gbm_envs"}[name[:4]])
    rec = {k: [] for k in ("action", "draw", "state", "next_state", "reward", "done", "risk", "policy",
                           "learn_loss", "learn_logtemp", "learn_params", "learn_step", "save_step",
                           "stored_state", "stored_next_state")}
    env_ids = []
    ctr = {"steps": 0}
    cur_u = []
    cf_np = _NpProxy(_RecordingRandom(cur_u.append))
    saved_np = cf.np
    cls = getattr(cf, name)
    orig_init, orig_step, orig_reset = cls.__init__, cls.step, cls.reset
    orig_sel, orig_learn, orig_save = algo_sac.Agent_sac.select_next_action, algo_sac.Agent_sac.learn, \
        algo_sac.Agent_sac.save_models
    orig_store = algo_sac.Agent_sac.store_transistion

    def init(self, *a, **kw):
        orig_init(self, *a, **kw)
        env_ids.append(id(self))

    def step(self, action):
        train = id(self) == env_ids[0]
        if train:
            rec["state"].append(self._c1_last.copy())
            rec["action"].append(np.asarray(action).astype(np.float64).copy())
            rec.setdefault("action_dtype", []).append(np.asarray(action).dtype == np.float64)
        cur_u.clear()
        s2, r, d, risk = orig_step(self, action)
        if train:
            rec["draw"].append(np.array(cur_u[0], dtype=np.float64).copy())
            rec["next_state"].append(np.asarray(s2, np.float64).copy())
            rec["reward"].append(float(r))
            rec["done"].append(list(d))
            rec["risk"].append(np.asarray(risk, np.float64).ravel().copy())
            self._c1_last = np.asarray(s2, np.float64).copy()
            ctr["steps"] += 1
        return s2, r, d, risk

    def reset(self):
        s = orig_reset(self)
        self._c1_last = np.asarray(s, np.float64).copy()
        return s

    def sel(self, state):
        a = orig_sel(self, state)
        rec["policy"].append(np.asarray(a).astype(np.float64).copy())
        return a

    def store(self, state, action, reward, next_state, done):
        rec["stored_state"].append(np.asarray(state, np.float64).copy())
        rec["stored_next_state"].append(np.asarray(next_state, np.float64).copy())
        return orig_store(self, state, action, reward, next_state, done)

    def learn(self):
        loss, logtemp, params = orig_learn(self)
        rec["learn_loss"].append(np.asarray([float(x) for x in loss], np.float64))
        rec["learn_logtemp"].append(float(logtemp))
        rec["learn_params"].append(np.asarray([float(x) for x in params], np.float64))
        rec["learn_step"].append(ctr["steps"] - 1)
        return loss, logtemp, params

    def save(self):
        rec["save_step"].append(ctr["steps"])
        orig_save(self)

    cf.np = cf_np
    cls.__init__, cls.step, cls.reset = init, step, reset
    algo_sac.Agent_sac.select_next_action, algo_sac.Agent_sac.learn = sel, learn
    algo_sac.Agent_sac.save_models, algo_sac.Agent_sac.store_transistion = save, store
    rl = importlib.import_module("scripts.rl_multiplicative")
    rl.Agent_sac = algo_sac.Agent_sac
    import contextlib
    import glob
    import io

    try:
        for f in glob.glob("results/test_multiplicative/**/*.npy", recursive=True):
            os.remove(f)
        inputs = dict(ref_main.inputs)
        inputs.update({"n_trials_mul": 1, "n_cumsteps_mul": float(n_steps), "gpu": "cpu", "buffer_gpu": False})
        inputs = utils.input_initialisation(inputs, [key], ["SAC"], ["MSE"], [1])
        inputs["test_agent"] = True
        inputs["ENV_KEY"] = key
        np.random.seed(seed)
        T.manual_seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            rl.multiplicative_env(ref_main.gym_envs, inputs, n_gambles=1)
        trial = np.load(glob.glob("results/test_multiplicative/**/*_trial.npy", recursive=True)[0])
        trial_risk = np.load(glob.glob("results/test_multiplicative/**/*_trial_risk.npy", recursive=True)[0])
    finally:
        cf.np = saved_np
        cls.__init__, cls.step, cls.reset = orig_init, orig_step, orig_reset
        algo_sac.Agent_sac.select_next_action, algo_sac.Agent_sac.learn = orig_sel, orig_learn
        algo_sac.Agent_sac.save_models, algo_sac.Agent_sac.store_transistion = orig_save, orig_store
    out = {k: np.asarray(v) for k, v in rec.items()}
    out["trial"] = trial
    out["trial_risk"] = trial_risk
    out["n_steps"] = np.array(n_steps)
    out["seed"] = np.array(seed)
    out["key"] = np.array(key)
    return out


def c1_gbm_trace():
    """F6-GBM: c1_trace on GBM_InvA (key 14, C2's env): the family whose state
    (wealth / 1e18) is not negligible, so the stored-state aliasing changes the
    critic's input."""
    return c1_trace(key=14)


# ----------------------------------------------------------------------------
# F6-market: the reference's own market loop (scripts/rl_market.py), recorded
# ----------------------------------------------------------------------------
def market_trace(obs_days, n_steps=2500, seed=0, key=22, algo="TD3", loss_fn="HUB", train_days=200):
    """scripts/rl_market.market_env as the reference runs it: main.py's tables
    (key 22 = SNP_InvB on tools/market_data/stooq_snp.npy), TD3, HUB, one trial
    of n_steps with eval every 1e3 steps (4 episodes), train_days 200 (so a
    dozen episodes end inside the run), seeded np.random + torch.  n_steps =
    2500 covers the warm-up (raw samples, < 1e3), the smoothing window (f64
    clip, <= 2e3) and the policy phase.  Recorded for the TRAINING env
    instance: each episode's start row and shuffled extract (time_slice /
    shuffle_data outside eval_market), every step's action as the env received
    it, the observation handed to step(), state / next_state / reward / done /
    risk; every select_next_action output and learn() return; every
    eval_market call's arguments; the steps of every save_models(); and the
    saved trial / trial_risk logs."""
    import importlib

    import main as ref_main
    import envs.market_envs as me
    from algos import algo_sac, algo_td3
    from tools import env_resources as er
    from tools import eval_episodes as ev
    from tools import utils

    agent_cls = algo_td3.Agent_td3 if algo == "TD3" else algo_sac.Agent_sac
    rec = {k: [] for k in ("action", "action_dtype", "obs", "state", "next_state", "reward", "done", "risk",
                           "policy", "learn_loss", "learn_logtemp", "learn_params", "save_step", "start_idx",
                           "extract", "reset_obs", "eval_start_idx", "eval_cum_steps", "eval_loss",
                           "eval_logtemp", "eval_params", "stored_state", "stored_next_state")}
    env_ids, ctx = [], {"eval": False, "steps": 0}
    cls = getattr(me, "Market_" + ref_main.gym_envs[str(key)][0][-4:] + ("_D1" if obs_days == 1 else "_Dx"))
    orig = dict(init=cls.__init__, step=cls.step, reset=cls.reset, ts=er.time_slice, sd=er.shuffle_data,
                ev=ev.eval_market, sel=agent_cls.select_next_action, learn=agent_cls.learn, save=agent_cls.save_models,
                store=agent_cls.store_transistion)

    def init(self, *a, **kw):
        env_ids.append(id(self))  # before the constructor's own reset(assets=None)
        orig["init"](self, *a, **kw)

    def train(self):
        return id(self) == env_ids[0] and not ctx["eval"]

    def step(self, action, next_assets):
        if train(self):
            rec["state"].append(self._mt_last.copy())
            rec["action"].append(np.asarray(action).astype(np.float64).copy())
            rec["action_dtype"].append(np.asarray(action).dtype == np.float64)
            rec["obs"].append(np.asarray(next_assets, np.float64).copy())
        s2, r, d, risk = orig["step"](self, action, next_assets)
        if train(self):
            rec["next_state"].append(np.asarray(s2, np.float64).copy())
            rec["reward"].append(float(r))
            rec["done"].append(list(d))
            rec["risk"].append(np.asarray(risk, np.float64).ravel().copy())
            self._mt_last = np.asarray(s2, np.float64).copy()
            ctx["steps"] += 1
        return s2, r, d, risk

    def reset(self, assets):
        s = orig["reset"](self, assets)
        if assets is not None and train(self):
            rec["reset_obs"].append(np.asarray(assets, np.float64).copy())
            self._mt_last = np.asarray(s, np.float64).copy()
        return s

    def time_slice(*a, **kw):
        out, start = orig["ts"](*a, **kw)
        if not ctx["eval"]:
            rec["start_idx"].append(int(start))
        return out, start

    def shuffle_data(*a, **kw):
        out = orig["sd"](*a, **kw)
        if not ctx["eval"]:
            rec["extract"].append(np.asarray(out, np.float64).copy())
        return out

    def eval_market(market_data, od, eval_start_idx, agent, inputs, eval_log, eval_risk_log, mstep, cum_steps, rnd,
                    eval_run, loss, logtemp, loss_params):
        rec["eval_start_idx"].append(int(eval_start_idx))
        rec["eval_cum_steps"].append(int(cum_steps))
        rec["eval_loss"].append(np.asarray([float(x) for x in loss], np.float64))
        rec["eval_logtemp"].append(float(logtemp))
        rec["eval_params"].append(np.asarray([float(x) for x in loss_params], np.float64))
        ctx["eval"] = True
        try:
            return orig["ev"](market_data, od, eval_start_idx, agent, inputs, eval_log, eval_risk_log, mstep,
                              cum_steps, rnd, eval_run, loss, logtemp, loss_params)
        finally:
            ctx["eval"] = False

    def sel(self, state):
        a = orig["sel"](self, state)
        rec["policy"].append(np.asarray(a).astype(np.float64).copy())
        return a

    def store(self, state, action, reward, next_state, done):
        rec["stored_state"].append(np.asarray(state, np.float64).copy())
        rec["stored_next_state"].append(np.asarray(next_state, np.float64).copy())
        return orig["store"](self, state, action, reward, next_state, done)

    def learn(self):
        loss, logtemp, params = orig["learn"](self)
        rec["learn_loss"].append(np.asarray([float(x) for x in loss], np.float64))
        rec["learn_logtemp"].append(float(logtemp))
        rec["learn_params"].append(np.asarray([float(x) for x in params], np.float64))
        return loss, logtemp, params

    def save(self):
        rec["save_step"].append(ctx["steps"])
        orig["save"](self)

    cls.__init__, cls.step, cls.reset = init, step, reset
    er.time_slice, er.shuffle_data, ev.eval_market = time_slice, shuffle_data, eval_market
    agent_cls.select_next_action, agent_cls.learn, agent_cls.save_models = sel, learn, save
    agent_cls.store_transistion = store
    rl = importlib.import_module("scripts.rl_market")
    import contextlib
    import glob
    import io

    try:
        data = np.load("/root/reference/tools/market_data/stooq_snp.npy", allow_pickle=False)
        inputs = dict(ref_main.inputs)
        inputs.update({"n_trials_mkt": 1, "n_cumsteps_mkt": float(n_steps), "eval_freq_mkt": 1e3, "n_eval_mkt": 4,
                       "train_days": float(train_days), "gpu": "cpu", "buffer_gpu": False})
        inputs = utils.input_initialisation(inputs, [key], [algo], [loss_fn], [1])
        inputs["test_agent"] = True
        inputs["ENV_KEY"] = key
        np.random.seed(seed)
        T.manual_seed(seed)
        for f in glob.glob("results/test_market/**/*.npy", recursive=True):
            os.remove(f)
        with contextlib.redirect_stdout(io.StringIO()):
            rl.market_env(ref_main.gym_envs, inputs, market_data=data, obs_days=obs_days)
        stem = glob.glob(f"results/test_market/**/*_D{obs_days}_T1*_trial.npy", recursive=True)[0][:-len("_trial.npy")]
        logs_out = {nm: np.load(stem + f"_{nm}.npy") for nm in ("trial", "eval", "trial_risk", "eval_risk")}
    finally:
        cls.__init__, cls.step, cls.reset = orig["init"], orig["step"], orig["reset"]
        er.time_slice, er.shuffle_data, ev.eval_market = orig["ts"], orig["sd"], orig["ev"]
        agent_cls.select_next_action, agent_cls.learn, agent_cls.save_models = orig["sel"], orig["learn"], orig["save"]
        agent_cls.store_transistion = orig["store"]
    out = {k: np.asarray(v) for k, v in rec.items() if k != "extract"}
    out["extract"] = np.stack(rec["extract"])  # every slice has train_length + 1 rows
    for nm, v in logs_out.items():
        out[nm] = v
    out["params"] = np.array([n_steps, seed, key, obs_days, train_days], dtype=np.int64)
    out["spec"] = np.array([algo, loss_fn])
    return out


def env_resources_kat(seed=123):
    """tools/env_resources.py's time_slice / shuffle_data / observed_market_state
    on stooq_usei rows with np.random seeded: the outputs and the generator
    state after each call (pins the draw order of the host restatement,
    rlmd_amd/env_resources.py)."""
    from tools import env_resources as er

    prices = np.load("/root/reference/tools/market_data/stooq_usei.npy")[:400]
    out = {"prices": prices}
    np.random.seed(seed)
    for i, (ext_days, sample_days, interval) in enumerate([(20, 60, 5), (33, 40, 3), (7, 390, 1), (12, 100, 4)]):
        sl, st = er.time_slice(prices, ext_days, 1, sample_days)
        sh = er.shuffle_data(sl, interval)
        out[f"case{i}/params"] = np.array([ext_days, sample_days, interval])
        out[f"case{i}/start"] = np.int64(st)
        out[f"case{i}/shuffled"] = sh
        out[f"case{i}/next_u"] = np.float64(np.random.random_sample())
        for d in (1, 3):
            for t in (0, 2):
                out[f"case{i}/obs_d{d}_t{t}"] = np.asarray(er.observed_market_state(sh, t, 1, d))
    return out


def market_traces():
    T.set_num_threads(2)  # the reference's small-batch learn() is slower on more threads beside other jobs
    out = {}
    for d in (1, 5):
        for k, v in market_trace(d).items():
            out[f"d{d}/{k}"] = v
    return out


# ----------------------------------------------------------------------------
# F10: *_fixed_final_lev (statistics captured at the reference's torch calls)
#      and coin_galaxy_brain_lev
# ----------------------------------------------------------------------------
class _StatRecorder(types.ModuleType):
    """``T`` of lev_exp recording what its fixed-final statistics return:
    std_mean (std, mean), median and mean, in call order."""

    def __init__(self):
        super().__init__("torch_proxy")
        self.calls = []

    def __getattr__(self, name):
        return getattr(T, name)

    def std_mean(self, x, *a, **kw):
        r = T.std_mean(x, *a, **kw)
        self.calls.append(("std_mean", float(r[0]), float(r[1]), x.detach().clone()))
        return r

    def median(self, x, *a, **kw):
        r = T.median(x, *a, **kw)
        self.calls.append(("median", float(r)))
        return r

    def mean(self, x, *a, **kw):
        r = T.mean(x, *a, **kw)
        self.calls.append(("mean", float(r)))
        return r


def _final_stats(calls, n_lev):
    """[n_lev, 12] in STAT_NAMES order from the recorded calls (per leverage: the
    all / top / adjusted groups' std_mean, median, mean(|.|) in that order) and
    the recorded final values [n_lev, investors]."""
    per = len(calls) // n_lev
    out, vals = np.zeros((n_lev, 12)), []
    for i in range(n_lev):
        c = calls[i * per:(i + 1) * per]
        sm = [x for x in c if x[0] == "std_mean"]
        md = [x[1] for x in c if x[0] == "median"]
        mn = [x[1] for x in c if x[0] == "mean"]
        out[i] = [sm[0][2], sm[1][2], sm[2][2], mn[0], mn[1], mn[2], sm[0][1], sm[1][1], sm[2][1], md[0], md[1], md[2]]
        vals.append(sm[0][3].numpy())
    return out, np.stack(vals)


def lev_final_fixtures(seed=43):
    import contextlib
    import io

    from lev import lev_exp

    out = {}
    cases = [("coin", 900, 30, 11, 100.0, (0.5, -0.4), 0.1, 1.0, 0.3),
             ("dice", 800, 25, 7, 100.0, (0.5, -0.5, 0.05), 0.2, 0.8, 0.3),
             ("dicesh", 700, 20, 5, 100.0, (0.5, -0.5, 0.05, -1.0, 5.0, -1.0), 0.1, 0.9, 0.4),
             ("gbm", 600, 35, 6, 100.0, (), 0.5, 2.0, 0.5)]
    saved = lev_exp.T
    try:
        for name, inv, hor, top, v0, rets, lo, hi, inc in cases:
            g = T.Generator().manual_seed(seed + inv)
            if name == "coin":
                outc = T.bernoulli(T.full((inv, hor), 0.5), generator=g)
            elif name == "gbm":
                outc = 0.0540025395205692 - 0.1897916175617430 ** 2 / 2 + 0.1897916175617430 * T.randn(
                    (inv, hor), generator=g)
            else:
                u = T.rand((inv, hor), generator=g)
                outc = T.where(u < 1 / 6, 0.0, T.where(u < 2 / 6, 1.0, 2.0))
            rec = _StatRecorder()
            lev_exp.T = rec
            with contextlib.redirect_stdout(io.StringIO()):
                fn = {"coin": lev_exp.coin_fixed_final_lev, "dice": lev_exp.dice_fixed_final_lev,
                      "dicesh": lev_exp.dice_sh_fixed_final_lev, "gbm": lev_exp.gbm_fixed_final_lev}[name]
                o_arg = outc.numpy() if name == "dicesh" else outc
                fn(T.device("cpu"), o_arg, top, v0, *rets, lo, hi, inc)
            lev_exp.T = saved
            n_lev = len(lev_exp.param_range(lo, hi, inc))
            st, vals = _final_stats(rec.calls, n_lev)
            out[name + "_outcomes"] = outc.numpy().astype(np.float32)
            out[name + "_args"] = np.array([inv, hor, top, v0, lo, hi, inc], dtype=np.float64)
            out[name + "_rets"] = np.array(rets, dtype=np.float64)
            out[name + "_stats"] = st
            out[name + "_values"] = vals
        # big-brain investors: coin with retention 0 only (a ratio > 0 raises a
        # TypeError in the reference's coin_optimal_lev), dice with 0 and > 0
        for name, inv, hor, top, v0, rets, lf, stop, roll in (
                ("coinbrain", 600, 24, 9, 100.0, (0.5, -0.4), 1.8, (0.1, 0.5, 0.2), (0.0, 0.0, 0.1)),
                ("dicebrain", 500, 20, 7, 100.0, (0.5, -0.5, 0.05), 1.6, (0.2, 0.6, 0.2), (0.5, 0.9, 0.2)),
                ("dicebrain0", 400, 18, 3, 100.0, (0.5, -0.5, 0.05), 1.6, (0.3, 0.3, 0.1), (0.0, 0.0, 0.1))):
            g = T.Generator().manual_seed(seed + inv + hor)
            if name == "coinbrain":
                outc = T.bernoulli(T.full((inv, hor), 0.5), generator=g)
                fn = lev_exp.coin_big_brain_lev
            else:
                u = T.rand((inv, hor), generator=g)
                outc = T.where(u < 1 / 6, 0.0, T.where(u < 2 / 6, 1.0, 2.0))
                fn = lev_exp.dice_big_brain_lev
            with contextlib.redirect_stdout(io.StringIO()):
                data = fn(T.device("cpu"), outc, inv, hor, top, v0, *rets, T.tensor(lf), *stop, *roll)
            out[name + "_outcomes"] = outc.numpy().astype(np.float32)
            out[name + "_args"] = np.array([inv, hor, top, v0, lf, *stop, *roll], dtype=np.float64)
            out[name + "_rets"] = np.array(rets, dtype=np.float64)
            out[name + "_data"] = data.numpy()
        grid = (0.1, 0.5, 0.1, 0.1, 0.4, 0.1, 0.4, 0.6, 0.1)  # len(rd) <= len(ru): the reference indexes rd by ru's size
        out["galaxy_args"] = np.array(grid, dtype=np.float64)
        out["galaxy"] = lev_exp.coin_galaxy_brain_lev(T.device("cpu"), *grid).numpy()
    finally:
        lev_exp.T = saved
    return out


# ----------------------------------------------------------------------------
# F9: the reference's readers (tools/aggregate_data.py) on the build's log files
# ----------------------------------------------------------------------------
def _logs_mod():
    import importlib.util

    spec = importlib.util.spec_from_file_location("make_golden_logs", os.path.join(HERE, "make_golden_logs.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def aggregate_fixtures():
    """mul_inv_aggregate (aggregate_data.py:289-353) and mul_inv_n_summary
    (:356-447) of the reference, run on log files the build wrote: the arrays the
    reference's figure scripts (scripts/gen_figures.py:344-359) would plot."""
    import main as ref_main
    from tools import aggregate_data as ag

    ml = _logs_mod()
    ml.write_build_logs(".")
    agg = ag.mul_inv_aggregate([8, 9, 10], 1, ref_main.gym_envs, dict(ml.AGG_INPUTS))
    summ = ag.mul_inv_n_summary(dict(ml.AGG_INPUTS), agg)
    names = ["reward", "lev", "stop", "reten", "loss", "tail", "shadow", "cmax", "keqv", "lev_sh"]
    out = {"aggregate": agg}
    for n, v in zip(names, summ):
        out["summary_" + n] = np.asarray(v, dtype=np.float64)
    return out


def main():
    work = tempfile.mkdtemp(prefix="rlmd_golden_")
    os.chdir(work)  # the reference creates ./results/... relative to cwd
    jobs = {
        "rng_kat.npz": rng_choice_kat,
        "env_traces.npz": env_traces,
        "market.npz": market_fixtures,
        "market_env.npz": market_env_traces,
        "critic_loss.npz": critic_loss_fixtures,
        "shadow.npz": shadow_fixtures,
        "multistep.npz": multistep_fixtures,
        "eval.npz": eval_fixtures,
        "eval_market.npz": eval_market_fixtures,
        "eval_market_full.npz": eval_market_full_fixtures,
        "logs.npz": log_fixtures,
        "learn.npz": learn_fixtures,
        "lev.npz": lev_fixtures,
        "c1_trace.npz": c1_trace,
        "c1_gbm_trace.npz": c1_gbm_trace,
        "market_trace.npz": market_traces,
        "env_resources_kat.npz": env_resources_kat,
        "aggregate.npz": aggregate_fixtures,
        "lev_final.npz": lev_final_fixtures,
    }
    only = sys.argv[1:]
    for fn, job in jobs.items():
        if only and fn not in only:
            continue
        data = job()
        np.savez_compressed(os.path.join(HERE, fn), **data)
        print("wrote", fn, len(data), "arrays,", os.path.getsize(os.path.join(HERE, fn)), "bytes")


if __name__ == "__main__":
    main()
