"""NumPy restatement of the reference environments, vectorised over lanes.

TEST INFRASTRUCTURE (see oracle/__init__.py).  Restates (majidsina/rlmd):
  coin     envs/coin_flip_envs.py:40-93 (consts), :150-216 (A), :290-362 (B), :436-521 (C)
  dice     envs/dice_roll_envs.py:39-96, :153-219, :293-365, :439-524
  gbm      envs/gbm_envs.py:43-90, :147-212, :286-357, :431-515
  dice_sh  envs/dice_roll_sh_envs.py:39-118, :160-235, :290-365, :420-502, :557-645
  market   envs/market_envs.py:38-73, :133-202 (A_D1), :611-682 (A_Dx), B/C variants
  dones    tools/env_resources.py:26-80 (any), :83-137 (all), :140-200 (market)
  slicing  tools/env_resources.py:203-291, scripts/rl_market.py:54-62, :202-214

Arithmetic follows the reference's dtypes under NumPy 2 (NEP 50) for f32
actions, as the agent produces them: wealth and returns are
float64; leverages are float32 for GBM / market (`f32 * Python int`) and
float64 for coin / dice (`f32 * np.float64`); stop-loss, retention and the
safe-haven leverage are float32 (`f32 + Python float`), as are `1e4 * stop_loss`,
`max(., MIN_VALUE)` and, on the first step of an episode (wealth still the
Python float 1e4), the bet size `active`.  Dice_SH_INSURED's leverage is f32
(`f32 * Python-float I_LEV_FACTOR`).  Remaining differences to the reference
are libm ulps and NumPy's float32 pairwise mean in the GBM risk log.
"""
import numpy as np

from . import philox as px

COIN, DICE, GBM, DICE_SH, MARKET = range(5)
ALIAS_FAMILIES = (COIN, DICE, GBM, MARKET)  # reference envs with an in-place self.next_state
INV_A, INV_B, INV_C, INV_INSURED = range(4)

INITIAL_VALUE = 1e4
MIN_VALUE = max(1e-2 * INITIAL_VALUE, 1)
MAX_ABS_ACTION = 0.99
MIN_WEIGHT = 1e-5

FAM = {
    #          MAX_VALUE MIN_REWARD MIN_RETURN        MAX_RETURN LEV_FACTOR
    COIN: (1e18, 1e-3, -0.9, 1e10, 1 / np.abs(0.5)),
    DICE: (1e18, 1e-3, -0.9, 1e10, 1 / np.abs(0.5)),
    GBM: (1e18, 1e-3, np.log(0.1), 1e10, 5),
    DICE_SH: (1e18, 1e-6, -0.99, 1e10, 1 / np.abs(0.5)),
    MARKET: (1e34, 1e-3, -0.9, 1e10, 3),
}
GBM_DRIFT = 0.0540025395205692
GBM_VOL = 0.1897916175617430
GBM_LOG_MEAN = GBM_DRIFT - GBM_VOL**2 / 2
SH_I_LEV = (-1 - 5) / (-0.5 - 5)
SH_UP_R, SH_MID_R, SH_DOWN_R = max(-1, -0.99), max(-1, -0.99), 5

COIN_VALS, COIN_P = np.array([0.5, -0.4]), np.array([0.5, 0.5])
DICE_VALS = np.array([0.5, -0.5, 0.05])
DICE_P = np.array([1 / 6, 1 / 6, 1 - (1 / 6 + 1 / 6)])


F32 = np.float32


def half_shift32(a32):
    """(a + MAX_ABS_ACTION) / 2 in float32, as NumPy 2 evaluates it for f32 a."""
    return (a32 + F32(MAX_ABS_ACTION)) / F32(2)


def choice_index(u, p):
    """NumPy legacy RandomState.choice(a, p): searchsorted(cumsum(p)/sum, u, 'right')."""
    cdf = np.cumsum(p)
    cdf = cdf / cdf[-1]
    return np.searchsorted(cdf, u, side="right")


def dims(family, investor, n, obs_days=1):
    """(state_dim, action_dim, risk_dim, draw_dim) of an env class."""
    if family == DICE_SH:
        a = {INV_INSURED: 1, INV_A: 2, INV_B: 3, INV_C: 4}[investor]
        return 6, a, 7, 1
    extra = {INV_A: 0, INV_B: 1, INV_C: 2}[investor]
    s = 4 + (obs_days * n if family == MARKET else n)
    r = (4 if n == 1 else 4 + n) + extra
    return s, n + extra, r, (0 if family == MARKET else n)


# ---------------------------------------------------------------------------
# market slicing (tools/env_resources.py:203-291)
# ---------------------------------------------------------------------------
def shuffle_rows(length, interval, perms):
    """Row map of shuffle_data: block b of `interval` rows (and the tail block)
    is permuted by perms[b] (the permutation np.random.permutation applied)."""
    out = np.empty(length, dtype=np.int64)
    full = length // interval
    for b in range(full):
        out[b * interval:(b + 1) * interval] = b * interval + np.asarray(perms[b])
    mod = length - full * interval
    if mod:
        out[full * interval:] = full * interval + np.asarray(perms[full])
    return out


def block_perm(seed, lane, episode, blk, bs):
    """Fisher–Yates permutation of one block of bs rows from Philox words."""
    p = list(range(bs))
    words = []
    k = 0
    for i in range(bs - 1, 0, -1):
        if k % 4 == 0:
            v = px.philox(seed, lane, episode, px.TAG_MKT_PERM, blk * 4 + k // 4)
            words = [int(w) for w in v]
        j = (words[k % 4] * (i + 1)) >> 32
        p[i], p[j] = p[j], p[i]
        k += 1
    return p


def observed_rows(t, action_days, obs_days, n):
    """(row, asset) index pairs of observed_market_state(extract, t, ad, d)."""
    if obs_days == 1:
        return np.full(n, t * action_days), np.arange(n)
    f = obs_days * n - 1 - np.arange(obs_days * n)
    return t * action_days + f // n, f % n


class OracleVecEnv:
    """N independent reference envs of one class, stepped in lock-step."""

    def __init__(self, family, investor, n_lanes, n_gambles=1, seed=0, prices=None,
                 obs_days=1, time_length=0, action_days=1, shuffle_days=1, sample_days=0):
        self.f, self.inv, self.N, self.n = family, investor, n_lanes, n_gambles
        self.seed = seed
        self.obs_days, self.time_length = max(obs_days, 1), time_length
        self.action_days, self.shuffle_days = max(action_days, 1), max(shuffle_days, 1)
        self.S, self.A, self.R, self.D = dims(family, investor, n_gambles, self.obs_days)
        self.prices = prices
        if family == MARKET:
            self.ext_len = time_length * self.action_days + 1
            self.start_range = prices.shape[0] - sample_days
        self.wealth = np.full(n_lanes, INITIAL_VALUE)
        self.time = np.ones(n_lanes, dtype=np.int64)
        self.episode = np.full(n_lanes, -1, dtype=np.int64)
        self.start = np.zeros(n_lanes, dtype=np.int64)
        self.rowmap = [None] * n_lanes
        self.step_ctr = 0
        self.reset()

    # -- market helpers -----------------------------------------------------
    def _episode_rows(self, lane):
        ep = int(self.episode[lane])
        L, D = self.ext_len, self.shuffle_days
        full = L // D
        perms = []
        for b in range(full + (1 if L % D else 0)):
            bs = D if b < full else L - full * D
            perms.append(block_perm(self.seed, lane, ep, b, bs) if D > 1 else [0])
        return int(self.start[lane]) + shuffle_rows(L, D, perms)

    def market_obs(self, lane, t):
        rows, assets = observed_rows(t, self.action_days, self.obs_days, self.n)
        return self.prices[self.rowmap[lane][rows], assets]

    # -- reset / step -------------------------------------------------------
    def reset(self, mask=None, start_at=None):
        """start_at (market): given first price row per lane (eval_market's gap
        index, tools/eval_episodes.py:481-492) instead of the Philox draw."""
        mask = np.ones(self.N, bool) if mask is None else np.asarray(mask, bool)
        mv = FAM[self.f][0]
        state = np.zeros((self.N, self.S))
        for lane in np.nonzero(mask)[0]:
            self.wealth[lane] = INITIAL_VALUE
            self.time[lane] = 1
            self.episode[lane] += 1
            st = np.zeros(self.S)
            st[0:4] = [INITIAL_VALUE, 0, 1, 1]
            if self.f == MARKET:
                v = px.philox(self.seed, lane, int(self.episode[lane]), px.TAG_MKT_START, 0)
                self.start[lane] = (int(px.below(v[0], v[1], self.start_range)) if start_at is None
                                    else int(start_at[lane]))
                self.rowmap[lane] = self._episode_rows(lane)
                if self.obs_days > 1:
                    st[4:] = self.market_obs(lane, 0)  # Dx reset: raw prices (market_envs.py:700)
            state[lane] = st / mv
        return state

    def philox_draws(self, step=None):
        step = self.step_ctr if step is None else step
        lanes = np.arange(self.N)
        if self.f == GBM:
            return px.normal_draws(self.seed, lanes, step, px.TAG_ENV_DRAW, self.D)
        return px.uniform_draws(self.seed, lanes, step, px.TAG_ENV_DRAW, self.D)

    def step(self, actions, draws=None):
        """actions [N, A] (f32 from the policy / warm-up sampler, or f64 inside the
        smoothing window, where np.clip with np.float64 bounds promotes them —
        utils.py:345-373); draws [N, D] (None: Philox at the step counter)."""
        arr = np.asarray(actions)
        AT = np.float64 if arr.dtype == np.float64 else np.float32  # dtype the env receives
        a32 = arr.astype(AT).reshape(self.N, self.A)
        a = a32.astype(np.float64)

        def hs(x):  # (a + MAX_ABS_ACTION) / 2 in the action dtype (Python floats weak)
            return (x + AT(MAX_ABS_ACTION)) / AT(2)

        if draws is None and self.f != MARKET:
            draws = self.philox_draws()
        self.step_ctr += 1
        mv, min_reward, min_return, max_return, LF = FAM[self.f]
        f, inv, n = self.f, self.inv, self.n
        w0 = self.wealth.copy()
        t = self.time.copy()
        sl = np.full(self.N, np.nan)
        ret = np.full(self.N, np.nan)
        lev_sh = np.full(self.N, np.nan)

        if f == DICE_SH:
            idx = choice_index(draws[:, 0], DICE_P)
            r = DICE_VALS[idx]
            r_sh32 = np.where(idx == 2, AT(SH_MID_R), np.where(idx == 0, AT(SH_UP_R), AT(SH_DOWN_R)))
            if inv == INV_INSURED:
                lev32 = a32[:, 0] * AT(SH_I_LEV)  # action * Python float
                lev = lev32.astype(np.float64)
                lev_sh32 = AT(1) - lev32
                lev_max = np.abs(lev) == MAX_ABS_ACTION * LF
                lev_min = np.abs(lev32) < AT(MIN_WEIGHT)
            else:
                off = {INV_A: 0, INV_B: 1, INV_C: 2}[inv]
                if inv in (INV_B, INV_C):
                    sl32 = hs(a32[:, 0])
                if inv == INV_C:
                    ret32 = hs(a32[:, 1])
                lev = a[:, off] * LF
                lev_sh32 = hs(a32[:, off + 1]) * AT(1)
                lev_max = np.abs(lev) == MAX_ABS_ACTION * LF
                lev_min = np.abs(lev) < MIN_WEIGHT
            R = lev * r + (lev_sh32 * r_sh32).astype(np.float64)
            lev_sh = lev_sh32.astype(np.float64)
            r_sh = np.where(idx == 2, SH_MID_R, np.where(idx == 0, SH_UP_R, SH_DOWN_R)).astype(np.float64)
            rets = np.stack([r, r_sh], 1)  # the state holds the Python-float r_sh
            lev_mean = lev
        else:
            off = {INV_A: 0, INV_B: 1, INV_C: 2}[inv]
            if inv == INV_B:
                sl32 = np.abs(a32[:, 0]) if f == COIN else hs(a32[:, 0])  # Q1
            elif inv == INV_C:
                sl32 = hs(a32[:, 0])
                ret32 = hs(a32[:, 1])
            if f == COIN:
                rets = COIN_VALS[choice_index(draws, COIN_P)]
            elif f == DICE:
                rets = DICE_VALS[choice_index(draws, DICE_P)]
            elif f == GBM:
                rets = GBM_LOG_MEAN + GBM_VOL * draws
            else:
                rets = np.stack([self.market_obs(l, t[l])[:n] / self.market_obs(l, 0)[:n] - 1
                                 for l in range(self.N)])
            use_all = f in (GBM, MARKET)  # lev_max uses np.all (Q4)
            f32lev = use_all and AT is np.float32  # f32 action * Python int stays f32
            if f32lev:
                lev32 = a32[:, off:off + n] * F32(LF)
                levs = lev32.astype(np.float64)
                lev_max = np.all(np.abs(lev32) == F32(MAX_ABS_ACTION * LF), 1)
                lev_min = np.all(np.abs(lev32) < F32(MIN_WEIGHT), 1)
            else:
                levs = a[:, off:off + n] * LF
                lev_max = (np.all if use_all else np.any)(np.abs(levs) == MAX_ABS_ACTION * LF, 1)
                lev_min = np.all(np.abs(levs) < MIN_WEIGHT, 1)
            R = np.sum(levs * rets, 1)
            # np.mean(lev): float32 pairwise mean for the f32 leverages of GBM / market
            lev_mean = (np.mean(lev32, 1) if f32lev else np.mean(levs, 1)).astype(np.float64)
        if inv in (INV_B, INV_C):
            sl = sl32.astype(np.float64)
        if inv == INV_C:
            ret = ret32.astype(np.float64)

        if f == GBM:
            R = np.maximum(R, min_return)
            g = np.minimum(np.exp(R), 1 + max_return)
        else:
            R = np.clip(R, min_return, max_return)
            g = 1 + R

        if inv in (INV_A, INV_INSURED):
            mw = np.full(self.N, MIN_VALUE)
            W = np.clip(w0 * g, MIN_VALUE, mv)
            done_active = np.zeros(self.N, bool)
        else:
            mw32 = np.maximum(AT(INITIAL_VALUE) * sl32, AT(MIN_VALUE))  # action dtype (Python floats weak)
            mw = mw32.astype(np.float64)
            if inv == INV_C:
                mw = np.where(w0 <= INITIAL_VALUE, mw, INITIAL_VALUE + (w0 - INITIAL_VALUE) * ret)
            # first step of an episode: wealth is the Python float 1e4 -> f32 subtraction
            active32 = np.maximum(AT(INITIAL_VALUE) - mw32, AT(0)).astype(np.float64)
            active = np.where(t == 1, active32, np.maximum(w0 - mw, 0))
            W = np.clip(mw + active * g, mw, mv)
            done_active = active == 0
        growth = W / INITIAL_VALUE
        reward = np.exp(np.log(growth) / t)

        ns = np.empty((self.N, self.S))
        ns[:, 0], ns[:, 1], ns[:, 2], ns[:, 3] = W, R, growth, reward
        if f == MARKET:
            m = self.obs_days * n
            for l in range(self.N):
                ns[l, 4:4 + m] = self.market_obs(l, t[l]) / self.market_obs(l, 0) - 1
        else:
            ns[:, 4:] = rets
        ns /= mv

        done_state = np.any(ns >= 1, 1)
        if f == MARKET:
            tl = self.time_length if self.obs_days == 1 else self.time_length - self.obs_days + 1
            done_time = t == tl
        else:
            done_time = np.zeros(self.N, bool)
        done = (done_time | (W == mw) | (reward < min_reward) | (R == min_return) | lev_max
                | lev_min | done_state | done_active)
        learn_done = done & ~done_state & ~done_time

        risk = np.full((self.N, self.R), np.nan)
        risk[:, 0], risk[:, 1], risk[:, 2] = reward, W, R
        if f == DICE_SH:
            risk[:, 3], risk[:, 4], risk[:, 5], risk[:, 6] = lev_mean, sl, ret, lev_sh
        else:
            risk[:, 3] = lev_mean
            k = 4
            if inv in (INV_B, INV_C):
                risk[:, k] = sl
                k += 1
            if inv == INV_C:
                risk[:, k] = ret
                k += 1
            if n > 1:
                risk[:, k:k + n] = levs
        self.wealth = W
        self.time = t + 1
        self.last_time = t
        return ns, reward, np.stack([done, learn_done], 1), risk

    def stored_state(self, obs, ns):
        """The state the reference's loop stores for the step just taken (obs: the
        pre-step observation, ns: step()'s next state).  Coin / dice / GBM / market
        envs return one self.next_state array that step() mutates in place
        (gbm_envs.py:125, 184-186, 212; market_envs.py:111, 172-174, 202); the loop
        keeps state = next_state and stores state after the next step
        (rl_multiplicative.py:213-245, rl_market.py:240-273; replay.py:164-167
        copies then), so from an episode's second step (t > 1) the stored state
        is the post-step state.  The first step stores reset()'s fresh array.
        Dice_SH returns a new array per step (dice_roll_sh_envs.py:336-339)."""
        if self.f not in ALIAS_FAMILIES:
            return obs
        return np.where((self.last_time > 1)[:, None], ns, obs)
