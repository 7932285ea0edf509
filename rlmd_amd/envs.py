"""Batched MI355X environments behind the reference's env interface.

``VecEnv`` steps N independent lanes of one reference env class per launch
(rlmd_env_step / rlmd_env_reset of librlmd_amd.so).  The reference-named
classes (``Coin_InvA`` ... ``Dice_SH_InvC``, ``Market_InvA_D1`` ...) keep the
Gym-style single-env API of envs/*_envs.py — ``reset()``, ``step(action)``
returning ``(next_state, reward, [done, learn_done], risk)``, plus
``observation_space`` / ``action_space`` / ``reward_range`` — on one lane of
the same kernels, so reference drivers can swap them in.
"""
import ctypes as C

import numpy as np
import torch

from . import _abi
from ._abi import check, ptr, stream_ptr

FAMILY = {"coin": _abi.COIN, "dice": _abi.DICE, "gbm": _abi.GBM, "dice_sh": _abi.DICE_SH,
          "market": _abi.MARKET}
INVESTOR = {"A": _abi.INV_A, "B": _abi.INV_B, "C": _abi.INV_C, "INSURED": _abi.INV_INSURED}
MAX_VALUE = {_abi.COIN: 1e18, _abi.DICE: 1e18, _abi.GBM: 1e18, _abi.DICE_SH: 1e18, _abi.MARKET: 1e34}
MIN_REWARD = {_abi.COIN: 1e-3, _abi.DICE: 1e-3, _abi.GBM: 1e-3, _abi.DICE_SH: 1e-6, _abi.MARKET: 1e-3}
MAX_ABS_ACTION = 0.99
# families whose reference env returns one self.next_state array mutated in place by
# every step (Dice_SH builds a new one per step); the vectorised trainer's replay
# rows follow the same rule (rlmd_train_set_stored_state)
ALIAS_FAMILIES = frozenset({_abi.COIN, _abi.DICE, _abi.GBM, _abi.MARKET})

def generator_state_key():
    """A hash of the driver-visible random state: NumPy's global MT19937 state and
    torch's CPU generator state, both read without advancing them."""
    import hashlib

    _, keys, pos, _, _ = np.random.get_state()
    h = hashlib.blake2b(np.ascontiguousarray(keys, dtype=np.uint32).tobytes(), digest_size=8)
    h.update(np.array([pos], dtype=np.int64).tobytes())
    h.update(torch.get_rng_state().numpy().tobytes())
    return h.digest()


class _StateKeyed:
    """Philox keys from the generator state.  Two objects created while the state
    has not moved (no draw in between) are kept apart by their position in that
    run of creations; the position restarts whenever the state moves, so a seed's
    keys do not depend on what the process created before it was seeded."""

    def __init__(self, tag):
        self.tag, self.last, self.n = tag, None, 0

    def __call__(self):
        import hashlib

        st = generator_state_key()
        if st == self.last:
            self.n += 1
        else:
            self.last, self.n = st, 0
        h = hashlib.blake2b(st + self.tag + self.n.to_bytes(4, "little"), digest_size=8)
        return int.from_bytes(h.digest(), "little") & 0x7FFFFFFF


_ENV_SEEDS = _StateKeyed(b"env")


def private_seed():
    """A Philox seed for a device env created without one.  Reading the generator
    states does not advance them: the reference's env constructors consume no
    draws, so drawing one here would shift the global stream the drivers consume
    in the reference's order (time_slice, shuffle_data, eval gaps).  Hashing the
    state makes the device env's noise follow the driver's np.random.seed(s) /
    torch.manual_seed(s), as the reference's env noise does."""
    return _ENV_SEEDS()


class VecEnv:
    """N lanes of one reference env class, stepped by one HIP kernel launch."""

    def __init__(self, family, investor, n_lanes, n_gambles=1, seed=0, prices=None, obs_days=1,
                 time_length=0, action_days=1, shuffle_days=1, sample_days=0, device="cuda:0", slice_groups=0):
        """slice_groups (market, a probe switch): lanes l and l' with l % G == l' % G
        draw the same episode slices and block shuffles; 0 = every lane its own."""
        self.family = FAMILY[family] if isinstance(family, str) else family
        self.investor = INVESTOR[investor] if isinstance(investor, str) else investor
        self.n_lanes, self.n_gambles, self.device = n_lanes, n_gambles, torch.device(device)
        self.seed = seed
        self.make_kw = dict(prices=prices, obs_days=obs_days, time_length=time_length, action_days=action_days,
                            shuffle_days=shuffle_days, sample_days=sample_days)
        cfg = _abi.EnvCfg(self.family, self.investor, n_lanes, n_gambles, obs_days, time_length,
                          action_days, shuffle_days, sample_days, int(slice_groups), seed)
        self._prices = None
        n_days = 0
        pp = None
        if prices is not None:
            self._prices = np.ascontiguousarray(prices, dtype=np.float64)
            if self._prices.ndim != 2 or self._prices.shape[1] != n_gambles:
                raise ValueError(f"prices must be [days, n_assets = {n_gambles}], got {self._prices.shape}")
            n_days = self._prices.shape[0]
            pp = self._prices.ctypes.data_as(C.c_void_p)
        h = C.c_void_p()
        check(_abi.lib().rlmd_env_create(C.byref(cfg), pp, n_days, C.byref(h)))
        self.h = h
        S, A, R, D = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        check(_abi.lib().rlmd_env_dims(h, C.byref(S), C.byref(A), C.byref(R), C.byref(D)))
        self.state_dim, self.action_dim, self.risk_dim, self.draw_dim = S.value, A.value, R.value, D.value
        dev = self.device
        self.next_state = torch.empty(n_lanes, self.state_dim, dtype=torch.float64, device=dev)
        self.reward = torch.empty(n_lanes, dtype=torch.float64, device=dev)
        self.done = torch.empty(n_lanes, 2, dtype=torch.uint8, device=dev)
        self.risk = torch.empty(n_lanes, self.risk_dim, dtype=torch.float64, device=dev)
        self.state = torch.empty(n_lanes, self.state_dim, dtype=torch.float64, device=dev)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _abi._LIB is not None:
            _abi.lib().rlmd_env_destroy(h)
            self.h = None

    def reset(self, mask=None):
        """Reset lanes (mask: bool/uint8 [N] on device, None = all); returns state f64 [N, S]."""
        m = None if mask is None else mask.to(torch.uint8).contiguous()
        check(_abi.lib().rlmd_env_reset(self.h, ptr(m), ptr(self.state), stream_ptr()))
        return self.state

    def step(self, actions, draws=None, risk=True):
        """actions [N, A] (device): f32, or f64 as inside the reference's smoothing
        window (every action-derived quantity then f64); draws f64 [N, D] to inject
        (None: Philox)."""
        f64 = actions.dtype == torch.float64
        a = actions.to(device=self.device, dtype=torch.float64 if f64 else torch.float32).contiguous()
        assert a.shape == (self.n_lanes, self.action_dim), a.shape
        d = None
        if draws is not None:
            d = draws.to(device=self.device, dtype=torch.float64).contiguous()
            assert d.shape == (self.n_lanes, self.draw_dim), d.shape
        fn = _abi.lib().rlmd_env_step_f64 if f64 else _abi.lib().rlmd_env_step
        check(fn(self.h, ptr(a), ptr(d), ptr(self.next_state), ptr(self.reward), ptr(self.done),
                 ptr(self.risk) if risk else None, stream_ptr()))
        return self.next_state, self.reward, self.done, self.risk

    def lane_state(self):
        w = np.empty(self.n_lanes, dtype=np.float64)
        t = np.empty(self.n_lanes, dtype=np.int32)
        check(_abi.lib().rlmd_env_lane_state(self.h, w.ctypes.data_as(C.c_void_p), t.ctypes.data_as(C.c_void_p)))
        return w, t

    def lane_start(self):
        """Market lanes' episode start rows (the reference's start_idx, rl_market.py:202-205)."""
        st = np.empty(self.n_lanes, dtype=np.int32)
        check(_abi.lib().rlmd_env_lane_start(self.h, st.ctypes.data_as(C.c_void_p)))
        return st


# ----------------------------------------------------------------------------
# Reference-named single-env classes (Gym interface of envs/*_envs.py)
# ----------------------------------------------------------------------------
class Box:
    """gym.spaces.Box subset used by the reference drivers."""

    def __init__(self, low, high, shape, dtype=np.float64):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def sample(self):
        return np.random.uniform(self.low, self.high).astype(self.dtype)


class _SingleEnv:
    family = None
    investor = None

    def __init__(self, n_gambles=1, device="cuda:0", seed=None, **kw):
        seed = private_seed() if seed is None else seed
        self._v = VecEnv(self.family, self.investor, 1, n_gambles, seed=seed, device=device, **kw)
        self.n_gambles = n_gambles
        self.reward_range = (MIN_REWARD[self._v.family], np.inf)
        self.observation_space = Box(-np.inf, np.inf, (self._v.state_dim,))
        self.action_space = Box(-MAX_ABS_ACTION, MAX_ABS_ACTION, (self._v.action_dim,))
        # the reference env's reused self.next_state buffer (None: a new array per step)
        self._next_state = (np.empty(self._v.state_dim, dtype=np.float64) if self._v.family in ALIAS_FAMILIES
                            else None)

    def reset(self):
        """A fresh array per call (gbm_envs.py:224-229)."""
        return self._v.reset()[0].cpu().numpy().copy()

    def step(self, action):
        """(next_state, reward, [done, learn_done], risk).  next_state is ONE array
        per env that every step overwrites in place for the families whose
        reference env does so (self.next_state: coin_flip_envs.py:128, 188-190,
        216; dice_roll_envs.py:131, 191-193; gbm_envs.py:125, 184-186, 212;
        market_envs.py:111, 172-174, 202): a driver that keeps
        ``state = next_state`` and stores ``state`` after the next step stores the
        post-step state, as the reference's loop does (rl_multiplicative.py:
        213-245).  Dice_SH returns a new array per step (dice_roll_sh_envs.py:
        336-339)."""
        return self._step(action, None)

    def _step(self, action, draws):
        """step() with optional injected draws f64 [1, D] (test hook)."""
        arr = np.asarray(action)
        a = torch.as_tensor(arr.astype(np.float64 if arr.dtype == np.float64 else np.float32).reshape(1, -1))
        ns, r, d, risk = self._v.step(a, draws=draws)
        d = d[0].cpu().numpy()
        s2 = ns[0].cpu().numpy()
        if self._next_state is not None:
            self._next_state[:] = s2
            s2 = self._next_state
        else:
            s2 = s2.copy()
        return s2, np.float64(r[0].item()), [bool(d[0]), bool(d[1])], risk[0].cpu().numpy().copy()


def _make(name, fam, inv, sh=False):
    if sh:
        def __init__(self, device="cuda:0", seed=None):
            _SingleEnv.__init__(self, 1, device=device, seed=seed)
    else:
        def __init__(self, n_gambles=1, device="cuda:0", seed=None):
            _SingleEnv.__init__(self, n_gambles, device=device, seed=seed)
    return type(name, (_SingleEnv,), {"family": fam, "investor": inv, "__init__": __init__})


_CLASSES = {}
for _p, _f in (("Coin", "coin"), ("Dice", "dice"), ("GBM", "gbm")):
    for _i in "ABC":
        _CLASSES[f"{_p}_Inv{_i}"] = _make(f"{_p}_Inv{_i}", _f, _i)
for _i, _inv in (("INSURED", "INSURED"), ("InvA", "A"), ("InvB", "B"), ("InvC", "C")):
    _CLASSES[f"Dice_SH_{_i}"] = _make(f"Dice_SH_{_i}", "dice_sh", _inv, sh=True)
globals().update(_CLASSES)


class _MarketEnv(_SingleEnv):
    """Market_Inv{A,B,C}_{D1,Dx}(n_assets, time_length, obs_days) of
    envs/market_envs.py with its interface: ``reset(assets)`` takes the
    episode's first observation and ``step(action, next_assets)`` the next one
    (scripts/rl_market.py:202-245 hands them over from its shuffled extract).
    The step is the device kernel of the vectorised loop; it reads the
    observation from a price table of time_length * action_days + 1 rows that
    this class fills one observation at a time (rlmd_env_write_prices): D1's
    observation is row t * action_days, Dx's the rows [t * action_days,
    t * action_days + obs_days) flattened and reversed
    (tools/env_resources.py:203-226), written back in row order.

    ``prices=`` instead supplies the whole extract at construction (the device
    then needs no observations; ``step(action)``)."""

    def __init__(self, n_assets, time_length, obs_days, prices=None, action_days=1, device="cuda:0", seed=None):
        self.obs_days, self.action_days, self._t = int(obs_days), int(action_days), 0
        self._feed = prices is None
        ext = (np.zeros((int(time_length) * self.action_days + 1, n_assets)) if self._feed
               else np.ascontiguousarray(prices, dtype=np.float64))
        _SingleEnv.__init__(self, n_assets, device=device, seed=seed, prices=ext, obs_days=obs_days,
                            time_length=time_length, action_days=action_days, sample_days=ext.shape[0] - 1)
        self.time_length = int(time_length) if self.obs_days == 1 else int(time_length) - self.obs_days + 1

    def _write_obs(self, t, obs):
        """The rows observation t was read from (observed_market_state inverted)."""
        n, d = self.n_gambles, self.obs_days
        obs = np.asarray(obs, dtype=np.float64).reshape(-1)
        rows = obs.reshape(1, n) if d == 1 else obs[::-1].reshape(-1, n)
        if rows.shape[0] != d:
            raise ValueError(f"observation of {obs.size} prices, expected obs_days x n_assets = {d * n}")
        rows = np.ascontiguousarray(rows)
        check(_abi.lib().rlmd_env_write_prices(self._v.h, rows.ctypes.data_as(C.c_void_p), t * self.action_days,
                                               rows.shape[0], stream_ptr()))

    def reset(self, assets=None):
        if self._feed:
            if assets is None:
                raise ValueError("reset(assets): the episode's first observation")
            self._write_obs(0, assets)
        self._t = 1
        return _SingleEnv.reset(self)

    def step(self, action, next_assets=None):
        if self._feed:
            if next_assets is None:
                raise ValueError("step(action, next_assets): the next observation")
            self._write_obs(self._t, next_assets)
        self._t += 1
        return _SingleEnv.step(self, action)


for _i in "ABC":
    for _d in ("D1", "Dx"):
        _CLASSES[f"Market_Inv{_i}_{_d}"] = type(f"Market_Inv{_i}_{_d}", (_MarketEnv,),
                                                {"family": "market", "investor": _i})
globals().update(_CLASSES)

ENV_CLASSES = dict(_CLASSES)
