// env.hip — batched multiplicative-gamble environments for gfx950.
//
// One lane = one independent Gym environment of the reference; one thread
// steps one lane (the work per lane is ~100 FP64 ops and a few dozen bytes, so
// the kernel is HBM/latency bound: SoA lane state, coalesced f32/f64 arrays).
//
// Reference semantics restated (file:line into majidsina/rlmd):
//   coin   envs/coin_flip_envs.py:150-216 (A), :290-362 (B, stop-loss = |a0| :308),
//          :436-521 (C); consts :40-93
//   dice   envs/dice_roll_envs.py:153-219, :293-365, :439-524; consts :39-96
//   gbm    envs/gbm_envs.py:147-212, :286-357, :431-515; consts :43-90
//   dice_sh envs/dice_roll_sh_envs.py:160-235 (INSURED), :290-365, :420-502, :557-645
//   market envs/market_envs.py:133-202 (D1), :611-682 (Dx) + B/C variants
//   dones  tools/env_resources.py:26-80 (any lev_max), :83-137 (all), :140-200 (market)
//   slicing tools/env_resources.py:203-291 (observed_market_state/time_slice/shuffle_data)
//
// Precision follows the reference's dtype flow under NumPy 2 for f32 actions
// (restated and pinned bit-exactly in oracle/envs.py): wealth and
// returns f64; GBM / market leverages f32 (`f32 * Python int`), coin / dice
// leverages f64 (`f32 * np.float64`); stop-loss, retention, safe-haven leverage,
// `1e4 * stop_loss`, `max(., MIN_VALUE)` and the first-step bet size f32;
// Dice_SH_INSURED leverage f32.  FP contraction is off so every rounding
// happens where NumPy's does.
#pragma clang fp contract(off)
#include <math.h>
#include <stdlib.h>
#include <stddef.h>
#include <string.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <vector>

#include "../../include/rlmd_abi.h"
#include "learn_kernels.h"
#ifdef RLMD_TIMING
// experiment builds only (tools/ts_probe.py actenv): act_env_kernel's acting-body
// stamps per workgroup — [0] / [6] realtime entry / exit, [1..5] cycles after each
// phase, [7] realtime at the start of the per-row sampling + env epilogue
__device__ unsigned long long g_ts_actenv[4096][8];
#define RLMD_TSA(i, v)                                                                    \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                                          \
      g_ts_actenv[blockIdx.x][i] = (v);                                                   \
      if ((i) == 5) g_ts_actenv[blockIdx.x][7] = __builtin_amdgcn_s_memrealtime();        \
    }                                                                                     \
  } while (0)
#endif
#include "rlmd_act_rows.h"
#include "rlmd_common.h"
#include "rlmd_internal.h"

namespace {

constexpr double kInitialValue = 1e4;
constexpr double kMinValue = 100.0;  // max(MIN_VALUE_RATIO * INITIAL_VALUE, 1)
constexpr double kMaxAbsAction = 0.99;
constexpr double kMinWeight = 1e-5;

struct FamConst {
  double max_value, min_reward, min_return, max_return, lev_factor;
};

__host__ __device__ constexpr FamConst fam_const(int fam) {
  switch (fam) {
    case RLMD_COIN: return {1e18, 1e-3, -0.9, 1e10, 2.0};
    case RLMD_DICE: return {1e18, 1e-3, -0.9, 1e10, 2.0};
    case RLMD_GBM: return {1e18, 1e-3, -2.3025850929940455 /* np.log(0.1) */, 1e10, 5.0};
    case RLMD_DICE_SH: return {1e18, 1e-6, -0.99, 1e10, 2.0};
    default: return {1e34, 1e-3, -0.9, 1e10, 3.0};
  }
}

// GBM: LOG_MEAN = DRIFT - VOL**2 / 2 (envs/gbm_envs.py:43-63)
constexpr double kGbmDrift = 0.0540025395205692;
constexpr double kGbmVol = 0.1897916175617430;
// dice_sh: I_LEV_FACTOR = (-1 - 5) / (-0.5 - 5) (envs/dice_roll_sh_envs.py:70)
constexpr double kShILev = (-1.0 - 5.0) / (-0.5 - 5.0);

#ifdef RLMD_TIMING
// experiment builds only (tools/ts_probe.py env): per-workgroup s_memrealtime at
// entry / exit of env_train_kernel and act_env_kernel, and thread 0's s_memtime
// phase stamps of block 0
__device__ unsigned long long g_ts_env[2048][8];
#define RLMD_TSE(i, v)                                                                  \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 2048) g_ts_env[blockIdx.x][i] = (v);           \
  } while (0)
#else
#define RLMD_TSE(i, v) \
  do {                 \
  } while (0)
#endif

struct EnvParams {
  int fam, inv, n_lanes, n, obs_days, time_length, action_days, shuffle_days;
  int state_dim, action_dim, risk_dim, draw_dim, ext_len, start_range, n_days;
  int slice_groups;  // market: lanes sharing slice draws in groups (lane % G; 0 = per lane)
  // replay rows store s = s' from an episode's second step on: the reference's
  // coin / dice / GBM / market envs return one self.next_state array mutated in
  // place (e.g. gbm_envs.py:125, 184-186, 212), its loop keeps state = next_state
  // (rl_multiplicative.py:245, rl_market.py:273) and stores state after the
  // next env.step (:218-220; replay.py:164-167 copies then); reset() returns a
  // fresh array (gbm_envs.py:224-229), so an episode's first row keeps the reset
  // state.  Dice_SH builds a new array per step (dice_roll_sh_envs.py:336): 0.
  int alias_state;
  uint64_t seed;
  const double* prices;  // market [n_days, n]
  // lane state
  double* wealth;
  int32_t* time;
  int32_t* start;
  uint32_t* episode;
  // per-episode log of the fused train step (nullable): one region of ep_cap
  // rows [step, lane, final reward, length, risk...] (ep_w floats) per wave,
  // ep_cnt[wave] = rows appended since the last drain (counts past ep_cap too)
  float* ep_rows;
  uint32_t* ep_cnt;
  int ep_cap, ep_w;
};

// --- categorical outcome from a uniform: NumPy legacy choice(a, p) =
// a[searchsorted(cumsum(p)/cumsum(p)[-1], u, 'right')] (pinned by tests/golden/rng_kat.npz).
__device__ __host__ inline double coin_outcome(double u) {
  const double c0 = 0.5, c1 = 0.5 + 0.5;
  const int idx = (c0 / c1 <= u) + (c1 / c1 <= u);
  return idx == 0 ? 0.5 : -0.4;
}
__device__ __host__ inline int dice_index(double u) {
  const double p0 = 1.0 / 6.0, p1 = 1.0 / 6.0, p2 = 1.0 - (1.0 / 6.0 + 1.0 / 6.0);
  const double c0 = p0, c1 = c0 + p1, c2 = c1 + p2;
  return (c0 / c2 <= u) + (c1 / c2 <= u) + (c2 / c2 <= u);
}
__device__ __host__ inline double dice_value(int idx) {
  return idx == 0 ? 0.5 : (idx == 1 ? -0.5 : 0.05);
}

// Fisher–Yates permutation of a block of `bs` (<= 16) rows for market shuffles.
// The permutation lives in one 64-bit register as 16 four-bit entries (no
// per-thread array, hence no scratch).
__device__ inline int market_perm(uint64_t seed, uint32_t lane, uint32_t ep, uint32_t blk, int bs,
                                  int pos) {
  uint64_t p = 0xFEDCBA9876543210ull;  // entry i = i
  rlmd_u32x4 w = {0, 0, 0, 0};
  for (int i = bs - 1, k = 0; i >= 1; --i, ++k) {
    if ((k & 3) == 0) w = rlmd_philox(seed, lane, ep, RLMD_TAG_MKT_PERM, blk * 4u + (k >> 2));
    const uint32_t word = (k & 3) == 0 ? w.x : (k & 3) == 1 ? w.y : (k & 3) == 2 ? w.z : w.w;
    const int j = (int)(((uint64_t)word * (uint64_t)(i + 1)) >> 32);
    const uint64_t pi = (p >> (4 * i)) & 15u, pj = (p >> (4 * j)) & 15u;
    p &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
    p |= (pj << (4 * i)) | (pi << (4 * j));
  }
  return (int)((p >> (4 * pos)) & 15u);
}

// the Philox counter of a lane's market slice draws (start row, block shuffles)
__device__ inline uint32_t slice_key(const EnvParams& P, uint32_t lane) {
  return P.slice_groups > 0 ? lane % (uint32_t)P.slice_groups : lane;
}

// source price row of extract row e (time_slice + shuffle_data)
__device__ inline int market_row(const EnvParams& P, uint32_t lane, int start, uint32_t ep, int e) {
  const int D = P.shuffle_days;
  if (D <= 1) return start + e;
  const int full = P.ext_len / D, blk = e / D, within = e % D;
  const int bs = blk < full ? D : P.ext_len - full * D;
  return start + blk * D + market_perm(P.seed, slice_key(P, lane), ep, (uint32_t)blk, bs, within);
}

// observed_market_state element k (tools/env_resources.py:203-226): D1 -> row t*ad
// asset k; Dx -> rows [t*ad, t*ad+d) flattened then reversed.
__device__ inline double market_obs(const EnvParams& P, uint32_t lane, int start, uint32_t ep,
                                    int t, int k) {
  int row, asset;
  if (P.obs_days == 1) {
    row = t * P.action_days;
    asset = k;
  } else {
    const int f = P.obs_days * P.n - 1 - k;
    row = t * P.action_days + f / P.n;
    asset = f % P.n;
  }
  return P.prices[(int64_t)market_row(P, lane, start, ep, row) * P.n + asset];
}

// np.sum / np.mean of a small array: NumPy's pairwise_sum for n <= 128
// (sequential below 8 elements, 8 accumulators otherwise).
template <typename T, typename GetF>
__device__ inline T np_sum(int n, GetF get) {
  T res;
  if (n < 8) {
    res = (T)0;
    for (int i = 0; i < n; ++i) res += get(i);
  } else {
    T r[8];
    for (int k = 0; k < 8; ++k) r[k] = get(k);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int k = 0; k < 8; ++k) r[k] += get(i + k);
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += get(i);
  }
  return res;
}
template <typename T, typename GetF>
__device__ inline T np_mean(int n, GetF get) {
  return np_sum<T>(n, get) / (T)n;
}


struct StepOut {
  double W, reward;
  bool done, learn_done;
};

struct NoDoneHook {
  __device__ void operator()(const StepOut&) const {}
};

// market: the action-independent relative prices obs(t, k) / obs(0, k) - 1 of a
// step, when a caller has them precomputed (kOn); otherwise read in the step
struct NoMrel {
  static constexpr bool kOn = false;
  __device__ double operator()(int) const { return 0.0; }
};
struct MrelRow {
  static constexpr bool kOn = true;
  const double* row;
  __device__ double operator()(int k) const { return row[k]; }
};

// One env step for one lane.  `act(i)` yields action i as AT, `draw(j)` the
// j-th uniform/normal.  Writes state element k through st(k, v) and risk
// element k through rk(k, v).
// AT is the dtype of the action array the reference's env.step receives: f32
// from the policy / warm-up sampler, f64 inside the smoothing window (np.clip
// with np.float64 bounds promotes, utils.py:345-373).  Every action-derived
// quantity follows NumPy 2's promotion from it: with f32 actions, GBM/market
// leverage (x Python int) and the half-shifted stop-loss / retention / safe-haven
// weights stay f32; with f64 actions everything is f64.
//
// FAM (the env family) is a template parameter, so each family's kernel holds
// only its own code; NG > 0 fixes n_gambles / n_assets at compile time (the
// n == 1 configurations), NG == 0 reads it from P.
template <int FAM, int NG, typename AT, typename ActF, typename DrawF, typename StF, typename RkF,
          typename DoneF = NoDoneHook, typename MrelF = NoMrel>
__device__ inline StepOut env_step_lane(const EnvParams& P, uint32_t lane, double w0, int t,
                                        int start, uint32_t ep, ActF act, DrawF draw, StF st,
                                        RkF rk, DoneF on_done = DoneF{}, MrelF mrel = MrelF{}) {
  constexpr FamConst C = fam_const(FAM);
  constexpr int fam = FAM;
  const int inv = P.inv, n = NG ? NG : P.n;
  const bool use_all = (fam == RLMD_GBM || fam == RLMD_MARKET);  // lev_max: np.all (Q4)
  const bool f32lev = use_all && sizeof(AT) == 4;                // lev = f32 action * int
  const double lev_cap64 = kMaxAbsAction * C.lev_factor;
  const float lev_cap32 = (float)lev_cap64;
  auto half_shift = [](AT a) -> AT { return (a + (AT)kMaxAbsAction) / (AT)2; };

  AT sl32 = (AT)NAN, ret32 = (AT)NAN, lev_sh32 = (AT)NAN;
  double R = 0.0, lev_mean = 0.0, lev0 = 0.0, r_sh = 0.0, r_die = 0.0;
  bool lev_max_any = false, lev_max_all = true, lev_min_all = true;
  int lev_off = 0;

  if (fam == RLMD_DICE_SH) {
    const int idx = dice_index(draw(0));
    r_die = dice_value(idx);
    r_sh = idx == 2 ? -0.99 : (idx == 0 ? -0.99 : 5.0);  // MID, UP -> -0.99 ; DOWN -> 5
    double lev;
    if (inv == RLMD_INV_INSURED) {
      const AT lev32 = act(0) * (AT)kShILev;  // action * Python float
      lev = (double)lev32;
      lev_sh32 = (AT)1 - lev32;
      lev_min_all = fabs(lev32) < (AT)kMinWeight;
    } else {
      const int ai = inv == RLMD_INV_A ? 0 : (inv == RLMD_INV_B ? 1 : 2);
      if (inv != RLMD_INV_A) sl32 = half_shift(act(0));
      if (inv == RLMD_INV_C) ret32 = half_shift(act(1));
      lev = (double)act(ai) * C.lev_factor;
      lev_sh32 = half_shift(act(ai + 1)) * (AT)1;
      lev_min_all = fabs(lev) < kMinWeight;
    }
    lev_max_any = fabs(lev) == lev_cap64;
    R = lev * r_die + (double)(lev_sh32 * (AT)r_sh);
    lev_mean = lev;
    lev0 = lev;
  } else {
    if (inv == RLMD_INV_B) {
      sl32 = fam == RLMD_COIN ? (AT)fabs(act(0)) : half_shift(act(0));  // Coin_InvB: |a0| (Q1)
      lev_off = 1;
    } else if (inv == RLMD_INV_C) {
      sl32 = half_shift(act(0));
      ret32 = half_shift(act(1));
      lev_off = 2;
    }
    auto ret_of = [&](int j) -> double {
      if (fam == RLMD_COIN) return coin_outcome(draw(j));
      if (fam == RLMD_DICE) return dice_value(dice_index(draw(j)));
      if (fam == RLMD_GBM) return (kGbmDrift - kGbmVol * kGbmVol / 2) + kGbmVol * draw(j);
      if constexpr (MrelF::kOn) return mrel(j);
      return market_obs(P, lane, start, ep, t, j) / market_obs(P, lane, start, ep, 0, j) - 1.0;
    };
    auto lev_of = [&](int j) -> double {
      const AT a = act(lev_off + j);
      return f32lev ? (double)((float)a * (float)C.lev_factor) : (double)a * C.lev_factor;
    };
    R = np_sum<double>(n, [&](int j) { return lev_of(j) * ret_of(j); });  // np.sum(lev * r)
    for (int j = 0; j < n; ++j) {
      const AT a = act(lev_off + j);
      if (f32lev) {
        const float l32 = (float)a * (float)C.lev_factor;
        lev_max_all &= fabsf(l32) == lev_cap32;
        lev_min_all &= fabsf(l32) < (float)kMinWeight;
      } else {
        const double lev = (double)a * C.lev_factor;
        lev_max_all &= fabs(lev) == lev_cap64;
        lev_max_any |= fabs(lev) == lev_cap64;
        lev_min_all &= fabs(lev) < kMinWeight;
      }
    }
    lev0 = lev_of(0);
    if (f32lev)
      lev_mean = (double)np_mean<float>(n, [&](int j) { return (float)act(lev_off + j) * (float)C.lev_factor; });
    else
      lev_mean = np_mean<double>(n, [&](int j) { return (double)act(lev_off + j) * C.lev_factor; });
  }

  // one-step return and growth factor
  double g;
  if (fam == RLMD_GBM) {
    R = fmax(R, C.min_return);
    g = fmin(exp(R), 1.0 + C.max_return);
  } else {
    R = fmin(fmax(R, C.min_return), C.max_return);
    g = 1.0 + R;
  }

  double W, mw;
  bool done_active = false;
  if (inv == RLMD_INV_A || inv == RLMD_INV_INSURED) {
    mw = kMinValue;
    W = fmin(fmax(w0 * g, kMinValue), C.max_value);
  } else {
    const AT mw32 = fmax((AT)kInitialValue * sl32, (AT)kMinValue);
    if (inv == RLMD_INV_C && w0 > kInitialValue)
      mw = kInitialValue + (w0 - kInitialValue) * (double)ret32;
    else
      mw = (double)mw32;
    // episode's first step: wealth is still the Python float 1e4 -> f32 subtraction
    const double active = t == 1 ? (double)fmax((AT)kInitialValue - mw32, (AT)0) : fmax(w0 - mw, 0.0);
    W = fmin(fmax(mw + active * g, mw), C.max_value);
    done_active = active == 0.0;
  }
  const double growth = W / kInitialValue;
  const double reward = exp(log(growth) / (double)t);

  // next state / MAX_VALUE (and done_state = any(next_state >= 1))
  bool done_state = false;
  auto put = [&](int k, double v) {
    const double s = v / C.max_value;
    done_state |= s >= 1.0;
    st(k, s);
  };
  put(0, W);
  put(1, R);
  put(2, growth);
  put(3, reward);
  if (fam == RLMD_DICE_SH) {
    put(4, r_die);
    put(5, r_sh);
  } else if (fam == RLMD_MARKET) {
    const int m = P.obs_days * n;
    for (int k = 0; k < m; ++k)
      put(4 + k, MrelF::kOn ? mrel(k)
                            : market_obs(P, lane, start, ep, t, k) / market_obs(P, lane, start, ep, 0, k) - 1.0);
  } else {
    for (int j = 0; j < n; ++j) {
      double r;
      if (fam == RLMD_COIN) r = coin_outcome(draw(j));
      else if (fam == RLMD_DICE) r = dice_value(dice_index(draw(j)));
      else r = (kGbmDrift - kGbmVol * kGbmVol / 2) + kGbmVol * draw(j);
      put(4 + j, r);
    }
  }

  const bool lev_max = use_all ? lev_max_all : lev_max_any;
  const bool done_time = fam == RLMD_MARKET &&
                         t == (P.obs_days == 1 ? P.time_length : P.time_length - P.obs_days + 1);
  const bool done = done_time || W == mw || reward < C.min_reward || R == C.min_return || lev_max ||
                    lev_min_all || done_state || done_active;
  StepOut o;
  o.W = W;
  o.reward = reward;
  o.done = done;
  o.learn_done = done && !done_state && !done_time;
  on_done(o);  // the done flags are known before the risk vector is emitted

  // risk vector
  rk(0, reward);
  rk(1, W);
  rk(2, R);
  if (fam == RLMD_DICE_SH) {
    rk(3, lev0);
    rk(4, (double)sl32);
    rk(5, (double)ret32);
    rk(6, (double)lev_sh32);
  } else {
    rk(3, lev_mean);
    int k = 4;
    if (inv == RLMD_INV_B || inv == RLMD_INV_C) rk(k++, (double)sl32);
    if (inv == RLMD_INV_C) rk(k++, (double)ret32);
    if (n > 1) {
      for (int j = 0; j < n; ++j) {
        const AT a = act(lev_off + j);
        rk(k + j, f32lev ? (double)((float)a * (float)C.lev_factor) : (double)a * C.lev_factor);
      }
    }
  }
  return o;
}

// draws for gamble j: Philox(seed, lane, step, ENV_DRAW, j/2), two per block
template <int FAM>
__device__ inline double philox_draw(const EnvParams& P, uint32_t lane, uint32_t step, int j) {
  const rlmd_u32x4 v = rlmd_philox(P.seed, lane, step, RLMD_TAG_ENV_DRAW, (uint32_t)(j >> 1));
  if (FAM == RLMD_GBM) {
    double z0, z1;
    rlmd_normal2(v, z0, z1);
    return (j & 1) ? z1 : z0;
  }
  return (j & 1) ? rlmd_u01(v.z, v.w) : rlmd_u01(v.x, v.y);
}

// reset one lane: episode start (market: new slice), state element writer
// start_at >= 0 (market): the episode's first price row is given (eval_market's
// gap index) instead of drawn.
// ep_now >= 0: the lane's current episode counter, already in a register (the
// training step's epilogue loaded it with the lane state; re-reading it here put
// a dependent global load into the tail of every wave with a finished lane).
template <int FAM, typename StF>
__device__ inline void env_reset_lane(const EnvParams& P, uint32_t lane, StF st, int start_at = -1,
                                      int64_t ep_now = -1) {
  P.wealth[lane] = kInitialValue;
  P.time[lane] = 1;
  const uint32_t ep = (ep_now >= 0 ? (uint32_t)ep_now : P.episode[lane]) + 1;
  P.episode[lane] = ep;
  constexpr FamConst C = fam_const(FAM);
  st(0, kInitialValue / C.max_value);
  st(1, 0.0);
  st(2, 1.0 / C.max_value);
  st(3, 1.0 / C.max_value);
  if (FAM == RLMD_MARKET) {
    const rlmd_u32x4 v = rlmd_philox(P.seed, slice_key(P, lane), ep, RLMD_TAG_MKT_START, 0);
    const int start = start_at >= 0 ? start_at : (int)rlmd_below(v.x, v.y, (uint64_t)P.start_range);
    P.start[lane] = start;
    const int m = P.obs_days * P.n;
    for (int k = 0; k < m; ++k)
      st(4 + k, P.obs_days == 1 ? 0.0 : market_obs(P, lane, start, ep, 0, k) / C.max_value);
  } else {
    for (int k = 4; k < P.state_dim; ++k) st(k, 0.0);
  }
}

// Finished-episode statistics of the fused train step: each launch writes one
// row {episodes, sum of final rewards, sum of lengths, 0} per workgroup into
// part_out; the next launch's block 0 (or rlmd_train_flush_stats) adds the
// rows of fold_src into the caller's f64[4] accumulator fold_dst.
struct StatFold {
  double* part_out;
  const double* fold_src;
  double* fold_dst;
  int rows;
};

// one 256-thread block: fixed-order strided sums, then a fixed tree.  fr: LDS
// [3][256] doubles — the caller's dynamic LDS where it has one (act_env_kernel
// folds before its acting body uses it), so that the fold's 6 KB do not cost
// the acting kernel a workgroup per CU
__device__ inline void fold_stat_rows(const double* src, int rows, double* dst, double (*fr)[256]) {
  const int i = threadIdx.x;
  double a = 0.0, b = 0.0, c = 0.0;
  for (int r = i; r < rows; r += blockDim.x) {
    a += src[(int64_t)r * 4 + 0];
    b += src[(int64_t)r * 4 + 1];
    c += src[(int64_t)r * 4 + 2];
  }
  fr[0][i] = a;
  fr[1][i] = b;
  fr[2][i] = c;
  __syncthreads();
  for (int h = blockDim.x >> 1; h > 0; h >>= 1) {
    if (i < h) {
      fr[0][i] += fr[0][i + h];
      fr[1][i] += fr[1][i + h];
      fr[2][i] += fr[2][i + h];
    }
    __syncthreads();
  }
  if (i < 3) dst[i] += fr[i][0];
  __syncthreads();
}

__global__ void __launch_bounds__(256) stat_fold_kernel(const double* src, int rows, double* dst) {
  __shared__ double fr[3][256];
  fold_stat_rows(src, rows, dst, fr);
}

template <int FAM>
__global__ void __launch_bounds__(256) env_reset_kernel(EnvParams P, const uint8_t* mask, double* state) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= P.n_lanes) return;
  if (mask && !mask[lane]) return;
  env_reset_lane<FAM>(P, lane, [&](int k, double v) {
    if (state) state[(int64_t)lane * P.state_dim + k] = v;
  });
}

template <int FAM, int NG, typename AT>
__global__ void __launch_bounds__(256) env_step_kernel(EnvParams P, uint32_t step, const AT* __restrict__ actions,
                                const double* __restrict__ draws, double* next_state,
                                double* reward, uint8_t* done, double* risk) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= P.n_lanes) return;
  const AT* a = actions + (int64_t)lane * P.action_dim;
  const double w0 = P.wealth[lane];
  const int t = P.time[lane];
  const int start = FAM == RLMD_MARKET ? P.start[lane] : 0;
  const uint32_t ep = P.episode[lane];
  StepOut o = env_step_lane<FAM, NG, AT>(
      P, lane, w0, t, start, ep, [&](int i) { return a[i]; },
      [&](int j) {
        return draws ? draws[(int64_t)lane * P.draw_dim + j] : philox_draw<FAM>(P, lane, step, j);
      },
      [&](int k, double v) { next_state[(int64_t)lane * P.state_dim + k] = v; },
      [&](int k, double v) {
        if (risk) risk[(int64_t)lane * P.risk_dim + k] = v;
      });
  P.wealth[lane] = o.W;
  P.time[lane] = t + 1;
  reward[lane] = o.reward;
  done[2 * lane] = o.done;
  done[2 * lane + 1] = o.learn_done;
}

// Upper bound of the action count when it is known at compile time (dice_sh:
// <= 4; NG > 0: NG + 2 for InvC), else 0 (read through memory per use).
// ring row of a lane: the host hands ring_base already reduced mod capacity, so
// one conditional subtract replaces the 64-bit remainder (a long software
// sequence on the lane's critical path); rings smaller than the lane count wrap
// more than once and keep the remainder
__device__ __forceinline__ int64_t ring_row(int64_t base, int64_t lane, int64_t cap) {
  int64_t r = base + lane;
  if (r >= cap) r = r - cap < cap ? r - cap : r % cap;
  return r;
}

template <int FAM, int NG>
constexpr int kActRegs = FAM == RLMD_DICE_SH ? 4 : (NG > 0 ? NG + 2 : 0);

// ---------------------------------------------------------------------------
// fused training step: action (warm-up draw | policy) -> action_window clip ->
// env step -> replay insert (s, a, r, s', learn_done) -> auto reset.
// ---------------------------------------------------------------------------
// AT = the dtype of the action array the reference's env.step receives:
// float64 during warm-up (action_space.sample() of the float64 Box) and inside
// the smoothing window (np.clip with np.float64 bounds, utils.py:345-373);
// float32 for policy actions afterwards.  The replay stores the f32 cast, as the
// reference's float64 buffer does when it batches to torch.float.
// Every load that does not depend on computed data (lane state, actions, the
// current observation) is issued before the first store, so the lane's memory
// traffic is one read round and one write round.
template <int FAM, int NG, typename AT>
__global__ void __launch_bounds__(256) env_train_kernel(EnvParams P, uint32_t step, const float* actions,
                                                        int random_actions, int abs_actions, double clip_lo,
                                                        double clip_hi, float* obs, rlmd::ReplayView rb,
                                                        int64_t ring_base, StatFold sf) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  RLMD_TSE(0, __builtin_amdgcn_s_memrealtime());
  RLMD_TSE(1, __builtin_amdgcn_s_memtime());
  // block 0 folds the previous launch's per-block rows into the caller's
  // accumulator first (its rows are complete: that launch has ended)
  if (blockIdx.x == 0 && sf.fold_src) {
    __shared__ double fr[3][256];
    fold_stat_rows(sf.fold_src, sf.rows, sf.fold_dst, fr);
  }
  double st_n = 0.0, st_r = 0.0, st_t = 0.0;  // finished-episode stats of this lane
  if (lane < P.n_lanes) {
    const int S = P.state_dim, A = P.action_dim;
    const double w0 = P.wealth[lane];
    const int t = P.time[lane];
    const int start = FAM == RLMD_MARKET ? P.start[lane] : 0;
    const uint32_t ep = P.episode[lane];
    // per-episode log: this wave's row count, loaded with the lane state
    const uint32_t ep_base = P.ep_rows ? P.ep_cnt[lane >> 6] : 0u;
    int64_t ep_slot = -1;
    // action i: warm-up Philox draw (|.| unless GBM/market) or the policy's, then the
    // smoothing-window clip
    // the policy's action i: a predicated buffer load (no branch around it, so it
    // is not waited on at a merge)
    const __amdgpu_buffer_rsrc_t ra = rlmd_rsrc(actions, actions ? (int64_t)P.n_lanes * A * 4 : 0);
    auto act_of = [&](int i) -> AT {
      const double pv = (double)rlmd_ldf(ra, (int64_t)lane * A + i, !random_actions && i < A);
      double v = pv;
      if (random_actions) {  // Box(-0.99, 0.99, float64).sample() = low + (high - low) * random_sample()
        const rlmd_u32x4 w = rlmd_philox(P.seed, lane, step, RLMD_TAG_WARMUP_ACTION, (uint32_t)(i >> 1));
        const double u = (i & 1) ? rlmd_u01(w.z, w.w) : rlmd_u01(w.x, w.y);
        v = -kMaxAbsAction + 2.0 * kMaxAbsAction * u;
        if (abs_actions) v = fabs(v);
      }
      if (sizeof(AT) == 4) return (AT)v;  // policy action outside the window: exact f32
      return (AT)fmin(fmax(v, clip_lo), clip_hi);
    };
    // the actions in named registers when their count is known at compile time (an
    // array here was promoted to LDS, each element's load waited on at its store)
    constexpr int AR = kActRegs<FAM, NG>;
    static_assert(AR <= 4, "action registers");
    const AT a0 = AR > 0 && 0 < A ? act_of(0) : (AT)0, a1 = AR > 1 && 1 < A ? act_of(1) : (AT)0;
    const AT a2 = AR > 2 && 2 < A ? act_of(2) : (AT)0, a3 = AR > 3 && 3 < A ? act_of(3) : (AT)0;
    auto act = [&](int i) -> AT {
      if constexpr (AR > 0) {
        return i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : a3;
      } else {
        return act_of(i);
      }
    };
    const int64_t row = ring_row(ring_base, lane, rb.capacity);
    // the stored s: the reference's aliased post-step state from an episode's
    // second step on (EnvParams::alias_state), else the current obs unchanged
    const bool alias = P.alias_state && t > 1;
    // gfx9 counts stores in vmcnt, so a store issued before the compute would be
    // waited on at the first use of a loaded value: the first 8 obs elements are
    // loaded now and stored after the step; the rest (market Dx only) are copied
    // here, before the next-state writes overwrite obs.
    const __amdgpu_buffer_rsrc_t ro = rlmd_rsrc(obs, (int64_t)P.n_lanes * S * 4);
    float s0[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s0[j] = rlmd_ldf(ro, (int64_t)lane * S + j, j < S && !alias);
    if (!alias) {
      for (int k0 = 8; k0 < S; k0 += 8) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rlmd_ldf(ro, (int64_t)lane * S + k0 + j, k0 + j < S);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j < S) rb.state[row * S + k0 + j] = v[j];
      }
    }

    // the one draw of a single-gamble lane depends on (seed, lane, step) only: its
    // Philox + f64 Box-Muller chain runs while the lane-state loads are in flight
    constexpr bool one_draw = NG == 1 && FAM != RLMD_MARKET;
    const double dr0 = one_draw ? philox_draw<FAM>(P, lane, step, 0) : 0.0;
    RLMD_TSE(2, __builtin_amdgcn_s_memtime());
    StepOut o = env_step_lane<FAM, NG, AT>(
        P, lane, w0, t, start, ep, act,
        [&](int j) { return one_draw ? dr0 : philox_draw<FAM>(P, lane, step, j); },
        [&](int k, double v) {
          const float f = (float)v;
          rb.next_state[row * S + k] = f;
          if (alias) rb.state[row * S + k] = f;
          obs[(int64_t)lane * S + k] = f;
        },
        [&](int k, double v) {
          if (ep_slot >= 0 && k < P.ep_w - 4) P.ep_rows[ep_slot * P.ep_w + 4 + k] = (float)v;
        },
        [&](const StepOut& so) {
          // finished lanes of this wave take consecutive rows of its region in lane
          // order (ballot prefix); the lowest finishing lane publishes the count
          if (!P.ep_rows) return;
          const uint64_t m = __ballot(so.done);
          if (m == 0) return;
          const int lid = threadIdx.x & 63;
          if (so.done) {
            const uint32_t at = ep_base + (uint32_t)__popcll(m & ((1ull << lid) - 1ull));
            if (at < (uint32_t)P.ep_cap) ep_slot = (int64_t)(lane >> 6) * P.ep_cap + at;
          }
          if (lid == __ffsll((unsigned long long)m) - 1) P.ep_cnt[lane >> 6] = ep_base + (uint32_t)__popcll(m);
        });
    RLMD_TSE(3, __builtin_amdgcn_s_memtime());
    if (ep_slot >= 0) {
      float* er = P.ep_rows + ep_slot * P.ep_w;
      er[0] = (float)step;
      er[1] = (float)lane;
      er[2] = (float)o.reward;
      er[3] = (float)t;
    }
    if (!alias) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < S) rb.state[row * S + j] = s0[j];
    }
    for (int i = 0; i < A; ++i) rb.action[row * A + i] = (float)act(i);
    rb.reward[row] = (float)o.reward;  // max(reward, r_abs_zero = -inf)
    rb.done[row] = o.learn_done;
    if (rb.n_steps > 1) rlmd::ms_record(rb, lane, row, o.learn_done);
    if (o.done) {
      st_n = 1.0;
      st_r = o.reward;
      st_t = (double)t;
      env_reset_lane<FAM>(P, lane, [&](int k, double v) { obs[(int64_t)lane * S + k] = (float)v; }, -1, ep);
    } else {
      P.wealth[lane] = o.W;
      P.time[lane] = t + 1;
    }
    RLMD_TSE(4, __builtin_amdgcn_s_memtime());
  }
  // episode statistics: a fixed-order block reduction into this block's row of
  // the launch's partial buffer (plain stores; device-scope atomics on one
  // address from every wave serialise across the XCDs and cost more than the
  // whole env step)
  if (sf.part_out) {
    __shared__ double red[3][256 / 64];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      st_n += __shfl_xor(st_n, m, 64);
      st_r += __shfl_xor(st_r, m, 64);
      st_t += __shfl_xor(st_t, m, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = st_n;
      red[1][w] = st_r;
      red[2][w] = st_t;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
      const int q = threadIdx.x;
      double v = 0.0;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) v += red[q][i];
      sf.part_out[(int64_t)blockIdx.x * 4 + q] = v;
    }
  }
  RLMD_TSE(5, __builtin_amdgcn_s_memtime());
  RLMD_TSE(6, __builtin_amdgcn_s_memrealtime());
}

// ---------------------------------------------------------------------------
// fused acting + env step (post-window policy steps of the training loop):
// rlmd_act_rows.h's 64-row acting body, then, on the row's own thread, the env
// step of env_train_kernel with the action still in registers and the
// observation still in LDS — one launch per vector step instead of two, and the
// actions never round-trip through HBM.  This file compiles with FP contraction
// off (the env's NumPy rounding), and so does act.hip: the fused and two-launch
// steps produce bit-equal actions, rings and wealth.
// ---------------------------------------------------------------------------
// the state width when it is a compile-time constant (0: run time): Dice_SH 6,
// coin / dice / GBM 4 + n at a fixed n; market rows depend on obs_days
template <int FAM, int NG>
constexpr int kStateRegs = FAM == RLMD_MARKET ? 0 : (FAM == RLMD_DICE_SH ? 6 : (NG > 0 ? 4 + NG : 0));

typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f32x2u __attribute__((ext_vector_type(2), aligned(4)));

// one row of N floats at a 4-byte aligned address as 16-, 8- and 4-byte stores
// (gfx950 global stores take dword alignment): a 5- or 6-float replay row is two
// store instructions instead of five or six
template <int N>
__device__ __forceinline__ void store_row(float* dst, const float* v) {
  int k = 0;
#pragma unroll
  for (; k + 4 <= N; k += 4) *reinterpret_cast<f32x4u*>(dst + k) = f32x4u{v[k], v[k + 1], v[k + 2], v[k + 3]};
  if constexpr (N % 4 >= 2) {
    *reinterpret_cast<f32x2u*>(dst + k) = f32x2u{v[k], v[k + 1]};
    k += 2;
  }
  if constexpr (N % 2 == 1) dst[k] = v[k];
}

// act_env_kernel's explicit arguments as laid out in the kernarg segment (in
// order, each at its natural alignment): their exact byte count bounds the
// argument prefetch
struct ActEnvKargs {
  rlmd::FusedActArgs a;
  EnvParams P;
  uint32_t step;
  float* obs;
  rlmd::ReplayView rb;
  int64_t ring_base;
  StatFold sf;
};

#ifndef RLMD_ACT_PARK
#define RLMD_ACT_PARK 1  // act_env_kernel: the lane state and draw parked in LDS across the acting body
#endif
template <int FAM, int NG, int H1P, int NB, int SP, int MA, int WPC>
__global__ void __launch_bounds__(256, H1P == 256 ? (MA == rlmd::actrows::kMaxA ? WPC : 2) : 1) act_env_kernel(rlmd::FusedActArgs a, EnvParams P, uint32_t step,
                                                      float* obs, rlmd::ReplayView rb, int64_t ring_base,
                                                      StatFold sf) {
  rlmd_kernarg_prefetch<(int)(offsetof(ActEnvKargs, sf) + sizeof(StatFold))>();
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (blockIdx.x == 0 && sf.fold_src)
    fold_stat_rows(sf.fold_src, sf.rows, sf.fold_dst, reinterpret_cast<double(*)[256]>(smem));
  const int tid = threadIdx.x;
  const int lane = blockIdx.x * rlmd::actrows::kRows + tid;  // this thread's env lane (tid < 64)
  const bool mine = tid < rlmd::actrows::kRows && lane < P.n_lanes;
  double w0 = 0.0, dr0 = 0.0;
  int t = 1, start = 0;
  uint32_t ep = 0, ep_base = 0;
  double st_n = 0.0, st_r = 0.0, st_t = 0.0;
  constexpr bool one_draw = NG == 1 && FAM != RLMD_MARKET;
  // the lane state, loaded with the acting body's first load round, and the
  // lane's draw (independent of the action: its f64 Box-Muller / uniform chain
  // runs under the acting body instead of in the epilogue's tail)
  auto pro = [&] {
    if (mine) {
      if (one_draw) dr0 = philox_draw<FAM>(P, lane, step, 0);
      w0 = P.wealth[lane];
      t = P.time[lane];
      if (FAM == RLMD_MARKET) start = P.start[lane];
      ep = P.episode[lane];
      ep_base = P.ep_rows ? P.ep_cnt[lane >> 6] : 0u;
    }
  };
  // the lane state and draw through LDS (rlmd_act_rows.h park()): [word][64 rows]
  constexpr bool PARK = RLMD_ACT_PARK && rlmd::actrows::act_park(H1P, SP, MA, WPC);
  constexpr rlmd::actrows::ActLds LYP = rlmd::actrows::act_lds(H1P, SP, MA, PARK);
  uint32_t* pk = reinterpret_cast<uint32_t*>(smem + LYP.total);
  constexpr int kR = rlmd::actrows::kRows;
  auto park = [&] {
    if (PARK && tid < kR) {
      const uint64_t wb = __builtin_bit_cast(uint64_t, w0), db = __builtin_bit_cast(uint64_t, dr0);
      pk[0 * kR + tid] = (uint32_t)wb;
      pk[1 * kR + tid] = (uint32_t)(wb >> 32);
      pk[2 * kR + tid] = (uint32_t)db;
      pk[3 * kR + tid] = (uint32_t)(db >> 32);
      pk[4 * kR + tid] = (uint32_t)t;
      pk[5 * kR + tid] = ep;
      pk[6 * kR + tid] = ep_base;
      pk[7 * kR + tid] = (uint32_t)start;
    }
  };
  auto epi = [&](int, int b, const float* acts, const float* obs_row) {
    if constexpr (PARK) {
      w0 = __builtin_bit_cast(double, (uint64_t)pk[0 * kR + tid] | ((uint64_t)pk[1 * kR + tid] << 32));
      dr0 = __builtin_bit_cast(double, (uint64_t)pk[2 * kR + tid] | ((uint64_t)pk[3 * kR + tid] << 32));
      t = (int)pk[4 * kR + tid];
      ep = pk[5 * kR + tid];
      ep_base = pk[6 * kR + tid];
      start = (int)pk[7 * kR + tid];
    }
    const int S = P.state_dim, A = P.action_dim;
    // the action by a fixed selection chain (no runtime-indexed register array)
    auto act = [&](int i) -> float {
      if constexpr (MA == 2) return i == 0 ? acts[0] : acts[1];
      else return i == 0 ? acts[0] : i == 1 ? acts[1] : i == 2 ? acts[2] : acts[3];
    };
    const int64_t row = ring_row(ring_base, b, rb.capacity);
    // the stored s: the aliased post-step state from an episode's second step on
    // (EnvParams::alias_state, env_train_kernel), else this row's observation
    const bool alias = P.alias_state && t > 1;
    int64_t ep_slot = -1;
    // a compile-time state width keeps the next state in registers (every put()
    // index is a constant once env_step_lane is inlined) for row-wide stores
    constexpr int SR = kStateRegs<FAM, NG>;
    float ns[SR > 0 ? SR : 1];
    const StepOut o = env_step_lane<FAM, NG, float>(
        P, b, w0, t, start, ep, act, [&](int j) { return one_draw ? dr0 : philox_draw<FAM>(P, b, step, j); },
        [&](int k, double v) {
          const float f = (float)v;
          if constexpr (SR > 0) {
            ns[k] = f;
          } else {
            rb.next_state[row * S + k] = f;
            if (alias) rb.state[row * S + k] = f;
            obs[(int64_t)b * S + k] = f;
          }
        },
        [&](int k, double v) {
          if (ep_slot >= 0 && k < P.ep_w - 4) P.ep_rows[ep_slot * P.ep_w + 4 + k] = (float)v;
        },
        [&](const StepOut& so) {
          if (!P.ep_rows) return;
          const uint64_t m = __ballot(so.done);
          if (m == 0) return;
          const int lid = threadIdx.x & 63;
          if (so.done) {
            const uint32_t at = ep_base + (uint32_t)__popcll(m & ((1ull << lid) - 1ull));
            if (at < (uint32_t)P.ep_cap) ep_slot = (int64_t)(b >> 6) * P.ep_cap + at;
          }
          if (lid == __ffsll((unsigned long long)m) - 1) P.ep_cnt[b >> 6] = ep_base + (uint32_t)__popcll(m);
        });
    if (ep_slot >= 0) {
      float* er = P.ep_rows + ep_slot * P.ep_w;
      er[0] = (float)step;
      er[1] = (float)b;
      er[2] = (float)o.reward;
      er[3] = (float)t;
    }
    if constexpr (SR > 0) {
      float s0[SR];
#pragma unroll
      for (int j = 0; j < SR; ++j) s0[j] = alias ? ns[j] : obs_row[j];
      store_row<SR>(rb.state + row * SR, s0);
      store_row<SR>(rb.next_state + row * SR, ns);
      if (!o.done) store_row<SR>(obs + (int64_t)b * SR, ns);  // a finished lane's obs is its reset state
    } else if (!alias) {
      for (int j = 0; j < S; ++j) rb.state[row * S + j] = obs_row[j];
    }
    if (A == 2)
      *reinterpret_cast<f32x2u*>(rb.action + row * 2) = f32x2u{act(0), act(1)};
    else
      for (int i = 0; i < A; ++i) rb.action[row * A + i] = act(i);
    rb.reward[row] = (float)o.reward;
    rb.done[row] = o.learn_done;
    if (rb.n_steps > 1) rlmd::ms_record(rb, b, row, o.learn_done);
    if (o.done) {
      st_n = 1.0;
      st_r = o.reward;
      st_t = (double)t;
      env_reset_lane<FAM>(P, b, [&](int k, double v) { obs[(int64_t)b * S + k] = (float)v; }, -1, ep);
    } else {
      P.wealth[b] = o.W;
      P.time[b] = t + 1;
    }
  };
  rlmd::actrows::act_rows<H1P, NB, SP, MA, PARK>(a, smem, pro, epi, park);
  if (sf.part_out) {  // the block's finished-episode statistics, as env_train_kernel
    __shared__ double red[3][256 / 64];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      st_n += __shfl_xor(st_n, m, 64);
      st_r += __shfl_xor(st_r, m, 64);
      st_t += __shfl_xor(st_t, m, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = st_n;
      red[1][w] = st_r;
      red[2][w] = st_t;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
      const int q = threadIdx.x;
      double v = 0.0;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) v += red[q][i];
      sf.part_out[(int64_t)blockIdx.x * 4 + q] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// evaluation episodes (tools/eval_episodes.py:176-399): every lane is one eval
// episode from its reset state, the policy's action held constant for the whole
// episode (action_window applied first when warmup < cum_step <= smoothing:
// float64 actions then), stepped until done or max_steps; the last step's
// reward, the step count and the last risk vector are kept.  Draws: injected
// [N, max_steps, D] or Philox at (lane, step_base + k).
// ---------------------------------------------------------------------------
template <int FAM, int NG, typename AT>
__global__ void __launch_bounds__(256) eval_rollout_kernel(EnvParams P, uint32_t step_base, const float* actions,
                                                           int max_steps, double clip_lo, double clip_hi,
                                                           const double* draws, double* reward_out,
                                                           int32_t* steps_out, double* risk_out) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= P.n_lanes) return;
  const int A = P.action_dim, D = P.draw_dim, R = P.risk_dim;
  auto act = [&](int i) -> AT {
    const double v = (double)actions[(int64_t)lane * A + i];
    if (sizeof(AT) == 4) return (AT)v;
    return (AT)fmin(fmax(v, clip_lo), clip_hi);
  };
  double w = P.wealth[lane];
  int t = P.time[lane];
  const int start = FAM == RLMD_MARKET ? P.start[lane] : 0;
  const uint32_t ep = P.episode[lane];
  double run_reward = 0.0;
  int k = 0;
  while (k < max_steps) {
    const StepOut o = env_step_lane<FAM, NG, AT>(
        P, lane, w, t, start, ep, act,
        [&](int j) {
          return draws ? draws[((int64_t)lane * max_steps + k) * D + j] : philox_draw<FAM>(P, lane, step_base + k, j);
        },
        [&](int, double) {},
        [&](int r, double v) {
          if (risk_out) risk_out[(int64_t)lane * R + r] = v;
        });
    run_reward = o.reward;
    ++k;
    if (o.done) break;
    w = o.W;
    ++t;
  }
  P.wealth[lane] = w;
  P.time[lane] = t;
  reward_out[lane] = run_reward;
  steps_out[lane] = k;
}

// ---------------------------------------------------------------------------
// market evaluation (tools/eval_episodes.py:402-611): every lane is one eval
// episode over the test slice starting at its gap index, re-shuffled in blocks of
// test_shuffle_days; the policy acts on every step (the caller runs the
// deterministic policy between steps), action_window applied when
// warmup < cum_steps <= smoothing (float64 actions then).  A lane stops at its
// first done; its last reward, step count and risk vector are kept.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) eval_market_reset_kernel(EnvParams P, const int32_t* start_at, float* obs,
                                                                double* reward, int32_t* steps, uint8_t* live) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= P.n_lanes) return;
  const int st = start_at[lane];
  steps[lane] = 0;
  reward[lane] = __builtin_nan("");
  // a start whose extract would leave the price table is refused per lane (never read)
  if (st < 0 || st + P.ext_len > P.n_days) {
    live[lane] = 0;
    return;
  }
  env_reset_lane<RLMD_MARKET>(P, lane, [&](int k, double v) { obs[(int64_t)lane * P.state_dim + k] = (float)v; },
                              st);
  live[lane] = 1;
}

template <int NG, typename AT>
__global__ void __launch_bounds__(256) eval_market_step_kernel(EnvParams P, const float* actions, double clip_lo,
                                                               double clip_hi, float* obs, double* reward_out,
                                                               int32_t* steps_out, double* risk_out, uint8_t* live) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= P.n_lanes || !live[lane]) return;
  const int A = P.action_dim, S = P.state_dim, R = P.risk_dim;
  auto act = [&](int i) -> AT {
    const double v = (double)actions[(int64_t)lane * A + i];
    if (sizeof(AT) == 4) return (AT)v;
    return (AT)fmin(fmax(v, clip_lo), clip_hi);
  };
  const double w0 = P.wealth[lane];
  const int t = P.time[lane];
  const int start = P.start[lane];
  const uint32_t ep = P.episode[lane];
  const StepOut o = env_step_lane<RLMD_MARKET, NG, AT>(
      P, lane, w0, t, start, ep, act, [&](int) { return 0.0; },
      [&](int k, double v) { obs[(int64_t)lane * S + k] = (float)v; },
      [&](int k, double v) {
        if (risk_out) risk_out[(int64_t)lane * R + k] = v;
      });
  reward_out[lane] = o.reward;
  steps_out[lane] = t;
  if (o.done) {
    live[lane] = 0;
  } else {
    P.wealth[lane] = o.W;
    P.time[lane] = t + 1;
  }
}

// ---------------------------------------------------------------------------
// market evaluation as ONE launch: each 16-lane workgroup runs its lanes' whole
// test slice in a day loop — the deterministic policy (the arithmetic of
// rlmd_act_rows.h's body at one 16-row MFMA tile: layer 1 on the f32 MFMA, bf16
// layer 2, DPP head sums, tanh) and then, on the lane's own thread, the market
// step of eval_market_step_kernel with the action in registers and the next
// observation written straight into LDS.  W1 / b1 are staged into LDS once,
// the head weights and biases sit in registers for the whole episode, and the
// fc2 fragments too where they fit (SAC 256/256: 32 x 16 B per lane); only the
// price rows are read per day.  Replaces the host loop of one acting and one
// step launch per day.  The loop ends when every lane of the block is done.
// ---------------------------------------------------------------------------
template <int NG, typename AT, int H1P, int NB, int SP>
__global__ void __launch_bounds__(256) eval_market_loop_kernel(rlmd::FusedActArgs a, EnvParams P, int T,
                                                               double clip_lo, double clip_hi, double* reward_out,
                                                               int32_t* steps_out, double* risk_out, uint8_t* live_io,
                                                               float* obs_out) {
  using namespace rlmd::actrows;
  constexpr int kR = 16;
  constexpr int HP = H1P + 8;
  constexpr int NT = L1Tiles<H1P>::NT, NTP = L1Tiles<H1P>::NTP;
  constexpr int nS = H1P / 32;
  constexpr bool kRegW2 = NB * nS <= 32;
  __shared__ __attribute__((aligned(16))) unsigned short h1s[kR * HP];
  __shared__ float part[4 * kR * 2 * kMaxA];
  __shared__ float w1s[SP * 16 * NTP + H1P];  // w1g [SP][16][NTP], then b1 [H1P]
  __shared__ float obs_s[kR * SP];
  __shared__ double risk_s[kR * 8];  // the lanes' last risk rows (risk_dim <= 8), written out once
  __shared__ double p0_s[kR * 16];   // the episode's first observed prices obs(0, k), k < m <= 16
  __shared__ double mrel_s[2 * kR * 16];  // obs(t, k) / obs(0, k) - 1, double-buffered by day parity
  float* const b1s = w1s + SP * 16 * NTP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * kR;
  const rlmd::NetOff& o = a.off;
  const int S = a.S, A = a.A, H1 = a.H1, H2 = a.H2;
  const int nh = a.algo == RLMD_SAC ? 2 * A : A;
  // ---- once per episode: head weights / fc2 bias of this wave's columns, the
  //      head biases, W1 / b1 / the first observations into LDS, lane state
  const int col0 = 16 * NB * wave;
  float hw[NB][2 * kMaxA];
  float b2v[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int c = col0 + 16 * nb + (lane & 15);
    const bool live = c < H2;
    b2v[nb] = live ? a.params[o.b2 + c] : 0.f;
#pragma unroll
    for (int h = 0; h < 2 * kMaxA; ++h) {
      const int64_t base = h < A ? o.w3 + (int64_t)h * H2 : o.w4 + (int64_t)(h - A) * H2;
      hw[nb][h] = live && h < nh ? a.params[base + c] : 0.f;
    }
  }
  const bf16x8* wf = reinterpret_cast<const bf16x8*>(a.w2bf) + (int64_t)(NB * wave) * nS * 64 + lane;
  bf16x8 wreg[kRegW2 ? NB : 1][kRegW2 ? nS : 1];
  if constexpr (kRegW2) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int s = 0; s < nS; ++s) wreg[nb][s] = wf[(nb * nS + s) * 64];
  }
  const bool mine = tid < kR && row0 + tid < a.n;
  const int b = row0 + tid;
  float mu_b[kMaxA], ls_b[kMaxA];
#pragma unroll
  for (int j = 0; j < kMaxA; ++j) {
    mu_b[j] = mine && j < A ? a.params[o.b3 + j] : 0.f;
    ls_b[j] = mine && j < A && a.algo == RLMD_SAC ? a.params[o.b4 + j] : 0.f;
  }
  bool alive = false;
  double w = 0.0, last_r = 0.0;
  int t = 0, start = 0, last_t = 0;
  uint32_t ep = 0;
  if (mine) {
    alive = live_io[b] != 0;
    w = P.wealth[b];
    t = P.time[b];
    start = P.start[b];
    ep = P.episode[b];
    last_r = reward_out[b];
    last_t = steps_out[b];
  }
  for (int e = tid; e < SP * 16 * NTP + H1P; e += 256) {
    const bool isb = e >= SP * 16 * NTP;
    const int k = e / (16 * NTP), jt = e - k * (16 * NTP);
    const int jj = jt / NTP, tt = jt - jj * NTP;
    const int c = isb ? e - SP * 16 * NTP : 16 * tt + jj;
    const bool ok = c < H1 && (isb || (tt < NT && k < S));
    w1s[e] = ok ? a.params[o.w1 + (isb ? H1 * S + c : c * S + k)] : 0.f;
  }
  for (int e = tid; e < kR * SP; e += 256) {
    const int r = e / SP, k = e - r * SP;
    obs_s[e] = (k < S && row0 + r < a.n) ? a.obs[(int64_t)(row0 + r) * S + k] : 0.f;
  }
  if (!__syncthreads_or(alive)) return;
  if (mine && risk_out)
    for (int k = 0; k < P.risk_dim; ++k) risk_s[tid * 8 + k] = risk_out[(int64_t)b * P.risk_dim + k];
  const int m = P.obs_days * (NG ? NG : P.n);  // observed prices per state (<= 16: host check)
  // wave 1's threads 64 + r precompute lane r's relative prices; p0_s is theirs
  const bool pre = tid >= 64 && tid < 64 + kR && row0 + tid - 64 < a.n && live_io[row0 + tid - 64] != 0;
  const int r1 = tid - 64, b1 = row0 + r1;
  int t1 = 0, start1 = 0;
  uint32_t ep1 = 0;
  if (pre) {
    t1 = P.time[b1];
    start1 = P.start[b1];
    ep1 = P.episode[b1];
    for (int k = 0; k < m; ++k) p0_s[r1 * 16 + k] = market_obs(P, b1, start1, ep1, 0, k);
  }
  auto mrel_fill = [&](int tday, int par) {
    double* dst = mrel_s + (par * kR + r1) * 16;
    for (int k = 0; k < m; ++k) dst[k] = market_obs(P, b1, start1, ep1, tday, k) / p0_s[r1 * 16 + k] - 1.0;
  };
  if (pre && t1 <= T) mrel_fill(t1, 0);
  __syncthreads();

  const int j = lane & 15, kl = lane >> 4;
  for (int day = 0; day < T; ++day) {
    // today's first price row is action-independent: its load is issued now and
    // lands under the policy forward (the step's own read then hits the cache)
    const bool probe = day == 10;
    if (probe) RLMD_TSE(0, __builtin_amdgcn_s_memtime());
    // ---- layer 1: wave w computes tiles w, w + 4, ... for the 16 rows (all of a
    //      wave's tiles issued together)
#pragma unroll
    for (int q = 0; q < (NT + 3) / 4; ++q) {
      const int tt = wave + 4 * q;
      if (NT % 4 == 0 || tt < NT) {  // no branch between the reads where 4 | NT
        f32x4 h = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < SP / 4; ++ks)
          h = __builtin_amdgcn_mfma_f32_16x16x4f32(w1s[((4 * ks + kl) * 16 + j) * NTP + tt],
                                                   obs_s[j * SP + 4 * ks + kl], h, 0, 0, 0);
        const f32x4 bias = *reinterpret_cast<const f32x4*>(&b1s[16 * tt + 4 * kl]);
        uint2 pk;
        pk.x = (uint32_t)f2bf_rne(fmaxf(h[0] + bias[0], 0.f)) | ((uint32_t)f2bf_rne(fmaxf(h[1] + bias[1], 0.f)) << 16);
        pk.y = (uint32_t)f2bf_rne(fmaxf(h[2] + bias[2], 0.f)) | ((uint32_t)f2bf_rne(fmaxf(h[3] + bias[3], 0.f)) << 16);
        *reinterpret_cast<uint2*>(&h1s[j * HP + 16 * tt + 4 * kl]) = pk;
      }
    }
    __syncthreads();
    if (probe) RLMD_TSE(1, __builtin_amdgcn_s_memtime());
    // ---- layer 2: 16 rows x 16 NB columns per wave, K = H1P in steps of 32
    f32x4 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int kq = 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < nS; ++s) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(&h1s[j * HP + 32 * s + kq]);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        bf16x8 bf;
        if constexpr (kRegW2) bf = wreg[nb][s];
        else bf = wf[(nb * nS + s) * 64];
        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[nb], 0, 0, 0);
      }
    }
    // ---- relu(h2 + b2) . heads, partial per row over this wave's columns
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      float ph[2 * kMaxA];
#pragma unroll
      for (int h = 0; h < 2 * kMaxA; ++h) ph[h] = 0.f;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const float v = fmaxf(acc[nb][rg] + b2v[nb], 0.f);
#pragma unroll
        for (int h = 0; h < 2 * kMaxA; ++h) ph[h] = fmaf(v, hw[nb][h], ph[h]);
      }
#pragma unroll
      for (int h = 0; h < 2 * kMaxA; ++h)
        if (h < nh) ph[h] = rlmd_row16_sum(ph[h]);
      if ((lane & 15) == 0) {
        const int r = 4 * (lane >> 4) + rg;
#pragma unroll
        for (int h = 0; h < 2 * kMaxA; ++h)
          if (h < nh) part[(wave * kR + r) * 2 * kMaxA + h] = ph[h];
      }
    }
    __syncthreads();
    if (probe) RLMD_TSE(2, __builtin_amdgcn_s_memtime());
    // ---- per lane: the deterministic action (eval_next_action), the market step
    // wave 1 (idle while wave 0 steps): tomorrow's relative prices, read by wave 0
    // after the end-of-day barrier (the lane's day index is t0 + day + 1 while it
    // is live; rows past the last step are never read)
    if (pre && t1 + day + 1 <= T) mrel_fill(t1 + day + 1, (day + 1) & 1);
    if (alive) {
      float acts[kMaxA] = {0.f, 0.f};
#pragma unroll
      for (int jj = 0; jj < kMaxA; ++jj) {
        if (jj >= A) break;
        float mu = mu_b[jj], ls_raw = 0.f;
        for (int q = 0; q < 4; ++q) mu += part[(q * kR + tid) * 2 * kMaxA + jj];
        if (a.algo == RLMD_SAC) {
          ls_raw = ls_b[jj];
          for (int q = 0; q < 4; ++q) ls_raw += part[(q * kR + tid) * 2 * kMaxA + A + jj];
          const rlmd::PolicyComp pc = rlmd::policy_comp(a.dist, mu, ls_raw, 0.f, a.ls_min, a.ls_max);
          acts[jj] = tanhf(pc.mu) * a.max_action;
        } else {
          acts[jj] = tanhf(mu) * a.max_action;
        }
      }
      auto act = [&](int i) -> AT {
        const double v = (double)(i == 0 ? acts[0] : acts[1]);
        if (sizeof(AT) == 4) return (AT)v;
        return (AT)fmin(fmax(v, clip_lo), clip_hi);
      };
      if (probe) RLMD_TSE(3, __builtin_amdgcn_s_memtime());
      const StepOut so = env_step_lane<RLMD_MARKET, NG, AT>(
          P, b, w, t, start, ep, act, [&](int) { return 0.0; },
          [&](int k, double v) { obs_s[tid * SP + k] = (float)v; },
          [&](int k, double v) { risk_s[tid * 8 + k] = v; }, NoDoneHook{}, MrelRow{mrel_s + ((day & 1) * kR + tid) * 16});
      last_r = so.reward;
      last_t = t;
      if (so.done) {
        alive = false;
      } else {
        w = so.W;
        ++t;
      }
      if (probe) RLMD_TSE(4, __builtin_amdgcn_s_memtime());
    }
    const int any_alive = __syncthreads_or(alive);
    if (probe) RLMD_TSE(5, __builtin_amdgcn_s_memtime());
    if (!any_alive) break;
  }
  if (mine) {
    P.wealth[b] = w;
    P.time[b] = t;
    reward_out[b] = last_r;
    steps_out[b] = last_t;
    live_io[b] = alive ? 1 : 0;
    for (int k = 0; k < S; ++k) obs_out[(int64_t)b * S + k] = obs_s[tid * SP + k];
    if (risk_out)
      for (int k = 0; k < P.risk_dim; ++k) risk_out[(int64_t)b * P.risk_dim + k] = risk_s[tid * 8 + k];
  }
}

template <int FAM>
__global__ void __launch_bounds__(256) env_obs_reset_kernel(EnvParams P, float* obs) {
  const int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= P.n_lanes) return;
  env_reset_lane<FAM>(P, lane, [&](int k, double v) { obs[(int64_t)lane * P.state_dim + k] = (float)v; });
}

// Host dispatch over the compile-time family (and n == 1) specialisations:
// ---------------------------------------------------------------------------
// per-episode log drain: exclusive scan of the waves' kept row counts (one
// workgroup), then one 64-lane workgroup per wave copies its rows into the
// packed output in wave order.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) ep_scan_kernel(const uint32_t* cnt, int n_waves, int cap, int64_t* offs,
                                                       int64_t* totals) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (n_waves + 1023) / 1024;
  int64_t kept = 0, seen = 0;
  for (int i = t * per; i < (t + 1) * per && i < n_waves; ++i) {
    const uint32_t c = cnt[i];
    kept += c < (uint32_t)cap ? c : (uint32_t)cap;
    seen += c;
  }
  part[t] = kept;
  __syncthreads();
  for (int h = 1; h < 1024; h <<= 1) {  // Hillis-Steele inclusive scan
    const int64_t v = t >= h ? part[t - h] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t o = part[t] - kept;
  for (int i = t * per; i < (t + 1) * per && i < n_waves; ++i) {
    offs[i] = o;
    const uint32_t c = cnt[i];
    o += c < (uint32_t)cap ? c : (uint32_t)cap;
  }
  // totals: [kept rows, rows appended]
  __shared__ unsigned long long seen_all;
  if (t == 0) seen_all = 0;
  __syncthreads();
  atomicAdd(&seen_all, (unsigned long long)seen);
  __syncthreads();
  if (t == 0) {
    totals[0] = part[1023];
    totals[1] = (int64_t)seen_all;
  }
}

__global__ void __launch_bounds__(64) ep_copy_kernel(const float* rows, const uint32_t* cnt, const int64_t* offs,
                                                     int cap, int w, float* out, int64_t out_cap) {
  const int wave = blockIdx.x;
  const uint32_t c = cnt[wave];
  const int64_t n = (int64_t)(c < (uint32_t)cap ? c : (uint32_t)cap) * w;
  const int64_t o = offs[wave] * w, lim = out_cap * w;
  const float* src = rows + (int64_t)wave * cap * w;
  for (int64_t i = threadIdx.x; i < n; i += 64)
    if (o + i < lim) out[o + i] = src[i];
}

// LAUNCH(FAM, NG) is expanded once per combination.
#define RLMD_ENV_DISPATCH(P, LAUNCH)                        \
  do {                                                      \
    const bool _one = (P).n == 1;                           \
    switch ((P).fam) {                                      \
      case RLMD_COIN:                                       \
        if (_one) { LAUNCH(RLMD_COIN, 1); } else { LAUNCH(RLMD_COIN, 0); } \
        break;                                              \
      case RLMD_DICE:                                       \
        if (_one) { LAUNCH(RLMD_DICE, 1); } else { LAUNCH(RLMD_DICE, 0); } \
        break;                                              \
      case RLMD_GBM:                                        \
        if (_one) { LAUNCH(RLMD_GBM, 1); } else { LAUNCH(RLMD_GBM, 0); } \
        break;                                              \
      case RLMD_DICE_SH:                                    \
        LAUNCH(RLMD_DICE_SH, 1);                            \
        break;                                              \
      default:                                              \
        if (_one) { LAUNCH(RLMD_MARKET, 1); } else { LAUNCH(RLMD_MARKET, 0); } \
        break;                                              \
    }                                                       \
  } while (0)

}  // namespace

// ============================================================================
// host side
// ============================================================================
struct rlmd_env_s {
  EnvParams P;
  uint32_t step_ctr = 0;
  double* d_prices = nullptr;
  // episode statistics of the fused train step (StatFold): two launches' worth
  // of per-block rows, the parity of the next launch, and the accumulator the
  // last launch's rows still owe (nullptr when nothing is pending)
  double* d_part = nullptr;
  int part_rows = 0, part_parity = 0;  // part_rows: per-parity capacity (64-lane blocks)
  int pend_rows = 0;                   // rows the pending launch wrote
  double* pending_dst = nullptr;
  // per-episode log (EnvParams::ep_rows / ep_cnt) and the drain's scratch
  int64_t* ep_offs = nullptr;
  int64_t* ep_tot = nullptr;
  // per-handle switches (one trainer per env handle; several may share a process):
  // the acting + env fusion (RLMD_NO_FUSED_ENV=1 at creation turns it off,
  // rlmd_train_set_fused after), and whether the last rlmd_train_step fused
  int fuse = 1;
  int last_fused = 0;
};

namespace rlmd {

int env_dims_for(const rlmd_env_cfg& c, int& S, int& A, int& R, int& D) {
  const int n = c.n_gambles;
  switch (c.family) {
    case RLMD_COIN:
    case RLMD_DICE:
    case RLMD_GBM:
    case RLMD_MARKET: {
      const int extra = c.investor == RLMD_INV_A ? 0 : (c.investor == RLMD_INV_B ? 1 : 2);
      S = 4 + (c.family == RLMD_MARKET ? c.obs_days * n : n);
      A = n + extra;
      R = (n == 1 ? 4 : 4 + n) + extra;
      D = c.family == RLMD_MARKET ? 0 : n;
      return 0;
    }
    case RLMD_DICE_SH:
      S = 6;
      A = c.investor == RLMD_INV_INSURED ? 1 : (c.investor == RLMD_INV_A ? 2 : (c.investor == RLMD_INV_B ? 3 : 4));
      R = 7;
      D = 1;
      return 0;
  }
  return 1;
}

void env_train_launch_params(rlmd_env_t env, EnvParams*& P);

int flush_stats(rlmd_env_t env, hipStream_t stream) {
  if (!env->pending_dst) return 0;
  const double* rows = env->d_part + (size_t)(env->part_parity ^ 1) * env->part_rows * 4;
  hipLaunchKernelGGL(stat_fold_kernel, dim3(1), dim3(256), 0, stream, rows, env->pend_rows, env->pending_dst);
  RLMD_LAUNCH_CHECK();
  env->pending_dst = nullptr;
  return 0;
}

int env_train(rlmd_env_t env, const rlmd::ReplayView& rb, int64_t ring_base, uint32_t step,
              float* actions, int random_actions, int abs_actions, int window, double clip_lo, double clip_hi,
              float* obs, double* ep_stats, hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop) {
  ring_base %= rb.capacity;
  const int N = env->P.n_lanes;
  const dim3 grid((N + 255) / 256), block(256);
  const bool f64 = window || random_actions;
  StatFold sf{nullptr, nullptr, nullptr, env->pend_rows};
  double* const last_rows = env->d_part + (size_t)(env->part_parity ^ 1) * env->part_rows * 4;
  if (env->pending_dst && env->pending_dst != ep_stats) {  // different accumulator: settle it now
    const int r = flush_stats(env, stream);
    if (r) return r;
  } else if (env->pending_dst) {
    sf.fold_src = last_rows;
    sf.fold_dst = env->pending_dst;
  }
  if (ep_stats) sf.part_out = env->d_part + (size_t)env->part_parity * env->part_rows * 4;
  // hipExtLaunchKernelGGL: the optional events are stamped at this dispatch's begin / end
#define TRAIN(F, NG)                                                                                          \
  {                                                                                                           \
    if (f64)                                                                                                  \
      hipExtLaunchKernelGGL((env_train_kernel<F, NG, double>), grid, block, 0, stream, ev_start, ev_stop, 0,  \
                            env->P, step, (const float*)actions, random_actions, abs_actions, clip_lo, clip_hi, \
                            obs, rb, ring_base, sf);                                                          \
    else                                                                                                      \
      hipExtLaunchKernelGGL((env_train_kernel<F, NG, float>), grid, block, 0, stream, ev_start, ev_stop, 0,   \
                            env->P, step, (const float*)actions, random_actions, abs_actions, clip_lo, clip_hi, \
                            obs, rb, ring_base, sf);                                                          \
  }
  RLMD_ENV_DISPATCH(env->P, TRAIN);
#undef TRAIN
  RLMD_LAUNCH_CHECK();
  env->pending_dst = ep_stats;
  if (ep_stats) {
    env->part_parity ^= 1;
    env->pend_rows = (int)grid.x;
  }
  return 0;
}

// the fused instantiations: one gamble / asset (market: one observed day), S <= 8,
// A <= 2; the env handle's switch (rlmd_train_set_fused; RLMD_NO_FUSED_ENV=1 at
// creation) turns the fusion off (separate acting and env launches)
bool env_act_fusable(rlmd_env_t env) {
  const EnvParams& P = env->P;
  // any n_gambles / assets / observation days whose action fits the acting body
  // (<= 2 actions) and whose state fits a 16-float staging row; the multi-asset
  // and Dx state widths above 8 take the 16-pitch market instantiation
  if (env->fuse != 1 || P.action_dim > actrows::kMaxA4 || P.state_dim > 16) return false;
  // 3-4 actions (investors C, Dice_SH B / C): the one-gamble / one-day shapes
  const bool ng1 = P.n == 1 && (P.fam != RLMD_MARKET || P.obs_days == 1);
  if (P.action_dim > actrows::kMaxA && !(ng1 && P.state_dim <= 8)) return false;
  return P.state_dim <= 8 || P.fam == RLMD_MARKET;
}

void env_set_last_fused(rlmd_env_t env, bool fused) { env->last_fused = fused ? 1 : 0; }

int env_act_train(rlmd_env_t env, const ReplayView& rb, int64_t ring_base, uint32_t step, const FusedActArgs& a,
                  int h1p, int nb, int sp, float* obs, double* ep_stats, hipStream_t stream, hipEvent_t ev_start,
                  hipEvent_t ev_stop, bool* launched) {
  *launched = false;
  ring_base %= rb.capacity;
  const EnvParams& P = env->P;
  const bool shape = (sp == 8 || sp == 16) && ((h1p == 256 && nb == 4) || (h1p == 416 && nb == 5));
  if (!env_act_fusable(env) || !shape || a.n != P.n_lanes) return 0;
  const int N = P.n_lanes;
  const dim3 grid((N + actrows::kRows - 1) / actrows::kRows), block(256);
  StatFold sf{nullptr, nullptr, nullptr, env->pend_rows};
  double* const last_rows = env->d_part + (size_t)(env->part_parity ^ 1) * env->part_rows * 4;
  if (env->pending_dst && env->pending_dst != ep_stats) {
    const int r = flush_stats(env, stream);
    if (r) return r;
  } else if (env->pending_dst) {
    sf.fold_src = last_rows;
    sf.fold_dst = env->pending_dst;
  }
  if (ep_stats) sf.part_out = env->d_part + (size_t)env->part_parity * env->part_rows * 4;
  // NG = 1: one gamble / asset, one observation day (the BASELINE configs); NG = 0:
  // n and the observation window read at run time (n_gambles / assets <= 2 with
  // A <= 2, market Dx at the 16-float staging pitch)
  const bool ng1 = P.n == 1 && (P.fam != RLMD_MARKET || P.obs_days == 1);
  RLMD_CHECK(ng1 || P.fam != RLMD_DICE_SH, "fused acting + env step: dice_sh has one die");
  RLMD_CHECK(sp == 8 || P.fam == RLMD_MARKET, "fused acting + env step: state wider than 8 (market only)");
  const bool wpc4 = actrows::act_wpc(h1p, P.action_dim > actrows::kMaxA ? actrows::kMaxA4 : actrows::kMaxA, grid.x) == 4;
#define FUSEDW(F, NG, H, B, SP, MA, W)                                                                                  \
  hipExtLaunchKernelGGL((act_env_kernel<F, NG, H, B, SP, MA, W>), grid, block,                                        \
                        actrows::act_lds_bytes(H, SP, MA, RLMD_ACT_PARK && actrows::act_park(H, SP, MA, W)) +               \
                            (RLMD_ACT_PARK && actrows::act_park(H, SP, MA, W) ? actrows::kParkBytes : 0), stream,            \
                        ev_start, ev_stop, 0, a, env->P, step, obs, rb, ring_base, sf)
#define FUSEDM(F, NG, H, B, SP, MA)                                                           \
  do {                                                                                        \
    if (wpc4) FUSEDW(F, NG, H, B, SP, MA, ((H) == 256 && (MA) == actrows::kMaxA) ? 4 : 3);    \
    else FUSEDW(F, NG, H, B, SP, MA, 3);                                                      \
  } while (0)
#define FUSED(F, NG, H, B, SP) FUSEDM(F, NG, H, B, SP, actrows::kMaxA)
  // 3-4 actions: one gamble / asset and one observation day (env_act_fusable)
  const bool ma4 = P.action_dim > actrows::kMaxA;
#define FUSED4(F)                                                \
  {                                                              \
    if (h1p == 256) FUSEDM(F, 1, 256, 4, 8, actrows::kMaxA4);    \
    else FUSEDM(F, 1, 416, 5, 8, actrows::kMaxA4);               \
  }
#define FUSED_FAM(F)                                 \
  {                                                  \
    if (ma4) FUSED4(F)                               \
    else if (ng1) {                                  \
      if (h1p == 256) FUSED(F, 1, 256, 4, 8);        \
      else FUSED(F, 1, 416, 5, 8);                   \
    } else {                                         \
      if (h1p == 256) FUSED(F, 0, 256, 4, 8);        \
      else FUSED(F, 0, 416, 5, 8);                   \
    }                                                \
  }
  RLMD_CHECK(!ma4 || (ng1 && sp == 8), "fused acting + env step: 3-4 actions need one gamble / asset and day");
  switch (P.fam) {
    case RLMD_COIN: FUSED_FAM(RLMD_COIN); break;
    case RLMD_DICE: FUSED_FAM(RLMD_DICE); break;
    case RLMD_GBM: FUSED_FAM(RLMD_GBM); break;
    case RLMD_DICE_SH:
      if (ma4) FUSED4(RLMD_DICE_SH)
      else if (h1p == 256) FUSED(RLMD_DICE_SH, 1, 256, 4, 8);
      else FUSED(RLMD_DICE_SH, 1, 416, 5, 8);
      break;
    default:
      if (sp == 16) {
        if (h1p == 256) FUSED(RLMD_MARKET, 0, 256, 4, 16);
        else FUSED(RLMD_MARKET, 0, 416, 5, 16);
      } else {
        FUSED_FAM(RLMD_MARKET);
      }
      break;
  }
#undef FUSED_FAM
#undef FUSED4
#undef FUSED
#undef FUSEDM
#undef FUSEDW
  RLMD_LAUNCH_CHECK();
  env->pending_dst = ep_stats;
  if (ep_stats) {
    env->part_parity ^= 1;
    env->pend_rows = (int)grid.x;
  }
  *launched = true;
  return 0;
}

int env_market_eval_reset(rlmd_env_t env, const int32_t* start_at, float* obs, double* reward, int32_t* steps,
                          uint8_t* live, hipStream_t stream) {
  RLMD_CHECK(env->P.fam == RLMD_MARKET, "market evaluation needs a market env");
  const int N = env->P.n_lanes;
  hipLaunchKernelGGL(eval_market_reset_kernel, dim3((N + 255) / 256), dim3(256), 0, stream, env->P, start_at, obs,
                     reward, steps, live);
  RLMD_LAUNCH_CHECK();
  return 0;
}

int env_market_eval_step(rlmd_env_t env, const float* actions, int window, double lo, double hi, float* obs,
                         double* reward, int32_t* steps, double* risk, uint8_t* live, hipStream_t stream) {
  const int N = env->P.n_lanes;
  const dim3 grid((N + 255) / 256), block(256);
#define MSTEP(NG, AT)                                                                                        \
  hipLaunchKernelGGL((eval_market_step_kernel<NG, AT>), grid, block, 0, stream, env->P, actions, lo, hi, obs, \
                     reward, steps, risk, live)
  if (env->P.n == 1) {
    if (window) MSTEP(1, double);
    else MSTEP(1, float);
  } else {
    if (window) MSTEP(0, double);
    else MSTEP(0, float);
  }
#undef MSTEP
  RLMD_LAUNCH_CHECK();
  return 0;
}

// the whole market evaluation in one launch (eval_market_loop_kernel) for the
// acting shapes with an instantiation; *launched = false leaves it to the
// caller's per-day loop.  Off with the env handle's acting + env fusion
// (RLMD_NO_FUSED_ENV=1, rlmd_train_set_fused(env, 0)).
int env_act_market_eval(rlmd_env_t env, const FusedActArgs& a, int h1p, int nb, int T, int window, double lo,
                        double hi, float* obs, double* reward, int32_t* steps, double* risk, uint8_t* live,
                        hipStream_t stream, bool* launched) {
  *launched = false;
  const bool off = env->fuse == 0;
  const EnvParams& P = env->P;
  const int sp = a.S <= 8 ? 8 : 16;
  if (off || P.fam != RLMD_MARKET || a.n != P.n_lanes || a.S > 16 || a.A > actrows::kMaxA || P.risk_dim > 8 ||
      P.obs_days * P.n > 16 ||
      !((h1p == 256 && nb == 4) || (h1p == 416 && nb == 5)))
    return 0;
  const dim3 grid((P.n_lanes + 15) / 16), block(256);
#define MLOOP(NG, AT, H, B, SPV)                                                                                   \
  hipLaunchKernelGGL((eval_market_loop_kernel<NG, AT, H, B, SPV>), grid, block, 0, stream, a, env->P, T, lo, hi, \
                     reward, steps, risk, live, obs)
#define MLOOP_SHAPE(NG, AT)                   \
  {                                           \
    if (h1p == 256 && sp == 8) MLOOP(NG, AT, 256, 4, 8);       \
    else if (h1p == 256) MLOOP(NG, AT, 256, 4, 16);            \
    else if (sp == 8) MLOOP(NG, AT, 416, 5, 8);                \
    else MLOOP(NG, AT, 416, 5, 16);                            \
  }
  if (P.n == 1) {
    if (window) MLOOP_SHAPE(1, double)
    else MLOOP_SHAPE(1, float)
  } else {
    if (window) MLOOP_SHAPE(0, double)
    else MLOOP_SHAPE(0, float)
  }
#undef MLOOP_SHAPE
#undef MLOOP
  RLMD_LAUNCH_CHECK();
  *launched = true;
  return 0;
}

int env_episode_steps(rlmd_env_t env) {
  const EnvParams& P = env->P;
  return P.obs_days == 1 ? P.time_length : P.time_length - P.obs_days + 1;
}

int env_lanes(rlmd_env_t env) { return env->P.n_lanes; }
int env_state_dim(rlmd_env_t env) { return env->P.state_dim; }
int env_action_dim(rlmd_env_t env) { return env->P.action_dim; }

}  // namespace rlmd

extern "C" {

int rlmd_env_create(const rlmd_env_cfg* cfg, const double* prices_host, int64_t n_days,
                    rlmd_env_t* out) {
  RLMD_CHECK(cfg && out, "null argument");
  RLMD_CHECK(cfg->family >= RLMD_COIN && cfg->family <= RLMD_MARKET, "bad family");
  RLMD_CHECK(cfg->n_lanes > 0, "n_lanes must be > 0");
  RLMD_CHECK(cfg->n_gambles >= 1 && cfg->n_gambles <= RLMD_MAX_GAMBLES, "n_gambles out of range");
  if (cfg->family == RLMD_DICE_SH)
    RLMD_CHECK(cfg->investor >= RLMD_INV_A && cfg->investor <= RLMD_INV_INSURED, "bad investor");
  else
    RLMD_CHECK(cfg->investor >= RLMD_INV_A && cfg->investor <= RLMD_INV_C, "bad investor");
  int S, A, R, D;
  rlmd::env_dims_for(*cfg, S, A, R, D);
  RLMD_CHECK(A <= RLMD_MAX_ACTION, "action dim too large");
  auto* e = new rlmd_env_s();
  e->fuse = getenv("RLMD_NO_FUSED_ENV") != nullptr ? 0 : 1;
  EnvParams& P = e->P;
  memset(&P, 0, sizeof(P));
  P.fam = cfg->family;
  P.inv = cfg->investor;
  P.n_lanes = cfg->n_lanes;
  P.n = cfg->n_gambles;
  P.obs_days = cfg->obs_days > 0 ? cfg->obs_days : 1;
  P.time_length = cfg->time_length;
  P.action_days = cfg->action_days > 0 ? cfg->action_days : 1;
  P.shuffle_days = cfg->shuffle_days > 0 ? cfg->shuffle_days : 1;
  P.state_dim = S;
  P.action_dim = A;
  P.risk_dim = R;
  P.draw_dim = D;
  P.seed = cfg->seed;
  P.slice_groups = cfg->slice_groups > 0 ? cfg->slice_groups : 0;
  P.alias_state = cfg->family != RLMD_DICE_SH;
  const size_t N = (size_t)cfg->n_lanes;
  if (cfg->family == RLMD_MARKET) {
    if (!prices_host || n_days <= 1 || cfg->time_length <= 0 || P.shuffle_days > 16) {
      delete e;
      RLMD_CHECK(false, "market env needs prices, time_length > 0 and shuffle_days <= 16");
    }
    P.ext_len = P.time_length * P.action_days + 1;
    P.n_days = (int)n_days;
    P.start_range = (int)(n_days - cfg->sample_days);
    if (P.start_range < 1 || P.start_range - 1 + P.ext_len > n_days) {
      delete e;
      RLMD_CHECK(false, "market sample_days inconsistent with n_days / time_length");
    }
    RLMD_HIP(hipMalloc(&e->d_prices, sizeof(double) * n_days * P.n));
    RLMD_HIP(hipMemcpy(e->d_prices, prices_host, sizeof(double) * n_days * P.n,
                       hipMemcpyHostToDevice));
    P.prices = e->d_prices;
  }
  RLMD_HIP(hipMalloc(&P.wealth, sizeof(double) * N));
  RLMD_HIP(hipMalloc(&P.time, sizeof(int32_t) * N));
  RLMD_HIP(hipMalloc(&P.start, sizeof(int32_t) * N));
  RLMD_HIP(hipMalloc(&P.episode, sizeof(uint32_t) * N));
  e->part_rows = (int)((N + 63) / 64);  // the fused kernel's 64-lane blocks; 256-lane launches use fewer
  RLMD_HIP(hipMalloc(&e->d_part, sizeof(double) * 8 * e->part_rows));
  RLMD_HIP(hipMemset(P.episode, 0xff, sizeof(uint32_t) * N));  // first reset -> episode 0
  RLMD_HIP(hipMemset(P.start, 0, sizeof(int32_t) * N));
#define RESET(F, NG) hipLaunchKernelGGL(env_reset_kernel<F>, dim3((N + 255) / 256), dim3(256), 0, 0, P, nullptr, nullptr)
  RLMD_ENV_DISPATCH(P, RESET);
#undef RESET
  RLMD_LAUNCH_CHECK();
  RLMD_HIP(hipDeviceSynchronize());
  *out = e;
  return 0;
}

int rlmd_env_destroy(rlmd_env_t env) {
  if (!env) return 0;
  (void)hipFree(env->P.wealth);
  (void)hipFree(env->P.time);
  (void)hipFree(env->P.start);
  (void)hipFree(env->P.episode);
  if (env->d_prices) (void)hipFree(env->d_prices);
  (void)hipFree(env->d_part);
  if (env->P.ep_rows) (void)hipFree(env->P.ep_rows);
  if (env->P.ep_cnt) (void)hipFree(env->P.ep_cnt);
  if (env->ep_offs) (void)hipFree(env->ep_offs);
  if (env->ep_tot) (void)hipFree(env->ep_tot);
  delete env;
  return 0;
}

int rlmd_env_dims(rlmd_env_t env, int32_t* S, int32_t* A, int32_t* R, int32_t* D) {
  RLMD_CHECK(env, "null env");
  if (S) *S = env->P.state_dim;
  if (A) *A = env->P.action_dim;
  if (R) *R = env->P.risk_dim;
  if (D) *D = env->P.draw_dim;
  return 0;
}

int rlmd_env_reset(rlmd_env_t env, const uint8_t* mask, double* state, void* stream) {
  RLMD_CHECK(env, "null env");
  const int N = env->P.n_lanes;
#define RESET(F, NG) \
  hipLaunchKernelGGL(env_reset_kernel<F>, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, env->P, mask, state)
  RLMD_ENV_DISPATCH(env->P, RESET);
#undef RESET
  RLMD_LAUNCH_CHECK();
  return 0;
}

int rlmd_env_step(rlmd_env_t env, const float* actions, const double* draws, double* next_state,
                  double* reward, uint8_t* done, double* risk, void* stream) {
  RLMD_CHECK(env && actions && next_state && reward && done, "null argument");
  const int N = env->P.n_lanes;
#define STEP(F, NG)                                                                                         \
  hipLaunchKernelGGL((env_step_kernel<F, NG, float>), dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, \
                     env->P, env->step_ctr, actions, draws, next_state, reward, done, risk)
  RLMD_ENV_DISPATCH(env->P, STEP);
#undef STEP
  RLMD_LAUNCH_CHECK();
  env->step_ctr++;
  return 0;
}

int rlmd_env_step_f64(rlmd_env_t env, const double* actions, const double* draws, double* next_state,
                      double* reward, uint8_t* done, double* risk, void* stream) {
  RLMD_CHECK(env && actions && next_state && reward && done, "null argument");
  const int N = env->P.n_lanes;
#define STEP(F, NG)                                                                                          \
  hipLaunchKernelGGL((env_step_kernel<F, NG, double>), dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, \
                     env->P, env->step_ctr, actions, draws, next_state, reward, done, risk)
  RLMD_ENV_DISPATCH(env->P, STEP);
#undef STEP
  RLMD_LAUNCH_CHECK();
  env->step_ctr++;
  return 0;
}

int rlmd_eval_rollout(rlmd_env_t env, const float* actions, int32_t max_steps, int64_t cum_step,
                      int32_t warmup_steps, int32_t smoothing_window, const double* draws, double* reward,
                      int32_t* steps, double* risk, void* stream) {
  RLMD_CHECK(env && actions && reward && steps, "null argument");
  RLMD_CHECK(max_steps >= 1, "max_steps must be >= 1");
  const int N = env->P.n_lanes;
  // eval_episodes.py:240-248: action_window when cum_steps <= smoothing_window,
  // which clips only past the warm-up (utils.py:366-371)
  const bool window = cum_step <= smoothing_window && cum_step > warmup_steps;
  double lo = -INFINITY, hi = INFINITY;
  if (window) {
    const double width = (sin(M_PI * ((double)cum_step / (double)smoothing_window - 0.5)) + 1.0) / 2.0;
    lo = width * -0.99;
    hi = width * 0.99;
  }
  const dim3 grid((N + 255) / 256), block(256);
#define EVAL(F, NG)                                                                                           \
  {                                                                                                           \
    if (window)                                                                                               \
      hipLaunchKernelGGL((eval_rollout_kernel<F, NG, double>), grid, block, 0, (hipStream_t)stream, env->P,  \
                         env->step_ctr, actions, max_steps, lo, hi, draws, reward, steps, risk);               \
    else                                                                                                      \
      hipLaunchKernelGGL((eval_rollout_kernel<F, NG, float>), grid, block, 0, (hipStream_t)stream, env->P,   \
                         env->step_ctr, actions, max_steps, lo, hi, draws, reward, steps, risk);               \
  }
  RLMD_ENV_DISPATCH(env->P, EVAL);
#undef EVAL
  RLMD_LAUNCH_CHECK();
  env->step_ctr += (uint32_t)max_steps;
  return 0;
}

int rlmd_env_lane_state(rlmd_env_t env, double* wealth, int32_t* time) {
  RLMD_CHECK(env, "null env");
  RLMD_HIP(hipDeviceSynchronize());
  const size_t N = env->P.n_lanes;
  if (wealth) RLMD_HIP(hipMemcpy(wealth, env->P.wealth, N * sizeof(double), hipMemcpyDeviceToHost));
  if (time) RLMD_HIP(hipMemcpy(time, env->P.time, N * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

int rlmd_env_lane_start(rlmd_env_t env, int32_t* start_host) {
  RLMD_CHECK(env && start_host, "null argument");
  RLMD_HIP(hipDeviceSynchronize());
  RLMD_HIP(hipMemcpy(start_host, env->P.start, env->P.n_lanes * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

int rlmd_env_write_prices(rlmd_env_t env, const double* rows_host, int64_t row0, int64_t n_rows, void* stream) {
  RLMD_CHECK(env && (rows_host || n_rows == 0), "null argument");
  const EnvParams& P = env->P;
  RLMD_CHECK(P.fam == RLMD_MARKET && env->d_prices, "price rows: market envs only");
  RLMD_CHECK(row0 >= 0 && n_rows >= 0 && row0 + n_rows <= P.n_days, "price rows outside the table");
  if (n_rows == 0) return 0;
  RLMD_HIP(hipMemcpyAsync(env->d_prices + row0 * P.n, rows_host, sizeof(double) * n_rows * P.n,
                          hipMemcpyHostToDevice, (hipStream_t)stream));
  return 0;
}

int rlmd_train_flush_stats(rlmd_env_t env, void* stream) {
  RLMD_CHECK(env, "null env");
  return rlmd::flush_stats(env, (hipStream_t)stream);
}

#ifdef RLMD_TIMING
int rlmd_debug_ts_env(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ts_env), sizeof(unsigned long long) * 8 * n) != hipSuccess;
}
int rlmd_debug_ts_actenv(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ts_actenv), sizeof(unsigned long long) * 8 * n) != hipSuccess;
}
#endif

int rlmd_train_set_fused(rlmd_env_t env, int32_t on) {
  RLMD_CHECK(env, "null env");
  env->fuse = on ? 1 : 0;
  return 0;
}

int rlmd_train_last_fused(rlmd_env_t env) { return env ? env->last_fused : 0; }

int rlmd_train_set_stored_state(rlmd_env_t env, int32_t mode) {
  RLMD_CHECK(env, "null env");
  RLMD_CHECK(mode == RLMD_STORE_REFERENCE || mode == RLMD_STORE_PRESTEP, "bad stored-state mode");
  env->P.alias_state = mode == RLMD_STORE_REFERENCE && env->P.fam != RLMD_DICE_SH;
  return 0;
}

int rlmd_train_stored_state(rlmd_env_t env) {
  return env && !env->P.alias_state && env->P.fam != RLMD_DICE_SH ? RLMD_STORE_PRESTEP : RLMD_STORE_REFERENCE;
}

int rlmd_train_episode_log(rlmd_env_t env, int32_t cap_per_wave) {
  RLMD_CHECK(env, "null env");
  RLMD_CHECK(cap_per_wave >= 0, "cap_per_wave must be >= 0");
  EnvParams& P = env->P;
  RLMD_HIP(hipDeviceSynchronize());
  if (P.ep_rows) (void)hipFree(P.ep_rows);
  if (P.ep_cnt) (void)hipFree(P.ep_cnt);
  if (env->ep_offs) (void)hipFree(env->ep_offs);
  if (env->ep_tot) (void)hipFree(env->ep_tot);
  P.ep_rows = nullptr;
  P.ep_cnt = nullptr;
  env->ep_offs = env->ep_tot = nullptr;
  P.ep_cap = cap_per_wave;
  P.ep_w = 4 + P.risk_dim;
  if (cap_per_wave == 0) return 0;
  const int64_t waves = ((int64_t)P.n_lanes + 63) / 64;
  RLMD_HIP(hipMalloc(&P.ep_rows, sizeof(float) * waves * cap_per_wave * P.ep_w));
  RLMD_HIP(hipMalloc(&P.ep_cnt, sizeof(uint32_t) * waves));
  RLMD_HIP(hipMalloc(&env->ep_offs, sizeof(int64_t) * waves));
  RLMD_HIP(hipMalloc(&env->ep_tot, sizeof(int64_t) * 2));
  RLMD_HIP(hipMemset(P.ep_cnt, 0, sizeof(uint32_t) * waves));
  RLMD_HIP(hipDeviceSynchronize());
  return 0;
}

int rlmd_train_episode_drain(rlmd_env_t env, float* out_dev, int64_t out_cap, int64_t* n_out_host,
                             int64_t* appended_host, void* stream) {
  RLMD_CHECK(env && n_out_host, "null argument");
  EnvParams& P = env->P;
  RLMD_CHECK(P.ep_rows, "episode log not enabled (rlmd_train_episode_log)");
  RLMD_CHECK(out_dev || out_cap == 0, "null output");
  const int waves = (P.n_lanes + 63) / 64;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ep_scan_kernel, dim3(1), dim3(1024), 0, st, P.ep_cnt, waves, P.ep_cap, env->ep_offs,
                     env->ep_tot);
  RLMD_LAUNCH_CHECK();
  if (out_cap > 0) {
    hipLaunchKernelGGL(ep_copy_kernel, dim3(waves), dim3(64), 0, st, P.ep_rows, P.ep_cnt, env->ep_offs, P.ep_cap,
                       P.ep_w, out_dev, out_cap);
    RLMD_LAUNCH_CHECK();
  }
  RLMD_HIP(hipMemsetAsync(P.ep_cnt, 0, sizeof(uint32_t) * waves, st));
  int64_t tot[2];
  RLMD_HIP(hipMemcpyAsync(tot, env->ep_tot, sizeof(tot), hipMemcpyDeviceToHost, st));
  RLMD_HIP(hipStreamSynchronize(st));
  *n_out_host = tot[0] < out_cap ? tot[0] : out_cap;
  if (appended_host) *appended_host = tot[1];
  return 0;
}

int rlmd_train_reset(rlmd_env_t env, float* obs, void* stream) {
  RLMD_CHECK(env && obs, "null argument");
  const int N = env->P.n_lanes;
#define ORESET(F, NG) \
  hipLaunchKernelGGL(env_obs_reset_kernel<F>, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, env->P, obs)
  RLMD_ENV_DISPATCH(env->P, ORESET);
#undef ORESET
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
