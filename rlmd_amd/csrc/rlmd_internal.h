// rlmd_internal.h — internal (non-ABI) declarations shared by the .hip units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlmd_abi.h"

#define RLMD_MAX_ACTION 48   // max action components per lane (market InvC with 40 assets + 2)
#define RLMD_MAX_GAMBLES 46  // n_gambles / n_assets
#define RLMD_MAX_BATCH 1024  // learner mini-batch upper bound (one workgroup sorts it)

namespace rlmd {

// Device view of the replay ring (SoA, f32; done as u8).  Multi-step mode
// (n_steps > 1, tools/replay.py:93-332) adds per-row tags and per-lane episode
// bookkeeping; transition p of lane l sits at row (p * lanes + l) % capacity.
struct ReplayView {
  float* state;       // [capacity, S]
  float* action;      // [capacity, A]
  float* reward;      // [capacity]
  float* next_state;  // [capacity, S]
  uint8_t* done;      // [capacity]
  int64_t capacity;
  int32_t S, A;
  int32_t n_steps;    // <= 1: single-step
  int32_t lanes;      // independent transition streams
  int32_t additive;   // 1: dynamics "A" (sum), 0: product
  double gamma;
  int32_t* tag;       // [capacity, 3]: lane-local position, episode ordinal, episode start
  int32_t* lane;      // [lanes, 4]: next position, finished episodes, in-progress start, end of episode 0
};

// Record the multi-step tags of a transition just written to `row` by lane `l`
// (one writer per lane per launch) and advance that lane's episode bookkeeping.
__device__ inline void ms_record(const ReplayView& rb, int l, int64_t row, bool done) {
  int4* lsp = reinterpret_cast<int4*>(rb.lane + 4 * (int64_t)l);  // one 16-B load, one 16-B store
  int4 ls = *lsp;
  const int32_t p = ls.x;
  int32_t* t = rb.tag + 3 * row;
  t[0] = p;
  t[1] = ls.y;
  t[2] = ls.z;
  if (done) {
    if (ls.y == 0) ls.w = p;
    ls.y += 1;
    ls.z = p + 1;
  }
  ls.x = p + 1;
  *lsp = ls;
}

ReplayView replay_view(rlmd_replay_t rb);
int64_t replay_mem_idx(rlmd_replay_t rb);
void replay_advance(rlmd_replay_t rb, int64_t n);

// window != 0: the smoothing-window clip [clip_lo, clip_hi] applies.  Warm-up
// (random_actions) and window steps hand the env float64 actions, as the
// reference's float64 action space and np.clip with np.float64 bounds do.
int env_train(rlmd_env_t env, const ReplayView& rb, int64_t ring_base, uint32_t step,
              float* actions, int random_actions, int abs_actions, int window, double clip_lo, double clip_hi,
              float* obs, double* ep_stats, hipStream_t stream, hipEvent_t ev_start = nullptr,
              hipEvent_t ev_stop = nullptr);
// market evaluation (eval_episodes.py:402-611): reset every lane at its given
// start row, then one policy-driven step of the still-running lanes
int env_market_eval_reset(rlmd_env_t env, const int32_t* start_at, float* obs, double* reward, int32_t* steps,
                          uint8_t* live, hipStream_t stream);
int env_market_eval_step(rlmd_env_t env, const float* actions, int window, double lo, double hi, float* obs,
                         double* reward, int32_t* steps, double* risk, uint8_t* live, hipStream_t stream);
int env_episode_steps(rlmd_env_t env);  // market: steps until done_time
int env_lanes(rlmd_env_t env);
void env_set_last_fused(rlmd_env_t env, bool fused);  // rlmd_train_last_fused of this handle
int env_state_dim(rlmd_env_t env);
int env_action_dim(rlmd_env_t env);

// mini-batch sampler: K independent mini-batches in one launch (one workgroup
// each), batch k = B distinct indices in [0, M) drawn with counter ctr + k, then
// gathered to offset k of every output; optionally writes the critic input
// [s | a] as xsa [K, B, S+A].  Multi-step mode: s / a are the history's initial
// next-state / action, r the n-step return, eff [K, B] the effective length
// (nullable); see oracle/replay.py.
int replay_sample_launch(const ReplayView& rb, int64_t M, int B, int K, uint64_t seed, uint64_t ctr,
                         int64_t* idx, float* s, float* a, float* r, float* s2, uint8_t* done, float* xsa,
                         int32_t* eff, hipStream_t stream);

}  // namespace rlmd
