// rlmd_internal.h — internal (non-ABI) declarations shared by the .hip units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlmd_abi.h"

#define RLMD_MAX_ACTION 48   // max action components per lane (market InvC with 40 assets + 2)
#define RLMD_MAX_GAMBLES 46  // n_gambles / n_assets
#define RLMD_MAX_BATCH 1024  // learner mini-batch upper bound (one workgroup sorts it)

namespace rlmd {

// Device view of the replay ring (SoA, f32; done as u8).
struct ReplayView {
  float* state;       // [capacity, S]
  float* action;      // [capacity, A]
  float* reward;      // [capacity]
  float* next_state;  // [capacity, S]
  uint8_t* done;      // [capacity]
  int64_t capacity;
  int32_t S, A;
};

ReplayView replay_view(rlmd_replay_t rb);
int64_t replay_mem_idx(rlmd_replay_t rb);
void replay_advance(rlmd_replay_t rb, int64_t n);

int env_train(rlmd_env_t env, const ReplayView& rb, int64_t ring_base, uint32_t step,
              float* actions, int random_actions, int abs_actions, float clip_lo, float clip_hi,
              float* obs, double* ep_stats, hipStream_t stream);
int env_lanes(rlmd_env_t env);
int env_state_dim(rlmd_env_t env);
int env_action_dim(rlmd_env_t env);

// mini-batch sampler: B distinct indices in [0, M) + gather; optionally writes
// the critic input [s | a] as xsa [B, S+A].
// dev_ctr (nullable): device counter used as the draw counter instead of ctr and
// incremented by the kernel (the learner's learn_step_cntr).
int replay_sample_launch(const ReplayView& rb, int64_t M, int B, uint64_t seed, uint64_t ctr,
                         int32_t* dev_ctr, int64_t* idx, float* s, float* a, float* r, float* s2,
                         uint8_t* done, float* xsa, hipStream_t stream);

}  // namespace rlmd
