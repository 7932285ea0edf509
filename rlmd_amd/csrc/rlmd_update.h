// rlmd_update.h — arguments of the fused update kernels (update.hip).
#pragma once
#include "learn_kernels.h"
#include "rlmd_adam.h"

namespace rlmd {

// The critic step of one update in one launch (update.hip critic_update_kernel).
// Grid: per critic n_w2 fc2.weight tiles (ti x tj of 32 x 32) + n_w1 blocks of
// 32 fc1 rows.  Row-packed operands (rows.hip rp_index) from fwd_rows.
struct CritUpdArgs {
  RowDims d;
  NetOff co;
  LossArgs loss;          // the critic loss inputs; qb / tb point at the forward's bias snapshot
  const uint8_t* m2[2];   // [h2 > 0] bytes (rows.hip m2_index == rp_index layout)
  const void* hp1[2];     // h1 row-packed, compute type
  const void* hp2[2];     // h2 row-packed, compute type
  const float* u1[2];     // backward basis row-packed, f32
  const float* w3s[2];    // q_value.weight snapshot [H2]
  const float* x;         // critic inputs [B, X]
  AdamArgs adam;          // both critics (p = critic 0's parameters, n = 2 x net size)
  int32_t ti, tj, n_w2, n_w1;
};

size_t critic_update_lds();
int critic_update_launch(const CritUpdArgs& a, hipStream_t st);

}  // namespace rlmd
