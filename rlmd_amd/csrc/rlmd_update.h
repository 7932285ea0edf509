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
  int32_t* rank_out;      // nullable: every row's top-k selection rank [B] (workgroup 0 writes it)
  // updates without an actor step (TD3's delayed actor): this update's critic
  // statistics as two extra workgroups of the same launch (B == 0: none)
  LossArgs cstats;
};

// The actor (+ temperature) step of one update in one launch
// (update.hip actor_update_kernel).  Grid: n_w2 fc2.weight tiles + n_w1 fc1
// blocks of the policy, head workgroups (b2 and the heads of 32 fc2 rows each),
// then two critic-statistics workgroups when cstats.B > 0.
struct ActUpdArgs {
  RowDims d;
  NetOff ao;
  SampleCfg smp;
  int32_t nq;              // critics in the actor loss: SAC 2 (min), TD3 1
  const float* qn[2];      // updated critics on (s, a_new), no head bias [B]
  const float* qb[2];      // their q_value.bias (not stepped in this launch)
  const float* dqda[2];    // dq/da per row [B][A] (qeval_rows)
  const float* logp;       // [B] (SAC)
  const float* save;       // sampling save [B][5A] (fwd_rows job 4)
  const uint8_t* am2;      // the policy's [h2 > 0], row-packed bytes
  const void* hp1a;        // the policy's h1 / h2 row-packed, compute type
  const void* hp2a;
  const float* ua;         // backward bases per head [nh][nrb * H1p * 16], f32
  const float* wheads;     // head weights' snapshot [nh][H2]
  const float* s;          // states [B][S]
  LearnState* st;
  float* stats;
  int32_t k, topk;
  float target_entropy;
  AdamArgs adam;           // the actor (+ temperature when adam.temp)
  LossArgs cstats;         // critic statistics workgroup (B == 0: none)
  int32_t ti, tj, n_w2, n_w1;
  // qeval_rows' column split (1 or 2): q and dq/da arrive as P partial sums, at
  // offsets p * B (q) and p * B * A (dq/da)
  int32_t qsplit;
};

size_t critic_update_lds();
int actor_update_n_w1(const RowDims& d);  // fc1 blocks of the actor step (TW1 units each)
int critic_update_tj(const RowDims& d);  // fc2.weight tile columns of the critic step (32 x 64 tiles at B <= 256)
int actor_update_launch(const ActUpdArgs& a, hipStream_t st);
int critic_update_launch(const CritUpdArgs& a, hipStream_t st);

}  // namespace rlmd
