// rlmd_loss.h — the critic loss as workgroup device functions, shared by the
// one-workgroup critic_loss_kernel (learn.hip) and the row kernels (rows.hip):
//   critic_row_loss   bootstrapped target, the loss and its derivative per row,
//                     with the block-wide means / variances the CIM kernel,
//                     the TCAU truncation and the Nagy scale need;
//   critic_sel_key    the top-k ordering key (descending l1 + l2, ties by row);
//   critic_loss_block the whole loss for one workgroup: top-k selection, dq,
//                     statistics, tail index, device-state updates.
// Restates tools/critic_loss.py:26-453 and algo_sac.py:347-473 /
// algo_td3.py:346-470.  Thread b owns mini-batch row b (blockDim.x >= B).
#pragma once
#include <math.h>

#include "learn_kernels.h"
#include "rlmd_block.h"

namespace rlmd {
namespace {

__device__ __forceinline__ void loss_and_grad(int lt, float q, float t, float c, float kern,
                                              float& l, float& dl) {
  const float d = t - q;
  switch (lt) {
    case RLMD_LOSS_MSE: l = d * d; dl = -2.f * d; break;
    case RLMD_LOSS_MSE2: l = d * d * d * d; dl = -4.f * d * d * d; break;
    case RLMD_LOSS_MSE4: { const float d2 = d * d; l = d2 * d2 * d2; dl = -6.f * d2 * d2 * d; break; }
    case RLMD_LOSS_MSE6: { const float d2 = d * d; l = d2 * d2 * d2 * d2; dl = -8.f * d2 * d2 * d2 * d; break; }
    case RLMD_LOSS_MAE: l = fabsf(d); dl = d > 0.f ? -1.f : (d < 0.f ? 1.f : 0.f); break;
    case RLMD_LOSS_HUB: {
      const float ad = fabsf(d);
      const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
      if (ad < 1.f) { l = 0.5f * ad * ad; dl = -ad * sg; }
      else { l = ad - 0.5f; dl = -sg; }
      break;
    }
    case RLMD_LOSS_HSC: { const float s = sqrtf(1.f + d * d); l = s - 1.f; dl = -d / s; break; }
    case RLMD_LOSS_CAU:
    case RLMD_LOSS_TCAU: {
      const float z = d / c;
      l = logf(1.f + z * z);
      dl = -(2.f * z / c) / (1.f + z * z);
      break;
    }
    default: {  // CIM
      const float e = expf(-(d * d) / (2.f * kern * kern)) / sqrtf(2.f * 3.14159265358979323846f * kern);
      l = 1.f - e;
      dl = -e * d / (kern * kern);
      break;
    }
  }
}

struct CriticRow {
  bool in;
  float y;
  float l[2], dl[2];
  float scale[2], kern[2];
  float s1[7];  // block sums: (t-q)^2 per critic, y, q per critic, Nagy terms
  float nan;    // block max of the NaN flag
};

// Per-row target and loss.  Every row's loads are issued unconditionally
// (range-checked buffer loads), so the prologue is one memory round trip.
// The row's inputs, issued as one load round (callers issue it ahead of their
// weight-fragment stream, so the loss never waits behind it: vmcnt is in order).
struct CriticLoads {
  float qt[2], q[2], rw, lpn;
  int eff;
  bool has_eff;
  uint8_t dn;
  // uniform scalars issued with the row loads: head biases, log alpha, Cauchy scales
  float tb[2], qb[2], log_alpha, cauchy[2];
};
// MAYSPLIT false: the caller knows a.qsplit == 1 and the second halves' loads are
// not issued at all (predicated off they still cost an addresser wave-instruction).
template <bool MAYSPLIT = true>
__device__ __forceinline__ CriticLoads critic_row_load(const LossArgs& a) {
  const int b = threadIdx.x, B = a.B;
  const bool in = b < B;
  const int64_t nB = (int64_t)B * 4;
  const bool h2 = MAYSPLIT && a.qsplit > 1;  // second half of the partial sums (fwd_rows column split)
  const int64_t nBq = h2 ? 2 * nB : nB;
  CriticLoads L;
  for (int g = 0; g < 2; ++g) {
    const __amdgpu_buffer_rsrc_t rt = rlmd_rsrc(a.tpart[g], nBq), rq = rlmd_rsrc(a.qpart[g], nBq);
    L.qt[g] = rlmd_ldf(rt, b, in) + (MAYSPLIT ? rlmd_ldf(rt, B + b, in && h2) : 0.f);
    L.q[g] = rlmd_ldf(rq, b, in) + (MAYSPLIT ? rlmd_ldf(rq, B + b, in && h2) : 0.f);
  }
  L.rw = rlmd_ldf(rlmd_rsrc(a.r, nB), b, in);
  // optional operands through zero-sized resources when absent (the load then
  // reads 0): no branch around a load, whose use would wait right there
  L.lpn = rlmd_ldf(rlmd_rsrc(a.logp_next, a.logp_next ? nB : 0), b, in);
  L.dn = __builtin_amdgcn_raw_buffer_load_b8(rlmd_rsrc(a.done, B), in ? b : 0x7fffffff, 0, 0);
  L.eff = (int)__builtin_bit_cast(
      int32_t, __builtin_amdgcn_raw_buffer_load_b32(rlmd_rsrc(a.eff, a.eff ? nB : 0), in ? b * 4 : 0x7fffffff, 0, 0));
  L.has_eff = a.eff != nullptr;
  // the values this update started from (LearnState slots: another workgroup of
  // the same launch may be writing this update's new ones)
  const int rs = slot_rd(a.cnt);
  for (int g = 0; g < 2; ++g) {
    L.tb[g] = a.tb[g][0];
    L.qb[g] = a.qb[g][0];
    L.cauchy[g] = a.st->cauchy[rs][g];
  }
  L.log_alpha = a.st->log_alpha[rs];
  return L;
}

// block: form the block sums (o.s1, o.nan and the CIM kernel / TCAU truncation
// that need them).  A caller that only needs the rows' losses and gradients
// passes critic_loss_needs_block(a) (false for every loss but CIM and TCAU): the
// two block reductions (six barriers) are skipped and o.s1 / o.nan / o.kern are 0.
__device__ __forceinline__ bool critic_loss_needs_block(const LossArgs& a) {
  return a.loss_type == RLMD_LOSS_CIM || a.loss_type == RLMD_LOSS_TCAU;
}
__device__ __forceinline__ void critic_row_loss(const LossArgs& a, float* red, CriticRow& o, const CriticLoads& L,
                                                bool block = true) {
  const int b = threadIdx.x, B = a.B;
  const bool in = b < B;
  const LearnState* st = a.st;
  float qt[2] = {L.qt[0], L.qt[1]}, q[2] = {L.q[0], L.q[1]};
  const float rw = L.rw, lpn = L.lpn;
  const uint8_t dn = L.dn;
  const int eff = L.has_eff ? L.eff : 1;
  float y = 0.f;
  for (int g = 0; g < 2; ++g) {
    qt[g] += L.tb[g];
    q[g] += L.qb[g];
  }
  if (in) {
    if (dn) qt[0] = qt[1] = 0.f;
    const float m = fminf(qt[0], qt[1]);
    const float ge = powf(a.gamma, (float)eff);
    if (a.algo == RLMD_SAC) y = (a.reward_scale * rw + ge * m) - expf(L.log_alpha) * lpn;
    else y = rw + ge * m;
  } else {
    q[0] = q[1] = 0.f;
  }
  const float scale[2] = {L.cauchy[0], L.cauchy[1]};
  // R1: means of (t - q)^2 (CIM kernel), of y, q (TCAU), Nagy terms; NaN flag
  const float e0 = (y - q[0]) * (y - q[0]), e1 = (y - q[1]) * (y - q[1]);
  const float z0 = (y - q[0]) / scale[0], z1 = (y - q[1]) / scale[1];
  float s1[7] = {in ? e0 : 0.f, in ? e1 : 0.f, in ? y : 0.f, in ? q[0] : 0.f, in ? q[1] : 0.f,
                 in ? 1.f / (1.f + z0 * z0) : 0.f, in ? 1.f / (1.f + z1 * z1) : 0.f};
  float m1[1] = {(in && (isnan(q[0]) || isnan(q[1]) || isnan(y))) ? 1.f : 0.f};
  float s2[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float my = 0.f, mq0 = 0.f, mq1 = 0.f;
  if (block) {  // workgroup-uniform
    block_allreduce<7, 1>(s1, m1, red);
    const float me0 = s1[0] / B, me1 = s1[1] / B;
    my = s1[2] / B;
    mq0 = s1[3] / B;
    mq1 = s1[4] / B;
    // R2: population variances (two-pass, like torch.std(unbiased=False))
    s2[0] = in ? (e0 - me0) * (e0 - me0) : 0.f;
    s2[1] = in ? (e1 - me1) * (e1 - me1) : 0.f;
    s2[2] = in ? (y - my) * (y - my) : 0.f;
    s2[3] = in ? (q[0] - mq0) * (q[0] - mq0) : 0.f;
    s2[4] = in ? (q[1] - mq1) * (q[1] - mq1) : 0.f;
    float m2[1] = {-INFINITY};
    block_allreduce<5, 0>(s2, m2, red);
  } else {
#pragma unroll
    for (int v = 0; v < 7; ++v) s1[v] = 0.f;
    m1[0] = 0.f;
  }
  const float kern[2] = {sqrtf(s2[0] / B), sqrtf(s2[1] / B)};
  // TCAU 3-sigma truncation (critic_loss.py:26-50)
  float yt[2] = {y, y}, qt_[2] = {q[0], q[1]};
  bool qtr[2] = {false, false};
  if (a.loss_type == RLMD_LOSS_TCAU) {
    const bool ytr = fabsf(y - my) > 3.f * sqrtf(s2[2] / B);
    const float mq[2] = {mq0, mq1}, sq[2] = {sqrtf(s2[3] / B), sqrtf(s2[4] / B)};
    for (int g = 0; g < 2; ++g) {
      qtr[g] = fabsf(q[g] - mq[g]) > 3.f * sq[g];
      qt_[g] = qtr[g] ? 0.f : q[g];
      yt[g] = ytr ? 0.f : y;
    }
  }
  for (int g = 0; g < 2; ++g) {
    loss_and_grad(a.loss_type, qt_[g], yt[g], scale[g], kern[g], o.l[g], o.dl[g]);
    if (qtr[g]) o.dl[g] = 0.f;
    o.scale[g] = scale[g];
    o.kern[g] = kern[g];
  }
  o.in = in;
  o.y = y;
  for (int v = 0; v < 7; ++v) o.s1[v] = s1[v];
  o.nan = m1[0];
}

__device__ __forceinline__ void critic_row_loss(const LossArgs& a, float* red, CriticRow& o) {
  critic_row_loss(a, red, o, critic_row_load(a));
}

// top-k order: descending l1 + l2, ties by row (critic_loss.py:438-441); ~0 = absent
__device__ __forceinline__ uint64_t critic_sel_key(const CriticRow& o) {
  return o.in ? ((uint64_t)(~f2key(o.l[0] + o.l[1])) << 32) | (uint32_t)threadIdx.x : ~0ull;
}

// The whole critic loss in one workgroup.  runs: LDS uint64 [blockDim.x];
// rank_of: LDS int [3 * blockDim.x]; red: LDS float [16 * 9].  dq written when
// a.dq[0] is set.
// MAXW: the block's waves (block_rank).  part: -1 the whole loss; 0 / 1 split
// over two workgroups: part 0 everything but critic 1's tail index, part 1 only
// that (stats[9]) — the two Zipf ranks run in parallel.
template <int MAXW = 16>
__device__ __forceinline__ void critic_loss_block(const LossArgs& a, uint64_t* runs, int* rank_of, float* red,
                                                  int part = -1) {
  const int b = threadIdx.x, B = a.B, nth = blockDim.x;
  CriticRow o;
  critic_row_loss(a, red, o);
  const bool in = o.in;
  const float* l = o.l;
  if (in && a.y_out && part <= 0) a.y_out[b] = o.y;
  const int k = B > a.k ? a.k : B;
  bool sel = in;
  int rank = b;
  if (B > a.k) {
    if (a.rank_in) {
      rank = in ? a.rank_in[b] : B;
    } else {
      block_rank<MAXW>(critic_sel_key(o), runs, rank_of);
      rank = in ? rank_of[b] : B;
    }
    sel = in && rank < k;
  }
  // R3: mean / min / max of the selected losses per critic
  float s3[2] = {sel ? l[0] : 0.f, sel ? l[1] : 0.f};
  float m3[4] = {sel ? l[0] : -INFINITY, sel ? l[1] : -INFINITY, sel ? -l[0] : -INFINITY,
                 sel ? -l[1] : -INFINITY};
  block_allreduce<2, 4>(s3, m3, red);
  // Zipf-plot tail index of the selected losses' order statistics
  // (critic_loss.py:238-266): each critic's selected losses ranked among
  // themselves, descending, ties by selection rank; that rank is the slot
  if (part != 1)
    block_rank<MAXW>(sel ? ((uint64_t)(~f2key(l[0])) << 32) | (uint32_t)rank : ~0ull, runs, rank_of + nth);
  if (part != 0)
    block_rank<MAXW>(sel ? ((uint64_t)(~f2key(l[1])) << 32) | (uint32_t)rank : ~0ull, runs, rank_of + 2 * nth);
  const int rz0 = sel && part != 1 ? rank_of[nth + rank] : 0, rz1 = sel && part != 0 ? rank_of[2 * nth + rank] : 0;
  const float lg0 = sel ? logf(l[0] + a.log_noise) : 0.f;
  const float lg1 = sel ? logf(l[1] + a.log_noise) : 0.f;
  float s4[2] = {lg0, lg1};
  float m4[1] = {-INFINITY};
  block_allreduce<2, 0>(s4, m4, red);
  float s5[2] = {sel ? a.zipf_x[rz0] * (lg0 - s4[0] / k) : 0.f, sel ? a.zipf_x[rz1] * (lg1 - s4[1] / k) : 0.f};
  block_allreduce<2, 0>(s5, m4, red);
  // gradients of grad_scale * (mean(l1[sel]) + mean(l2[sel])) w.r.t. q
  if (in && a.dq[0]) {
    a.dq[0][b] = sel ? a.grad_scale * o.dl[0] / (float)k : 0.f;
    a.dq[1][b] = sel ? a.grad_scale * o.dl[1] / (float)k : 0.f;
  }
  if (b == 0 && part == 1) {  // critic 1's tail index only
    LearnState* st = a.st;
    a.stats[9] = 1.f / (s5[1] / a.zipf_x2);
    if (isnan(a.stats[9]) && atomicOr(&st->nan_flag, RLMD_STATUS_NAN_STATS) == 0) st->nan_update = a.cnt;
  }
  if (b == 0 && part != 1) {
    LearnState* st = a.st;
    float newc[2];
    for (int g = 0; g < 2; ++g) {  // Nagy Cauchy-scale update (critic_loss.py:74-101)
      const float ie = 1.f / (o.s1[5 + g] / B);
      newc[g] = ie > 1.f ? o.scale[g] * sqrtf(ie - 1.f) : o.scale[g];
      a.stats[0 + g] = s3[g] / k;
      a.stats[2 + g] = -m3[2 + g];
      a.stats[4 + g] = m3[g];
      a.stats[6 + g] = NAN;
      if (g == 0 || part < 0) a.stats[8 + g] = 1.f / (s5[g] / a.zipf_x2);
    }
    st->cauchy[slot_wr(a.cnt)][0] = newc[0];
    st->cauchy[slot_wr(a.cnt)][1] = newc[1];
    st->kernel[0] = o.kern[0];
    st->kernel[1] = o.kern[1];
    // NaN guards (tests/test_live_learning.py): bit 0 = NaN in the mini-batch's
    // q1 / q2 / target (sac_ / td3_critic_stability :29-116), bit 1 = NaN in the
    // critic statistics loss[0:6] + loss[8:10] (critic_learning :119-255, whose
    // exit() becomes this sticky flag); nan_update = learn counter at first set
    int32_t fl = 0;
    if (o.nan > 0.f) fl |= RLMD_STATUS_NAN_BATCH;
    bool sn = false;
#pragma unroll
    for (int v = 0; v < 10; ++v)
      if (v < 6 || v == 8 || (v == 9 && part < 0)) sn |= isnan(a.stats[v]);
    if (sn) fl |= RLMD_STATUS_NAN_STATS;
    // sticky; atomic: with part 1 running alongside, the first to set it stamps nan_update
    if (fl && atomicOr(&st->nan_flag, fl) == 0) st->nan_update = a.cnt;
    if (!a.keep_actor_slot) a.stats[10] = NAN;
    // no temperature step in this update: log alpha is the value it started from
    if (!a.keep_logtemp_slot) a.stats[11] = a.algo == RLMD_SAC ? st->log_alpha[slot_rd(a.cnt)] : NAN;
    a.stats[12] = newc[0];
    a.stats[13] = newc[1];
    a.stats[14] = o.kern[0];
    a.stats[15] = o.kern[1];
  }
}

}  // namespace
}  // namespace rlmd
