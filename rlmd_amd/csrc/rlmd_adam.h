// rlmd_adam.h — the optimiser step as per-element device code, applied in the
// epilogue of the weight-gradient GEMM (gemm.hip): the workgroup that owns an
// output tile of dW / db has the whole mini-batch reduction in registers and
// steps those parameters in place.
//
// Restates torch.optim.Adam defaults (_single_tensor_adam: betas .9/.999,
// eps 1e-8, bias corrections from Python floats), the Polyak target update
// (algo_sac.py:597-615 / algo_td3.py:533-563) and the SAC temperature step
// (algo_sac.py:580-595), plus the bf16/f32 compute copies of fc2.weight that
// the row kernels read (rows.hip RowNet: wc [H2p][H1p], wt [H1p][H2p]).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "learn_kernels.h"
#include "rlmd_common.h"

namespace rlmd {

struct AdamArgs {
  float* p;        // parameters of the stepped nets (index 0 = first element)
  const float* g;  // gradient slab 0 at the same index (locates GEMM outputs)
  float* m;
  float* v;
  float* target;  // Polyak target (nullable)
  int64_t n;
  float lr, tau;
  int32_t cnt;             // learn_step_cntr of this update (written back to LearnState)
  int32_t interval;        // Adam step count t = learn_cntr / interval
  float step_size, bc2_sqrt;            // lr / (1 - b1^t), sqrt(1 - b2^t): host-side, as torch's Python floats
  float temp_step_size, temp_bc2_sqrt;  // the same for the temperature step
  int32_t polyak_interval; // Polyak when learn_cntr % polyak_interval == 0 (0 = never)
  LearnState* st;
  int32_t temp;            // also step log_alpha (SAC)
  float lr_temp;
  int32_t temp_interval;
  float* stats;
  // compute copies of fc2.weight (rows.hip RowNet) refreshed for the updated
  // nets: net = i / net_size (ncopy nets), element (n, k) of its fc2.weight
  int32_t ncopy, bf16;
  int64_t net_size, w2_off;
  int32_t H1, H2, H1p, H2p;
  void* wc[2];
  void* wt[2];
  void* twc[2];  // Polyak targets' copies (nullable)
  void* twt[2];
};

namespace {

__device__ __forceinline__ void store_copy(void* base, int64_t i, float v, int bf16) {
  if (bf16) {
    unsigned u = __float_as_uint(v);
    u += 0x7fffu + ((u >> 16) & 1u);  // RNE (finite weights)
    rlmd_st_wt(static_cast<unsigned short*>(base) + i, (unsigned short)(u >> 16));
  } else {
    rlmd_st_wt(static_cast<float*>(base) + i, v);
  }
}

__device__ __forceinline__ bool adam_polyak(const AdamArgs& a) {
  return a.target && a.polyak_interval > 0 && (a.cnt % a.polyak_interval) == 0;
}

// One parameter's optimiser state, loaded ahead of its gradient (range-checked
// buffer loads: an element index < 0 reads zeros and is never stored).
struct AdamIn {
  float m, v, p, t;
};

__device__ __forceinline__ AdamIn adam_load(const AdamArgs& a, int i, bool polyak) {
  const int n4 = (int)(a.n * 4), off = i >= 0 ? i * 4 : 0x7fffffff;
  AdamIn o;
  o.m = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                     rlmd_rsrc_wave(a.m, n4), off, 0, 0));
  o.v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                     rlmd_rsrc_wave(a.v, n4), off, 0, 0));
  o.p = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                     rlmd_rsrc_wave(a.p, n4), off, 0, 0));
  o.t = polyak ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                               rlmd_rsrc_wave(a.target, n4),
                                               off, 0, 0))
               : 0.f;
  return o;
}

// Compute-copy destinations of one net (wc / wt and the Polyak target's).
struct CopyDst {
  void *wc, *wt, *twc, *twt;
};
// For a workgroup-uniform net: read the kernel-argument pointers once, up front.
__device__ __forceinline__ CopyDst copy_dst(const AdamArgs& a, int net) {
  return net == 0 ? CopyDst{a.wc[0], a.wt[0], a.twc[0], a.twt[0]} : CopyDst{a.wc[1], a.wt[1], a.twc[1], a.twt[1]};
}

// One parameter: Adam with gradient g, then Polyak; the new value and target
// value returned (the caller writes the compute copies).
__device__ __forceinline__ void adam_core(const AdamArgs& a, int i, float g, const AdamIn& in, bool polyak, float& p,
                                          float& tv) {
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
  float m = in.m, v = in.v;
  m = m + (1.f - b1) * (g - m);
  v = v * b2 + (1.f - b2) * g * g;
  rlmd_st_wt(a.m + i, m);
  rlmd_st_wt(a.v + i, v);
  const float denom = sqrtf(v) / a.bc2_sqrt + eps;
  p = in.p - a.step_size * (m / denom);
  rlmd_st_wt(a.p + i, p);
  tv = 0.f;
  if (polyak) {
    tv = a.tau * p + (1.f - a.tau) * in.t;
    rlmd_st_wt(a.target + i, tv);
  }
}

// One parameter: Adam with gradient g, then Polyak and the compute copies.
// jw2: the element's index inside its net's fc2.weight (-1: not fc2.weight).
__device__ __forceinline__ void adam_apply_dst(const AdamArgs& a, int i, float g, const AdamIn& in, bool polyak,
                                               int jw2, const CopyDst& cd) {
  float p, tv;
  adam_core(a, i, g, in, polyak, p, tv);
  if (jw2 >= 0) {
    const int n = jw2 / a.H1, k = jw2 - n * a.H1;
    const int64_t ic = frag_index(n, k, a.H1p, a.bf16), it = frag_index(k, n, a.H2p, a.bf16);
    store_copy(cd.wc, ic, p, a.bf16);
    store_copy(cd.wt, it, p, a.bf16);
    if (polyak && cd.twc) {
      store_copy(cd.twc, ic, tv, a.bf16);
      store_copy(cd.twt, it, tv, a.bf16);
    }
  }
}

// The same for any element of the stepped nets (net = i / net_size per lane).
__device__ __forceinline__ void adam_apply(const AdamArgs& a, int i, float g, const AdamIn& in, bool polyak) {
  int jw2 = -1, net = 0;
  if (a.ncopy) {
    const int ns = (int)a.net_size;
    net = i / ns;
    const int j = i - net * ns - (int)a.w2_off;
    if (net < a.ncopy && j >= 0 && j < a.H1 * a.H2) jw2 = j;
  }
  adam_apply_dst(a, i, g, in, polyak, jw2, copy_dst(a, net));
}

// Once per step (one thread): the learner counter and the temperature Adam.
// The critics' call (temp = 0; every update makes it, before any actor step)
// carries log alpha into this update's slot; an actor call with a temperature
// step then overwrites that slot from the update's starting value.
__device__ __forceinline__ void adam_scalar_step(const AdamArgs& a) {
  LearnState* st = a.st;
  const int rs = slot_rd(a.cnt), ws = slot_wr(a.cnt);
  st->learn_cntr = a.cnt;
  if (!a.temp) {
    st->log_alpha[ws] = st->log_alpha[rs];
    return;
  }
  if (a.cnt % a.temp_interval == 0) {
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
    const float g = st->pad_temp_grad;
    const float m = st->temp_m + (1.f - b1) * (g - st->temp_m);
    const float v = st->temp_v * b2 + (1.f - b2) * g * g;
    st->temp_m = m;
    st->temp_v = v;
    const float denom = sqrtf(v) / a.temp_bc2_sqrt + eps;
    st->log_alpha[ws] = st->log_alpha[rs] - a.temp_step_size * (m / denom);
  }
  if (a.stats) a.stats[11] = st->log_alpha[ws];
}

}  // namespace
}  // namespace rlmd
