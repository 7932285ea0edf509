// rlmd_policy.h — the SAC policy's stochastic action per component, shared by
// the acting kernel (act.hip), the head kernel (learn.hip) and the row kernels
// of the update (rows.hip, forward and backward).
//
// ActorNetwork (algos/networks_sac.py) offers three samplers, chosen by
// inputs["s_dist"] (algo_sac.py:207-218, :326-343, :525-542):
//   "N"   stochastic_uv_gaussian  (:136-178)  u = mu + eps sigma, Normal log-density
//   "L"   stochastic_uv_laplace   (:180-220)  torch Laplace.rsample: w ~ U(eps_f32 - 1, 1),
//                                             u = mu - sigma sign(w) log1p(-|w|), Laplace log-density
//   "MVN" stochastic_mv_gaussian  (:222-258)  the scale is used as a VARIANCE: cov =
//                                             diag(scale), L = cholesky = diag(sqrt(scale)),
//                                             u = mu + L eps, MultivariateNormal log-density
// after forward() (:101-134): sigma = exp(clamp(log_scale, min, max)), the NaN
// scrub (mu -> 0, scale -> 3).  Every sampler then bounds a = tanh(u) max_action
// and subtracts sum log(1 - (a / max_action)^2 + reparam_noise).
#pragma once
#include <math.h>

#include "rlmd_common.h"

namespace rlmd {
namespace {

constexpr float kHalfLog2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
constexpr double kF32Eps = 1.1920928955078125e-07;        // torch.finfo(float32).eps

// Philox noise of component j of row b: a standard normal (N, MVN) or the
// Laplace sampler's uniform in (eps - 1, 1).  The normal is an f32 Box-Muller
// pair from 24-bit uniforms with the hardware log / sin / cos (the reference
// draws this exploration noise in f32 with torch; an f64 pair here was a
// ~5k-cycle chain on the target pass's critical path).  The env's own draws
// (env.hip) keep NumPy's f64 construction.
__device__ __forceinline__ float policy_draw(int dist, uint64_t seed, uint32_t b, uint32_t ctr, uint32_t tag,
                                             int j) {
  const rlmd_u32x4 v = rlmd_philox(seed, b, ctr, tag, (uint32_t)(j >> 1));
  if (dist == RLMD_DIST_L) {
    const double u01 = (j & 1) ? rlmd_u01(v.z, v.w) : rlmd_u01(v.x, v.y);
    const float w = (float)((kF32Eps - 1.0) + (2.0 - kF32Eps) * u01);
    return fminf(w, 0x1.fffffep-1f);  // strictly below 1: log1p(-|w|) finite
  }
  const float u1 = (float)(v.x >> 8) * 0x1p-24f;  // [0, 1): 1 - u1 in (0, 1]
  const float u2 = (float)(v.z >> 8) * 0x1p-24f;
  const float r = __fsqrt_rn(-2.f * __logf(1.f - u1));
  float sn, cs;
  __sincosf(6.28318530717958647692f * u2, &sn, &cs);
  return (j & 1) ? r * sn : r * cs;
}

// One component of the sampler.  In: mu and the log-scale head with biases,
// the noise (eps, or w for Laplace).  Out: the scrubbed mu, sigma (the standard
// deviation; sqrt of the variance head for MVN), the reparameterised u, the
// noise's multiplier c (du/dsigma: eps, or -sign(w) log1p(-|w|)), and this
// component's log-density terms: N and L add `lp` to the row's sum; MVN adds
// `m2` to the Mahalanobis sum and `hld` to the half log-determinant.
struct PolicyComp {
  float mu, sigma, u, c, lp, m2, hld;
};

__device__ __forceinline__ PolicyComp policy_comp(int dist, float mu, float ls_raw, float noise, float ls_min,
                                                  float ls_max) {
  PolicyComp o;
  const float ls = fminf(fmaxf(ls_raw, ls_min), ls_max);
  float scale = expf(ls);
  if (!isfinite(mu)) mu = 0.f;  // NaN scrub (networks_sac.py:131-134), per element
  if (!isfinite(scale)) scale = 3.f;
  o.mu = mu;
  o.lp = o.m2 = o.hld = 0.f;
  if (dist == RLMD_DIST_L) {
    const float sg = noise > 0.f ? 1.f : (noise < 0.f ? -1.f : 0.f);
    const float l1p = log1pf(-fabsf(noise));
    o.sigma = scale;
    o.u = mu - (scale * sg) * l1p;
    o.c = -sg * l1p;
    o.lp = -logf(2.f * scale) - fabsf(o.u - mu) / scale;
  } else if (dist == RLMD_DIST_MVN) {
    const float sd = sqrtf(scale);  // cholesky(diag(var))
    o.sigma = sd;
    o.u = mu + sd * noise;
    o.c = noise;
    const float z = (o.u - mu) / sd;  // triangular solve of a diagonal factor
    o.m2 = z * z;
    o.hld = logf(sd);
  } else {
    o.sigma = scale;
    o.u = mu + noise * scale;
    o.c = noise;
    const float d = o.u - mu;
    o.lp = -(d * d) / (2.f * (scale * scale)) - logf(scale) - kHalfLog2Pi;
  }
  return o;
}

// Row log-probability from the summed terms (A components): MVN as
// MultivariateNormal.log_prob, then minus the summed tanh corrections.
__device__ __forceinline__ float policy_logp(int dist, int A, float lp_sum, float m2_sum, float hld_sum,
                                             float jac_sum) {
  const float lp = dist == RLMD_DIST_MVN ? -0.5f * ((float)A * (2.f * kHalfLog2Pi) + m2_sum) - hld_sum : lp_sum;
  return lp - jac_sum;
}

// Backward of one component: dL/da (da), dL/dlogp (dlp) -> dL/dmu and dL/d
// log_scale_raw (zero outside the clamp's pass-through range).
__device__ __forceinline__ void policy_comp_bwd(int dist, float mu, float sigma, float c, float u, float ls_raw,
                                                float da, float dlp, float max_action, float reparam_noise,
                                                float ls_min, float ls_max, float& dmu, float& dls) {
  const float t = tanhf(u);
  const float om = 1.f - t * t;
  const float d = u - mu;
  float dlpn_du, dlpn_dmu, dlpn_dsig;
  if (dist == RLMD_DIST_L) {
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    dlpn_du = -sg / sigma;
    dlpn_dmu = sg / sigma;
    dlpn_dsig = -1.f / sigma + fabsf(d) / (sigma * sigma);
  } else {
    dlpn_du = -d / (sigma * sigma);
    dlpn_dmu = d / (sigma * sigma);
    dlpn_dsig = (d * d) / (sigma * sigma * sigma) - 1.f / sigma;
  }
  const float dlogp_du = dlpn_du + 2.f * t * om / (om + reparam_noise);
  const float du = da * max_action * om + dlp * dlogp_du;
  dmu = du + dlp * dlpn_dmu;
  const float dsig = du * c + dlp * dlpn_dsig;
  const bool live = ls_raw >= ls_min && ls_raw <= ls_max;  // clamp passes [min, max]
  // dsigma/dlog_scale: sigma (N, L); sqrt(exp(ls)) / 2 for the MVN variance head
  dls = live ? dsig * (dist == RLMD_DIST_MVN ? 0.5f * sigma : sigma) : 0.f;
}

}  // namespace
}  // namespace rlmd
