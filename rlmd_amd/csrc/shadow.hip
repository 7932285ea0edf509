// shadow.hip — power-law shadow means of the critic losses on the device (gfx950).
//
// Replaces tools/utils.py:374-400 (shadow_means) and :441-471 (agent_shadow_mean),
// evaluated by the reference at every evaluation and episode end on the loss list
// learn() returned (algo_sac.py:502-514): loss[6:8] <- shadow mean of critic 1 / 2,
//
//   low, high = min * low_mul, max * high_mul
//   shadow    = low + (high - low) * exp(a / high) * (a / high)**a
//                     * gamma(1 - a) * gammaincc(1 - a, a / high)      if a < 1
//             = the empirical mean loss[0 | 1]                          otherwise,
//
// with a = the Zipf tail index loss[8 | 9].  The loss entries are float32 0-d
// arrays, so every operation above is float32 under NumPy 2 (checked on the
// reference: the result is np.float32): SciPy's gamma / gammaincc float32 loops
// evaluate in double and round once; exp, pow, *, +, - are float32 ops in the
// order written.  gammaincc is restated from the published Cephes igamc
// algorithm SciPy uses (scipy/special/cephes/igam.c: the branch selection and
// the igam / igamc power series and the Legendre continued fraction; a <= 20 and
// far from the Temme regime, which a = 1 - alpha with alpha in (-19, 1) is).
#include <math.h>

#pragma clang fp contract(off)

#include "rlmd_common.h"
#include "rlmd_internal.h"

namespace {

constexpr double kMachEp = 1.11022302462515654042e-16;
constexpr double kMaxLog = 7.09782712893383996843e2;
constexpr double kBig = 4.503599627370496e15;
constexpr double kBigInv = 2.22044604925031308085e-16;
constexpr int kMaxIter = 2000;

// x^a e^-x / Gamma(a)
__device__ double igam_fac(double a, double x) {
  const double ax = a * log(x) - x - lgamma(a);
  if (ax < -kMaxLog) return 0.0;
  return exp(ax);
}

__device__ double igam_series(double a, double x) {
  const double ax = igam_fac(a, x);
  if (ax == 0.0) return 0.0;
  double r = a, c = 1.0, ans = 1.0;
  for (int i = 0; i < kMaxIter; ++i) {
    r += 1.0;
    c *= x / r;
    ans += c;
    if (c <= kMachEp * ans) break;
  }
  return ans * ax / a;
}

__device__ double igamc_series(double a, double x) {
  double fac = 1.0, sum = 0.0;
  for (int n = 1; n < kMaxIter; ++n) {
    fac *= -x / n;
    const double term = fac / (a + n);
    sum += term;
    if (fabs(term) <= kMachEp * fabs(sum)) break;
  }
  const double logx = log(x);
  const double term = -expm1(a * logx - lgamma(1.0 + a));
  return term - exp(a * logx - lgamma(a)) * sum;
}

__device__ double igamc_cf(double a, double x) {
  const double ax = igam_fac(a, x);
  if (ax == 0.0) return 0.0;
  double y = 1.0 - a, z = x + y + 1.0, c = 0.0;
  double pkm2 = 1.0, qkm2 = x, pkm1 = x + 1.0, qkm1 = z * x;
  double ans = pkm1 / qkm1;
  for (int i = 0; i < kMaxIter; ++i) {
    c += 1.0;
    y += 1.0;
    z += 2.0;
    const double yc = y * c;
    const double pk = pkm1 * z - pkm2 * yc;
    const double qk = qkm1 * z - qkm2 * yc;
    double t = 1.0;
    if (qk != 0.0) {
      const double r = pk / qk;
      t = fabs((ans - r) / r);
      ans = r;
    }
    pkm2 = pkm1;
    pkm1 = pk;
    qkm2 = qkm1;
    qkm1 = qk;
    if (fabs(pk) > kBig) {
      pkm2 *= kBigInv;
      pkm1 *= kBigInv;
      qkm2 *= kBigInv;
      qkm1 *= kBigInv;
    }
    if (t <= kMachEp) break;
  }
  return ans * ax;
}

// regularised upper incomplete gamma Q(a, x) (Cephes igamc branch selection)
__device__ double gammaincc(double a, double x) {
  if (x < 0.0 || a < 0.0 || isnan(a) || isnan(x)) return NAN;
  if (a == 0.0) return x > 0.0 ? 0.0 : NAN;
  if (x == 0.0) return 1.0;
  if (isinf(a)) return isinf(x) ? NAN : 1.0;
  if (isinf(x)) return 0.0;
  if (x > 1.1) return x < a ? 1.0 - igam_series(a, x) : igamc_cf(a, x);
  if (x <= 0.5) return -0.4 / log(x) < a ? 1.0 - igam_series(a, x) : igamc_series(a, x);
  return x * 1.1 < a ? 1.0 - igam_series(a, x) : igamc_series(a, x);
}

// SciPy's gamma for float32 inputs: Cephes Gamma in double, NaN at poles
__device__ double sp_gamma(double a) {
  if (a <= 0.0 && a == floor(a)) return NAN;
  return tgamma(a);
}

__device__ float shadow_mean(float alpha, float mn, float mx, float low_mul, float high_mul) {
  const float low = mn * low_mul, high = mx * high_mul;
  const float a1 = 1.0f - alpha;
  const float x = alpha / high;
  const float up = (float)sp_gamma((double)a1) * (float)gammaincc((double)a1, (double)x);
  return low + (high - low) * expf(x) * powf(x, alpha) * up;
}

// shadow_means on float64 inputs (the aggregation path: tools/aggregate_data.py
// passes float64 arrays, so every operation is double)
__device__ double shadow_mean_f64(double alpha, double mn, double mx, double low_mul, double high_mul) {
  const double low = mn * low_mul, high = mx * high_mul;
  const double x = alpha / high;
  const double up = sp_gamma(1.0 - alpha) * gammaincc(1.0 - alpha, x);
  return low + (high - low) * exp(x) * pow(x, alpha) * up;
}

// shadow_equiv (tools/utils.py:406-438): the max multiplier m with
// shadow_means(alpha, min, max, min_mul, m) == mean, from x0 = 1 (x0 itself when
// alpha >= 1 or NaN).  The reference solves it with MINPACK hybrd; in one
// dimension that is a Newton iteration on a forward-difference derivative
// (step sqrt(eps)|x|) inside a trust region of 100 |x0| scaled by |f'|, which
// is restated here with step halving while |f| does not decrease, stopping at
// hybrd's xtol (1.49012e-8 relative) or f == 0.
__global__ void __launch_bounds__(64) shadow_equiv_kernel(const double* mean, const double* alpha, const double* mn,
                                                          const double* mx, double min_mul, int64_t n, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = alpha[i], mu = mean[i], lo = mn[i], hi = mx[i];
  if (!(a < 1.0)) {
    out[i] = 1.0;
    return;
  }
  auto F = [&](double m) { return shadow_mean_f64(a, lo, hi, min_mul, m) - mu; };
  constexpr double kXtol = 1.49012e-8, kEps = 1.4901161193847656e-8;  // sqrt(DBL_EPSILON)
  double x = 1.0, f = F(x);
  const double delta_scale = 100.0;  // hybrd's factor: trust radius 100 |x0| in scaled units
  for (int it = 0; it < 200 && f != 0.0 && isfinite(f); ++it) {
    const double h = kEps * (x != 0.0 ? fabs(x) : 1.0);
    const double J = (F(x + h) - f) / h;
    if (!(J != 0.0) || !isfinite(J)) break;
    double p = -f / J;
    const double cap = delta_scale * fabs(x);
    if (fabs(p) > cap) p = p > 0 ? cap : -cap;
    double fn = F(x + p);
    for (int k = 0; k < 60 && !(isfinite(fn) && fabs(fn) < fabs(f)); ++k) {
      p *= 0.5;
      fn = F(x + p);
    }
    if (!(isfinite(fn) && fabs(fn) <= fabs(f))) break;
    x += p;
    f = fn;
    if (fabs(p) <= kXtol * fabs(x)) break;
  }
  out[i] = x;
}

// one thread per (row, critic): stats rows [loss[11] | ...] with leading dimension ld
__global__ void __launch_bounds__(64) shadow_kernel(const float* stats, int rows, int ld, float low_mul,
                                                    float high_mul, float* out, int ldo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * rows) return;
  const int row = i >> 1, c = i & 1;
  const float* l = stats + (int64_t)row * ld;
  const float alpha = l[8 + c];
  out[(int64_t)row * ldo + c] = alpha < 1.0f ? shadow_mean(alpha, l[2 + c], l[4 + c], low_mul, high_mul) : l[c];
}

}  // namespace

extern "C" {

int rlmd_shadow_means(const float* stats_dev, int32_t rows, int32_t ld, float low_mul, float high_mul,
                      float* shadow_dev, int32_t ldo, void* stream) {
  RLMD_CHECK(stats_dev && shadow_dev, "null argument");
  RLMD_CHECK(rows >= 0 && ld >= 11 && ldo >= 2, "bad shape");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(shadow_kernel, dim3((2 * rows + 63) / 64), dim3(64), 0, (hipStream_t)stream, stats_dev, rows,
                     ld, low_mul, high_mul, shadow_dev, ldo);
  RLMD_LAUNCH_CHECK();
  return 0;
}

int rlmd_shadow_equiv(const double* mean_dev, const double* alpha_dev, const double* min_dev, const double* max_dev,
                      double min_mul, int64_t n, double* out_dev, void* stream) {
  RLMD_CHECK(mean_dev && alpha_dev && min_dev && max_dev && out_dev, "null argument");
  RLMD_CHECK(n >= 0, "bad length");
  if (n == 0) return 0;
  hipLaunchKernelGGL(shadow_equiv_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     mean_dev, alpha_dev, min_dev, max_dev, min_mul, n, out_dev);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
