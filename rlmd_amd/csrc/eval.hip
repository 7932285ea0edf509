// eval.hip — evaluation summary statistics on the device (gfx950).
//
// Replaces the NumPy summary of tools/eval_episodes.py:289-330 over one batch of
// evaluation episodes (rlmd_eval_rollout's outputs), bit-for-bit with NumPy:
//   np.mean               pairwise summation (numpy/_core/src/umath/loops_utils.h:
//                         sequential below 8 elements, 8 accumulators up to 128,
//                         recursive halving above), then one division;
//   np.std(ddof=0)        mean, squared deviations, pairwise sum, division, sqrt;
//   np.percentile(q, method="median_unbiased")
//                         Hyndman & Fan type 8: virtual index n q + (1/3 + q/3) - 1,
//                         clamped neighbours, NumPy's two-sided lerp.
// One workgroup: ranks sort the three sample vectors in LDS (ties by index, a
// stable sort), then one thread evaluates the statistics in NumPy's order.
// Built with -ffp-contract=off (rlmd_amd/build.py): a contracted lerp or
// deviation product would round differently from NumPy.
#include <math.h>

#pragma clang fp contract(off)

#include "rlmd_common.h"
#include "rlmd_internal.h"

namespace {

constexpr int kMaxEval = 1024;

__device__ double pairwise_sum(const double* x, int n) {
  if (n < 8) {
    double res = 0.0;  // NumPy starts from -0.0 only for empty reductions; here n >= 1
    for (int i = 0; i < n; ++i) res = i == 0 ? x[0] : res + x[i];
    return n == 0 ? 0.0 : res;
  }
  if (n <= 128) {
    double r[8];
    for (int k = 0; k < 8; ++k) r[k] = x[k];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int k = 0; k < 8; ++k) r[k] += x[i + k];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x[i];
    return res;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(x, n2) + pairwise_sum(x + n2, n - n2);
}

__device__ double np_mean(const double* x, int n) { return pairwise_sum(x, n) / (double)n; }

// np.mean(np.abs(x - m)) and np.std(x, ddof=0) need a scratch vector
__device__ double np_mad(const double* x, int n, double m, double* tmp) {
  for (int i = 0; i < n; ++i) tmp[i] = fabs(x[i] - m);
  return np_mean(tmp, n);
}
__device__ double np_std(const double* x, int n, double* tmp) {
  const double m = pairwise_sum(x, n) / (double)n;
  for (int i = 0; i < n; ++i) {
    const double d = x[i] - m;
    tmp[i] = d * d;
  }
  return sqrt(pairwise_sum(tmp, n) / (double)n);
}

// np.percentile(x, q100, method="median_unbiased") on the sorted sample s
__device__ double np_percentile_mu(const double* s, int n, double q100) {
  const double q = q100 / 100.0;
  const double alpha = 1.0 / 3.0, beta = 1.0 / 3.0;
  const double vi = (double)n * q + (alpha + q * (1.0 - alpha - beta)) - 1.0;
  double prev_f = floor(vi);
  int prev = (int)prev_f, next = prev + 1;
  if (vi >= (double)(n - 1)) {
    prev_f = -1.0;
    prev = next = n - 1;
  } else if (vi < 0.0) {
    prev_f = 0.0;
    prev = next = 0;
  }
  const double gamma = vi - prev_f;
  const double a = s[prev], b = s[next];
  const double d = b - a;
  return gamma >= 0.5 ? b - d * (1.0 - gamma) : a + d * gamma;
}

__device__ void rank_sort(const double* x, double* out, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double v = x[i];
    int r = 0;
    for (int j = 0; j < n; ++j) r += (x[j] < v) || (x[j] == v && j < i);
    out[r] = v;
  }
}

// stats[17] = eval_episodes.py:322-338 in order, then mean stop-loss and mean
// retention (risk columns 4 and 5, printed for InvB / InvC), NaN when absent.
__global__ void __launch_bounds__(1024) eval_stats_kernel(const double* reward, const int32_t* steps,
                                                          const double* risk, int n, int R, int has_stop,
                                                          int has_ret, double* stats) {
  __shared__ double rw[kMaxEval], val[kMaxEval], st[kMaxEval], lev[kMaxEval];
  __shared__ double srw[kMaxEval], sval[kMaxEval], sst[kMaxEval], tmp[kMaxEval];
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    rw[i] = reward[i];
    val[i] = risk[(int64_t)i * R + 1];
    lev[i] = risk[(int64_t)i * R + 3];
    st[i] = (double)steps[i];
  }
  __syncthreads();
  rank_sort(rw, srw, n);
  rank_sort(val, sval, n);
  rank_sort(st, sst, n);
  __syncthreads();
  if (threadIdx.x != 0) return;
  const double mean_reward = np_mean(rw, n);
  const double med_reward = np_percentile_mu(srw, n, 50.0);
  const double reward_95 = np_percentile_mu(srw, n, 5.0);
  const double mad_reward = np_mad(rw, n, mean_reward, tmp);
  const double std_reward = np_std(rw, n, tmp);
  const double mean_val = np_mean(val, n);
  const double med_val = np_percentile_mu(sval, n, 50.0);
  const double val_95 = np_percentile_mu(sval, n, 5.0);
  const double mad_val = np_mad(val, n, mean_val, tmp);
  const double mean_lev = np_mean(lev, n);
  const double mean_step = np_mean(st, n);
  const double med_step = np_percentile_mu(sst, n, 50.0);
  const double step_95 = np_percentile_mu(sst, n, 5.0);
  const double mad_step = np_mad(st, n, mean_step, tmp);
  const double std_step = np_std(st, n, tmp);
  stats[0] = mean_lev * 100;
  stats[1] = (mean_reward - 1) * 100;
  stats[2] = (med_reward - 1) * 100;
  stats[3] = (reward_95 - 1) * 100;
  stats[4] = mad_reward * 100;
  stats[5] = std_reward * 100;
  stats[6] = mean_val;
  stats[7] = med_val;
  stats[8] = val_95;
  stats[9] = mad_val;
  stats[10] = mean_step;
  stats[11] = med_step;
  stats[12] = step_95;
  stats[13] = mad_step;
  stats[14] = std_step;
  double col[2] = {NAN, NAN};
  for (int c = 0; c < 2; ++c) {
    if ((c == 0 && !has_stop) || (c == 1 && !has_ret)) continue;
    for (int i = 0; i < n; ++i) tmp[i] = risk[(int64_t)i * R + 4 + c];
    col[c] = np_mean(tmp, n);
  }
  stats[15] = col[0];
  stats[16] = col[1];
}

}  // namespace

extern "C" {

int rlmd_eval_stats(const double* reward, const int32_t* steps, const double* risk, int32_t n, int32_t risk_dim,
                    int32_t investor, double* stats, void* stream) {
  RLMD_CHECK(reward && steps && risk && stats, "null argument");
  RLMD_CHECK(n >= 1 && n <= kMaxEval, "eval statistics: 1..1024 episodes");
  RLMD_CHECK(risk_dim >= 4, "risk vector too short");
  const int has_stop = investor == RLMD_INV_B || investor == RLMD_INV_C;
  const int has_ret = investor == RLMD_INV_C;
  hipLaunchKernelGGL(eval_stats_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, reward, steps, risk, n,
                     risk_dim, has_stop, has_ret, stats);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
