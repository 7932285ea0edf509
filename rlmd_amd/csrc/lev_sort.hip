// lev_sort.hip — fixed-leverage sweeps with per-step sorts (gfx950).
//
// Replaces dice_smart_lev (lev/lev_exp.py:586-705), gbm_smart_lev (:1008-1119)
// and dice_sh_smart_lev (:1209-1332) — and, statistics of the final values only,
// the *_fixed_final_lev family (:56-127, :508-585, :935-1007, :1121-1208):
// for every leverage l each investor's value
// is multiplied step by step by its gamble factor (float32, as the reference's
// torch tensors), and after each step t >= 1 the values are sorted descending:
// the first `top` form the top group, the rest the adjusted group, and the
// table column [mean, mean_top, mean_adj, mad x3, std x3, median x3, lev] is
// stored (std unbiased=False, median = the lower middle element, torch.median).
//
// Unlike the coin flip (lev.hip: the value is monotone in one up-count, so
// histograms replace the sorts) a die's value depends on two counts and a GBM
// path's on a continuous sum, so the order really is sorted here, once per
// (step, leverage), on the device:
//   lev_advance_kernel   values *= factor(outcome[i][t]) for every (lev, investor)
//                        (categorical: factor table [lev][3] from the host,
//                        computed with the reference's f32 arithmetic; GBM:
//                        expf(lev * outcome)), one pass over the u8 / f32 column
//   hipcub DeviceRadixSort::SortKeysDescending per leverage (f32 keys)
//   lev_sorted_sums_kernel  per (lev, chunk): group sums in f64 (pass 1), then
//                        |v - mean| and (v - mean)^2 sums (pass 2), fixed
//                        chunk order — deterministic
//   lev_sorted_fold_kernel  one thread per lev: fold the chunks, write the column
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>

#include <algorithm>
#include <vector>

#include "../../include/rlmd_abi.h"
#include "rlmd_common.h"

#define RLMD_TRY_INT(x)    \
  do {                     \
    const int _r = (x);    \
    if (_r) return _r;     \
  } while (0)

namespace {

constexpr int kChunks = 64;  // partial-sum chunks per leverage
constexpr int kT = 256;

struct SortedArgs {
  int kind;  // 0 categorical (u8 outcomes 0/1/2), 1 GBM (f32 outcomes)
  const uint8_t* cat;
  const float* gbm;
  int64_t investors, ld;
  int n_lev;
  const float* table;  // [n_lev][3] (categorical)
  const float* levs;   // [n_lev]
  float* val;          // [n_lev][investors]
};

__device__ __forceinline__ float factor(const SortedArgs& a, int l, int64_t i, int t) {
  if (a.kind == 0) {
    const int o = a.cat[i * a.ld + t];
    return a.table[l * 3 + (o > 2 ? 2 : o)];
  }
  return expf(a.levs[l] * a.gbm[i * a.ld + t]);
}

// t == 0: val = value_0 * factor(t = 0); else val *= factor(t)
__global__ void __launch_bounds__(kT) lev_advance_kernel(SortedArgs a, int t, float value_0) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int l = blockIdx.y;
  if (i >= a.investors) return;
  float* v = a.val + (int64_t)l * a.investors + i;
  const float g = factor(a, l, i, t);
  *v = t == 0 ? value_0 * g : *v * g;
}

// group sums over sorted-descending values s[0, N): all, top = [0, top), adj =
// [top, N).  pass 0: sums; pass 1: |v - m| and (v - m)^2 with the means m.
template <typename VT>
__global__ void __launch_bounds__(kT) lev_sorted_sums_kernel(const VT* sorted, int64_t N, int64_t top,
                                                             const double* means, int pass, double* part) {
  const int l = blockIdx.y, c = blockIdx.x;
  const VT* s = sorted + (int64_t)l * N;
  const int64_t per = (N + kChunks - 1) / kChunks, b0 = c * per, b1 = b0 + per < N ? b0 + per : N;
  double acc[6] = {0, 0, 0, 0, 0, 0};  // pass 0: all, top, adj ; pass 1: |.| all/top/adj, sq all/top/adj
  const double ma = pass ? means[l * 3 + 0] : 0.0, mt = pass ? means[l * 3 + 1] : 0.0,
               md = pass ? means[l * 3 + 2] : 0.0;
  for (int64_t i = b0 + threadIdx.x; i < b1; i += kT) {
    const double v = s[i];
    const bool is_top = i < top;
    if (!pass) {
      acc[0] += v;
      acc[is_top ? 1 : 2] += v;
    } else {
      const double da = v - ma, dg = v - (is_top ? mt : md);
      acc[0] += fabs(da);
      acc[3] += da * da;
      acc[is_top ? 1 : 2] += fabs(dg);
      acc[is_top ? 4 : 5] += dg * dg;
    }
  }
  __shared__ double red[6][kT];
  for (int q = 0; q < 6; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int h = kT / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
      for (int q = 0; q < 6; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + h];
    __syncthreads();
  }
  if ((int)threadIdx.x < 6) part[((int64_t)l * kChunks + c) * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// pass 0: means of the three groups; pass 1: the table column at step t
// rows: table rows per configuration; row0: where the 12 statistics go; the
// n_extra constants extra[l][*] fill rows row0 + 12 ... (the sweeps' lev row,
// the big-brain stop / roll rows)
template <typename VT>
__global__ void lev_sorted_fold_kernel(const VT* sorted, int64_t N, int64_t top, int n_lev, const double* part,
                                       int pass, double* means, const float* extra, int n_extra, float* data,
                                       int rows, int row0, int steps, int t) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n_lev) return;
  double s[6] = {0, 0, 0, 0, 0, 0};
  for (int c = 0; c < kChunks; ++c)
    for (int q = 0; q < 6; ++q) s[q] += part[((int64_t)l * kChunks + c) * 6 + q];
  const double na = (double)N, nt = (double)top, nd = (double)(N - top);
  if (!pass) {
    means[l * 3 + 0] = s[0] / na;
    means[l * 3 + 1] = s[1] / nt;
    means[l * 3 + 2] = s[2] / nd;
    return;
  }
  const VT* v = sorted + (int64_t)l * N;
  // lower medians: ascending index (n - 1) / 2 of each group, read from the
  // descending order
  auto med = [&](int64_t lo, int64_t n) -> double { return n > 0 ? (double)v[lo + n - 1 - (n - 1) / 2] : NAN; };
  const float col[12] = {(float)means[l * 3 + 0], (float)means[l * 3 + 1], (float)means[l * 3 + 2],
                         (float)(s[0] / na), (float)(s[1] / nt), (float)(s[2] / nd),
                         (float)sqrt(s[3] / na), (float)sqrt(s[4] / nt), (float)sqrt(s[5] / nd),
                         (float)med(0, N), (float)med(0, top), (float)med(top, N - top)};
  for (int r = 0; r < 12; ++r) data[((int64_t)l * rows + row0 + r) * steps + t] = col[r];
  for (int e = 0; e < n_extra; ++e) data[((int64_t)l * rows + row0 + 12 + e) * steps + t] = extra[l * n_extra + e];
}

// ---------------------------------------------------------------------------
// big-brain investors (coin_big_brain_lev :270-452, dice_big_brain_lev :741-932):
// configuration c = (roll, stop) sets each investor's leverage from its own
// value every step — lev = lev_factor (1 - L / v) with L the stop-loss floor
// stop * value_0, or, when roll > 0 and v > value_0, the rolling floor
// value_0 + roll (v - value_0) (coin_optimal_lev :240-267, dice_optimal_lev
// :704-738) — in the reference's arithmetic (coin f32; dice f64 values, see
// optimal_lev; this file compiles with FP contraction off).  Per step: the leverages' statistics (rows 12-23, then stop
// and roll), the value step v = v (1 + lev r), the new leverages, the values'
// statistics (rows 0-11).
// ---------------------------------------------------------------------------
struct BrainArgs {
  const uint8_t* cat;  // outcome codes [investors][ld]
  int64_t investors, ld;
  double ret[3];       // return per outcome code (f32 values for coin, f64 for dice)
  float value_0, lev_factor;
  const float* cfg;    // [n_cfg][5]: stop floor value_min, roll, initial leverage, roll > 0, stop level
  void* val;           // [n_cfg][investors] VT
  void* lev;           // [n_cfg][investors] VT
};

// coin (VT float, lev_exp.py:240-267): every quantity f32.  dice (VT double,
// :704-738, :741-932): outcomes are cast to float64, so values are f64; with
// roll 0 the leverage is f64 too (f32 lev_factor / value_min against the f64
// value), with roll > 0 dice_optimal_lev first casts the values to f32 and the
// leverage is all f32.
template <typename VT>
__device__ __forceinline__ VT optimal_lev(VT v, float v0, float vmin, float roll, bool rolling, float lf) {
  if (!rolling) return (VT)lf * ((VT)1 - (VT)vmin / v);
  const float vf = (float)v;
  const float loss = vf <= v0 ? vmin : v0 + roll * (vf - v0);
  return (VT)(lf * (1.f - loss / vf));
}

// t == 0: v = value_0 (1 + lev0 r[0]); else v = v (1 + lev r[t]); then lev = optimal(v)
template <typename VT>
__global__ void __launch_bounds__(kT) lev_brain_advance_kernel(BrainArgs a, int t) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int c = blockIdx.y;
  if (i >= a.investors) return;
  const float* k = a.cfg + 5 * c;
  const int o = a.cat[i * a.ld + t];
  const VT r = (VT)a.ret[o > 2 ? 2 : o];
  const int64_t j = (int64_t)c * a.investors + i;
  VT* val = static_cast<VT*>(a.val);
  VT* lev = static_cast<VT*>(a.lev);
  const VT v = t == 0 ? (VT)a.value_0 * ((VT)1 + (VT)k[2] * r) : val[j] * ((VT)1 + lev[j] * r);
  val[j] = v;
  lev[j] = optimal_lev<VT>(v, a.value_0, k[0], k[1], k[3] != 0.f, a.lev_factor);
}

template <typename VT = float>
size_t sort_temp_bytes(int64_t investors) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortKeysDescending(nullptr, bytes, (const VT*)nullptr, (VT*)nullptr, (int)investors);
  return (bytes + 255) & ~(size_t)255;
}

}  // namespace

extern "C" {

int64_t rlmd_lev_sorted_workspace_bytes(int64_t investors, int32_t n_lev) {
  if (investors <= 0 || investors > INT32_MAX || n_lev <= 0) return -1;
  const int64_t vals = 2 * (int64_t)n_lev * investors * 4;  // values + sorted copy
  const int64_t sums = (int64_t)n_lev * kChunks * 6 * 8 + (int64_t)n_lev * 3 * 8 + (int64_t)n_lev * 16 * 4;
  return ((vals + 255) & ~255ll) + ((sums + 255) & ~255ll) + (int64_t)sort_temp_bytes(investors);
}

static int sweep_sorted(int32_t kind, const void* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                        int64_t top, float value_0, const float* table_host, const float* levs_host, int32_t n_lev,
                        void* workspace, int64_t workspace_bytes, float* data_dev, float* data_T_dev, void* stream,
                        bool final_only) {
  RLMD_CHECK(kind == 0 || kind == 1, "kind: 0 categorical, 1 gbm");
  RLMD_CHECK(outcomes_dev && workspace && data_dev && levs_host, "null argument");
  RLMD_CHECK(investors > 0 && investors <= INT32_MAX && horizon >= (final_only ? 1 : 2) && ld >= horizon,
             "bad sizes");
  RLMD_CHECK(n_lev > 0 && n_lev <= 1024, "n_lev out of range");
  RLMD_CHECK(kind == 1 || table_host, "categorical sweep needs the factor table");
  const int64_t need = rlmd_lev_sorted_workspace_bytes(investors, n_lev);
  RLMD_CHECK(workspace_bytes >= need, "workspace smaller than rlmd_lev_sorted_workspace_bytes");
  const int64_t tp = top < investors ? (top > 0 ? top : 0) : investors;
  hipStream_t st = (hipStream_t)stream;
  unsigned char* w = static_cast<unsigned char*>(workspace);
  const int64_t vals = 2 * (int64_t)n_lev * investors * 4;
  float* val = reinterpret_cast<float*>(w);
  float* sorted = val + (int64_t)n_lev * investors;
  unsigned char* w2 = w + ((vals + 255) & ~255ll);
  double* part = reinterpret_cast<double*>(w2);
  double* means = part + (int64_t)n_lev * kChunks * 6;
  float* small = reinterpret_cast<float*>(means + (int64_t)n_lev * 3);  // levs [n_lev] | table [n_lev][3]
  const int64_t sums = (int64_t)n_lev * kChunks * 6 * 8 + (int64_t)n_lev * 3 * 8 + (int64_t)n_lev * 16 * 4;
  void* tmp = w2 + ((sums + 255) & ~255ll);
  size_t tmp_bytes = sort_temp_bytes(investors);
  RLMD_HIP(hipMemcpyAsync(small, levs_host, sizeof(float) * n_lev, hipMemcpyHostToDevice, st));
  if (kind == 0)
    RLMD_HIP(hipMemcpyAsync(small + n_lev, table_host, sizeof(float) * 3 * n_lev, hipMemcpyHostToDevice, st));
  SortedArgs a{};
  a.kind = kind;
  a.cat = static_cast<const uint8_t*>(outcomes_dev);
  a.gbm = static_cast<const float*>(outcomes_dev);
  a.investors = investors;
  a.ld = ld;
  a.n_lev = n_lev;
  a.levs = small;
  a.table = small + n_lev;
  a.val = val;
  const dim3 grid_adv((unsigned)((investors + kT - 1) / kT), (unsigned)n_lev);
  const int steps = final_only ? 1 : horizon - 1;
  for (int t = 0; t < horizon; ++t) {
    hipLaunchKernelGGL(lev_advance_kernel, grid_adv, dim3(kT), 0, st, a, t, value_0);
    RLMD_LAUNCH_CHECK();
    if (final_only ? t < horizon - 1 : t == 0) continue;
    for (int l = 0; l < n_lev; ++l) {
      RLMD_HIP(hipcub::DeviceRadixSort::SortKeysDescending(tmp, tmp_bytes, val + (int64_t)l * investors,
                                                           sorted + (int64_t)l * investors, (int)investors, 0, 32,
                                                           st));
    }
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(lev_sorted_sums_kernel<float>, dim3(kChunks, n_lev), dim3(kT), 0, st, sorted, investors, tp,
                         means, pass, part);
      RLMD_LAUNCH_CHECK();
      hipLaunchKernelGGL(lev_sorted_fold_kernel<float>, dim3((n_lev + 63) / 64), dim3(64), 0, st, sorted, investors,
                         tp, n_lev, part, pass, means, small, 1, data_dev, 13, 0, steps, final_only ? 0 : t - 1);
      RLMD_LAUNCH_CHECK();
    }
  }
  if (data_T_dev)
    RLMD_HIP(hipMemcpyAsync(data_T_dev, val, sizeof(float) * n_lev * investors, hipMemcpyDeviceToDevice, st));
  return 0;
}

int rlmd_lev_sweep_sorted(int32_t kind, const void* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                          int64_t top, float value_0, const float* table_host, const float* levs_host, int32_t n_lev,
                          void* workspace, int64_t workspace_bytes, float* data_dev, float* data_T_dev,
                          void* stream) {
  return sweep_sorted(kind, outcomes_dev, investors, horizon, ld, top, value_0, table_host, levs_host, n_lev,
                      workspace, workspace_bytes, data_dev, data_T_dev, stream, false);
}

int rlmd_lev_final_sorted(int32_t kind, const void* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                          int64_t top, float value_0, const float* table_host, const float* levs_host, int32_t n_lev,
                          void* workspace, int64_t workspace_bytes, float* stats_dev, float* values_dev,
                          void* stream) {
  return sweep_sorted(kind, outcomes_dev, investors, horizon, ld, top, value_0, table_host, levs_host, n_lev,
                      workspace, workspace_bytes, stats_dev, values_dev, stream, true);
}

int64_t rlmd_lev_brain_workspace_bytes(int64_t investors, int32_t n_cfg) {
  if (investors <= 0 || investors > INT32_MAX || n_cfg <= 0) return -1;
  const int64_t vals = 3 * (int64_t)n_cfg * investors * 8;  // values, leverages, sorted copy (f64 at most)
  const int64_t sums = (int64_t)n_cfg * kChunks * 6 * 8 + (int64_t)n_cfg * 3 * 8 + (int64_t)n_cfg * 8 * 4;
  const int64_t tmp = (int64_t)std::max(sort_temp_bytes<float>(investors), sort_temp_bytes<double>(investors));
  return ((vals + 255) & ~255ll) + ((sums + 255) & ~255ll) + tmp;
}

}  // extern "C"

template <typename VT>
static int lev_brain(const uint8_t* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld, int64_t top,
                     float value_0, const double* rets3, float lev_factor, const float* cfg_host, int32_t n_cfg,
                     void* workspace, float* data_dev, hipStream_t st) {
  const int64_t tp = top < investors ? (top > 0 ? top : 0) : investors;
  unsigned char* w = static_cast<unsigned char*>(workspace);
  const int64_t NC = (int64_t)n_cfg * investors;
  VT* val = reinterpret_cast<VT*>(w);
  VT* lev = val + NC;
  VT* sorted = lev + NC;
  unsigned char* w2 = w + ((3 * NC * 8 + 255) & ~255ll);
  double* part = reinterpret_cast<double*>(w2);
  double* means = part + (int64_t)n_cfg * kChunks * 6;
  float* cfg = reinterpret_cast<float*>(means + (int64_t)n_cfg * 3);  // [n_cfg][5] | extra [n_cfg][2]
  float* extra = cfg + 5 * n_cfg;
  const int64_t sums = (int64_t)n_cfg * kChunks * 6 * 8 + (int64_t)n_cfg * 3 * 8 + (int64_t)n_cfg * 8 * 4;
  void* tmp = w2 + ((sums + 255) & ~255ll);
  size_t tmp_bytes = sort_temp_bytes<VT>(investors);
  std::vector<float> ex(2 * (size_t)n_cfg);
  for (int c = 0; c < n_cfg; ++c) {  // rows 24 / 25: stop level and roll
    ex[2 * c] = cfg_host[5 * c + 4];
    ex[2 * c + 1] = cfg_host[5 * c + 1];
  }
  RLMD_HIP(hipMemcpyAsync(cfg, cfg_host, sizeof(float) * 5 * n_cfg, hipMemcpyHostToDevice, st));
  RLMD_HIP(hipMemcpyAsync(extra, ex.data(), sizeof(float) * 2 * n_cfg, hipMemcpyHostToDevice, st));
  BrainArgs a{};
  a.cat = outcomes_dev;
  a.investors = investors;
  a.ld = ld;
  for (int q = 0; q < 3; ++q) a.ret[q] = rets3[q];
  a.value_0 = value_0;
  a.lev_factor = lev_factor;
  a.cfg = cfg;
  a.val = val;
  a.lev = lev;
  const dim3 grid_adv((unsigned)((investors + kT - 1) / kT), (unsigned)n_cfg);
  const int steps = horizon - 1;
  auto stats = [&](const VT* src, int row0, const float* ext, int n_ext, int t) -> int {
    for (int c = 0; c < n_cfg; ++c)
      RLMD_HIP(hipcub::DeviceRadixSort::SortKeysDescending(tmp, tmp_bytes, src + (int64_t)c * investors,
                                                           sorted + (int64_t)c * investors, (int)investors, 0,
                                                           (int)(8 * sizeof(VT)), st));
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(lev_sorted_sums_kernel<VT>, dim3(kChunks, n_cfg), dim3(kT), 0, st, sorted, investors, tp,
                         means, pass, part);
      RLMD_LAUNCH_CHECK();
      hipLaunchKernelGGL(lev_sorted_fold_kernel<VT>, dim3((n_cfg + 63) / 64), dim3(64), 0, st, sorted, investors,
                         tp, n_cfg, part, pass, means, ext, n_ext, data_dev, 26, row0, steps, t);
      RLMD_LAUNCH_CHECK();
    }
    return 0;
  };
  hipLaunchKernelGGL(lev_brain_advance_kernel<VT>, grid_adv, dim3(kT), 0, st, a, 0);
  RLMD_LAUNCH_CHECK();
  for (int t = 0; t < steps; ++t) {
    RLMD_TRY_INT(stats(lev, 12, extra, 2, t));
    hipLaunchKernelGGL(lev_brain_advance_kernel<VT>, grid_adv, dim3(kT), 0, st, a, t + 1);
    RLMD_LAUNCH_CHECK();
    RLMD_TRY_INT(stats(val, 0, nullptr, 0, t));
  }
  return 0;
}

extern "C" {

int rlmd_lev_brain(int32_t f64, const uint8_t* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                   int64_t top, float value_0, const double* rets_host3, float lev_factor, const float* cfg_host,
                   int32_t n_cfg, void* workspace, int64_t workspace_bytes, float* data_dev, void* stream) {
  RLMD_CHECK(outcomes_dev && rets_host3 && cfg_host && workspace && data_dev, "null argument");
  RLMD_CHECK(investors > 0 && investors <= INT32_MAX && horizon >= 2 && ld >= horizon, "bad sizes");
  RLMD_CHECK(n_cfg > 0 && n_cfg <= 4096, "n_cfg out of range");
  RLMD_CHECK(workspace_bytes >= rlmd_lev_brain_workspace_bytes(investors, n_cfg),
             "workspace smaller than rlmd_lev_brain_workspace_bytes");
  if (f64)
    return lev_brain<double>(outcomes_dev, investors, horizon, ld, top, value_0, rets_host3, lev_factor, cfg_host,
                             n_cfg, workspace, data_dev, (hipStream_t)stream);
  return lev_brain<float>(outcomes_dev, investors, horizon, ld, top, value_0, rets_host3, lev_factor, cfg_host, n_cfg,
                          workspace, data_dev, (hipStream_t)stream);
}

}  // extern "C"
