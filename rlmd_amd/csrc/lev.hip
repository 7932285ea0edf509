// lev.hip — fixed-leverage coin-flip Monte-Carlo sweep on the device (gfx950).
//
// Replaces lev/lev_exp.py:128-237 (coin_smart_lev), run by lev/coin_flip.py:
// 160-189 at 1e6 investors x 3e3 steps over 10 leverages: for each leverage
// and each step, every investor's value is multiplied by 1 + l*up_r (outcome 1)
// or 1 + l*down_r, the values are SORTED and 12 summary statistics of all / the
// top `top` / the rest are stored: 3e4 sorts of 1e6 floats.
//
// Here no sort happens.  After n outcomes an investor's value depends only on
// its up-count k (v(k) = v0 gu^k gd^(n-k), monotone in k), so the sorted order
// at step n is the order of the up-count histogram H[n-1][k], and every
// statistic is a weighted sum over <= n+1 bins.  Three kernels:
//   lev_prefix_kernel   one thread per investor streams its row once: the
//                       up-count before each 64-step chunk (u16 [chunks][I]),
//                       and the final values data_T as the reference's
//                       sequential float32 products (bit-exact);
//   lev_hist_kernel     (investor block, chunk): LDS histogram of the 64 steps'
//                       up-counts over the block's k window, flushed with
//                       atomics into H [T][T+1] (global atomics when the window
//                       exceeds LDS);
//   lev_stats_kernel    (step, leverage): rank-ordered bins, block scan of the
//                       counts, f32 bin values, sums in double, medians by rank.
// The outcome matrix is u8 [I][ld] (the reference holds a float tensor of 0/1:
// 4x the bytes); HBM traffic is ~2 passes over it plus H.
#include <math.h>

#include <algorithm>

#include "rlmd_common.h"
#include "rlmd_internal.h"

namespace {

constexpr int kChunk = 64;        // steps per histogram chunk
constexpr int kHistThreads = 1024;  // lev_hist_kernel workgroup: 16 waves share one LDS histogram
constexpr int kInvPerThread = 4;    // investors per thread in lev_hist_kernel
constexpr int kHistLds = 24576;    // u32 LDS bins per hist workgroup (96 KB)
constexpr int kMaxLev = 32;

struct LevArgs {
  const uint8_t* outcomes;
  int64_t ld;
  int32_t investors, horizon, top, n_lev;
  float value_0;
  float gu[kMaxLev], gd[kMaxLev], lev[kMaxLev];
  uint16_t* pre;   // [chunks][investors]
  uint32_t* hist;  // [horizon][horizon + 1]
  float* data;     // [n_lev][13][horizon - 1]
  float* data_T;   // [n_lev][investors] (nullable)
};

// the 64 outcomes of one row chunk as four 16-byte words (rows padded to 64
// steps); walked with compile-time indices so nothing spills to scratch
struct Chunk64 {
  uint32_t w[16];
  __device__ __forceinline__ void load(const uint8_t* row, int t0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(row + t0 + 16 * q);
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  }
  __device__ __forceinline__ int up(int b) const { return ((w[b >> 2] >> (8 * (b & 3))) & 0xff) == 1; }
};

template <int NL>
__global__ void __launch_bounds__(256) lev_prefix_kernel(LevArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.investors) return;
  const uint8_t* row = a.outcomes + (int64_t)i * a.ld;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2 val[NL > 0 ? NL / 2 : 1], gu[NL > 0 ? NL / 2 : 1], gd[NL > 0 ? NL / 2 : 1];
#pragma unroll
  for (int l = 0; l < (NL > 0 ? NL / 2 : 1); ++l) {
    val[l] = f32x2{a.value_0, a.value_0};
    gu[l] = f32x2{a.gu[2 * l], a.gu[2 * l + 1]};
    gd[l] = f32x2{a.gd[2 * l], a.gd[2 * l + 1]};
  }
  int k = 0;
  const int chunks = (a.horizon + kChunk - 1) / kChunk;
  Chunk64 nx;
  nx.load(row, 0);
  for (int c = 0; c < chunks; ++c) {
    a.pre[(int64_t)c * a.investors + i] = (uint16_t)k;
    const Chunk64 ch = nx;
    if (c + 1 < chunks) nx.load(row, (c + 1) * kChunk);  // next chunk in flight while this one is walked
    const int tn = min(kChunk, a.horizon - c * kChunk);
#pragma unroll
    for (int tt = 0; tt < kChunk; ++tt) {
      if (tt < tn) {
        const int o = ch.up(tt);
        k += o;
        if constexpr (NL > 0) {
          // initial = value_0 * g[:, 0]; value_t = initial * g[:, t + 1]
          // (lev_exp.py:170-176): one f32 product per step, two leverages per
          // packed multiply (v_pk_mul_f32)
#pragma unroll
          for (int l = 0; l < NL / 2; ++l) val[l] *= o ? gu[l] : gd[l];
        }
      }
    }
  }
  if constexpr (NL > 0) {
#pragma unroll
    for (int l = 0; l < NL; ++l)
      if (l < a.n_lev) a.data_T[(int64_t)l * a.investors + i] = val[l >> 1][l & 1];
  }
}

__global__ void __launch_bounds__(kHistThreads) lev_hist_kernel(LevArgs a) {
  __shared__ uint32_t h[kHistLds];
  __shared__ int s_lo, s_hi;
  const int c = blockIdx.y, t0 = c * kChunk, tn = min(kChunk, a.horizon - t0);
  const int base = blockIdx.x * kHistThreads * kInvPerThread;
  const int H1 = a.horizon + 1;
  int st[kInvPerThread], lo = 1 << 30, hi = -1;
#pragma unroll
  for (int j = 0; j < kInvPerThread; ++j) {
    const int i = base + j * kHistThreads + threadIdx.x;
    st[j] = i < a.investors ? a.pre[(int64_t)c * a.investors + i] : -1;
    if (st[j] >= 0) {
      lo = min(lo, st[j]);
      hi = max(hi, st[j]);
    }
  }
  if (threadIdx.x == 0) {
    s_lo = 1 << 30;
    s_hi = -1;
  }
  __syncthreads();
  atomicMin(&s_lo, lo);
  atomicMax(&s_hi, hi);
  __syncthreads();
  const int klo = s_lo, W = s_hi - s_lo + kChunk + 1;
  if (s_hi < 0) return;  // uniform: no investors in this block
  const bool in_lds = (int64_t)W * tn <= kHistLds;
  if (in_lds) {
    for (int e = threadIdx.x; e < W * tn; e += kHistThreads) h[e] = 0;
    __syncthreads();
  }
#pragma unroll 1
  for (int j = 0; j < kInvPerThread; ++j) {
    if (st[j] < 0) continue;
    const int i = base + j * kHistThreads + threadIdx.x;
    Chunk64 ch;
    ch.load(a.outcomes + (int64_t)i * a.ld, t0);
    int k = st[j];
#pragma unroll
    for (int tt = 0; tt < kChunk; ++tt) {
      if (tt < tn) {
        k += ch.up(tt);
        if (in_lds) atomicAdd(&h[tt * W + (k - klo)], 1u);
        else atomicAdd(&a.hist[(int64_t)(t0 + tt) * H1 + k], 1u);
      }
    }
  }
  if (!in_lds) return;
  __syncthreads();
  for (int e = threadIdx.x; e < W * tn; e += kHistThreads) {
    const uint32_t v = h[e];
    if (v) {
      const int tt = e / W, k = klo + e - tt * W;
      atomicAdd(&a.hist[(int64_t)(t0 + tt) * H1 + k], v);
    }
  }
}

__device__ double block_sum(double v, double* red) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += red[q];
  return s;
}

// f32 value of a bin: v0 * gu^k * gd^m, rounded once.  Formed in log space so
// the two powers cannot overflow / underflow independently (inf * 0 = NaN for a
// populated bin whose true value is finite); a zero factor with a positive
// exponent gives 0, as the reference's sequential products do; a value past
// the f32 range rounds to inf, as they do too.
__device__ __forceinline__ float bin_value(float v0, float gu, float gd, int k, int m) {
  if (v0 == 0.f || (k > 0 && gu == 0.f) || (m > 0 && gd == 0.f)) return 0.f;
  double lg = log((double)v0);
  if (k > 0) lg += (double)k * log((double)gu);
  if (m > 0) lg += (double)m * log((double)gd);
  return (float)exp(lg);
}

// one workgroup per (step t, leverage): the table column data[lev][:, t]
__global__ void __launch_bounds__(256) lev_stats_kernel(LevArgs a) {
  extern __shared__ unsigned char smem[];
  const int t = blockIdx.x, l = blockIdx.y;
  const int n = t + 2;  // outcomes behind the reference's value_t (lev_exp.py:172-176)
  const int nb = n + 1;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);  // rank order (descending value)
  uint32_t* cum = cnt + nb;                           // exclusive prefix
  float* val = reinterpret_cast<float*>(cum + nb);
  __shared__ uint32_t part[256];
  __shared__ double red[4];
  const float gu = a.gu[l], gd = a.gd[l];
  const bool up_first = gu >= gd;
  const uint32_t* hrow = a.hist + (int64_t)(n - 1) * (a.horizon + 1);
  for (int r = threadIdx.x; r < nb; r += 256) {
    const int k = up_first ? n - r : r;
    cnt[r] = hrow[k];
    val[r] = bin_value(a.value_0, gu, gd, k, n - k);
  }
  __syncthreads();
  const int per = (nb + 255) / 256, r0 = threadIdx.x * per, r1 = min(nb, r0 + per);
  uint32_t s = 0;
  for (int r = r0; r < r1; ++r) s += cnt[r];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int q = 0; q < 256; ++q) {
      const uint32_t v = part[q];
      part[q] = acc;
      acc += v;
    }
  }
  __syncthreads();
  s = part[threadIdx.x];
  for (int r = r0; r < r1; ++r) {
    cum[r] = s;
    s += cnt[r];
  }
  __syncthreads();
  const uint32_t N = (uint32_t)a.investors, top = min((uint32_t)a.top, N), nadj = N - top;
  auto split = [&](int r, uint32_t& ct, uint32_t& ca) {
    const uint32_t c0 = cum[r], c = cnt[r];
    ct = c0 >= top ? 0u : min(c, top - c0);
    ca = c - ct;
  };
  double s_all = 0, s_top = 0, s_adj = 0;
  for (int r = threadIdx.x; r < nb; r += 256) {
    uint32_t ct, ca;
    split(r, ct, ca);
    if (!cnt[r]) continue;  // empty bins may hold inf values (0 * inf)
    const double v = val[r];
    s_all += cnt[r] * v;
    if (ct) s_top += ct * v;
    if (ca) s_adj += ca * v;
  }
  const double m_all = block_sum(s_all, red) / N;
  const double m_top = block_sum(s_top, red) / top;
  const double m_adj = block_sum(s_adj, red) / nadj;
  double d_all = 0, d_top = 0, d_adj = 0, q_all = 0, q_top = 0, q_adj = 0;
  for (int r = threadIdx.x; r < nb; r += 256) {
    uint32_t ct, ca;
    split(r, ct, ca);
    if (!cnt[r]) continue;
    const double v = val[r];
    const double ea = v - m_all, et = v - m_top, ed = v - m_adj;
    d_all += cnt[r] * fabs(ea);
    q_all += cnt[r] * ea * ea;
    if (ct) {
      d_top += ct * fabs(et);
      q_top += ct * et * et;
    }
    if (ca) {
      d_adj += ca * fabs(ed);
      q_adj += ca * ed * ed;
    }
  }
  float* col = a.data + (int64_t)l * 13 * (a.horizon - 1) + t;
  const int64_t rs = a.horizon - 1;
  const double mad_all = block_sum(d_all, red) / N, std_all = sqrt(block_sum(q_all, red) / N);
  const double mad_top = block_sum(d_top, red) / top, std_top = sqrt(block_sum(q_top, red) / top);
  const double mad_adj = block_sum(d_adj, red) / nadj, std_adj = sqrt(block_sum(q_adj, red) / nadj);
  // lower medians (torch.median): ascending index (G-1)/2 of a group starting at
  // descending rank g0 -> rank g0 + G-1 - (G-1)/2
  const uint32_t q_med[3] = {N - 1 - (N - 1) / 2, top ? top - 1 - (top - 1) / 2 : 0,
                             nadj ? top + nadj - 1 - (nadj - 1) / 2 : 0};
  for (int r = threadIdx.x; r < nb; r += 256) {
    const uint32_t c0 = cum[r], c = cnt[r];
#pragma unroll
    for (int g = 0; g < 3; ++g)
      if (c && q_med[g] >= c0 && q_med[g] < c0 + c && (g == 0 || (g == 1 ? top : nadj) > 0))
        col[(9 + g) * rs] = val[r];
  }
  if (threadIdx.x == 0) {
    col[0 * rs] = (float)m_all;
    col[1 * rs] = (float)m_top;
    col[2 * rs] = (float)m_adj;
    col[3 * rs] = (float)mad_all;
    col[4 * rs] = (float)mad_top;
    col[5 * rs] = (float)mad_adj;
    col[6 * rs] = (float)std_all;
    col[7 * rs] = (float)std_top;
    col[8 * rs] = (float)std_adj;
    if (!top) col[10 * rs] = NAN;
    if (!nadj) col[11 * rs] = NAN;
    col[12 * rs] = a.lev[l];
  }
}

int64_t chunks_of(int horizon) { return (horizon + kChunk - 1) / kChunk; }

}  // namespace

extern "C" {

int64_t rlmd_lev_workspace_bytes(int64_t investors, int32_t horizon) {
  if (investors < 0 || horizon < 1) return -1;
  const int64_t pre = (chunks_of(horizon) * investors * 2 + 255) / 256 * 256;
  return pre + (int64_t)horizon * (horizon + 1) * 4;
}

int rlmd_lev_coin_sweep(const uint8_t* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld, int64_t top,
                        float value_0, float up_r, float down_r, const float* levs_host, int32_t n_lev,
                        void* workspace_dev, int64_t workspace_bytes, float* data_dev, float* data_T_dev,
                        void* stream) {
  RLMD_CHECK(outcomes_dev && levs_host && workspace_dev && data_dev, "null argument");
  RLMD_CHECK(investors >= 1 && investors < (1ll << 31) && horizon >= 2 && horizon <= 65535, "bad shape");
  RLMD_CHECK(workspace_bytes >= rlmd_lev_workspace_bytes(investors, horizon),
             "workspace smaller than rlmd_lev_workspace_bytes(investors, horizon)");
  RLMD_CHECK(ld >= horizon && ld % 16 == 0 && ((uintptr_t)outcomes_dev & 15) == 0,
             "outcome rows: 16-byte aligned, leading dimension a multiple of 16 and >= horizon");
  RLMD_CHECK(ld >= chunks_of(horizon) * kChunk, "outcome rows padded to a multiple of 64 steps");
  RLMD_CHECK(n_lev >= 1 && n_lev <= kMaxLev && top >= 0, "bad leverage count / top");
  const int64_t stats_lds = (int64_t)(horizon + 2) * 12;
  RLMD_CHECK(stats_lds <= 64 * 1024, "horizon too long for the stats workgroup's LDS (<= 5459)");
  hipStream_t s = (hipStream_t)stream;
  LevArgs a{};
  a.outcomes = outcomes_dev;
  a.ld = ld;
  a.investors = (int32_t)investors;
  a.horizon = horizon;
  a.top = (int32_t)std::min<int64_t>(top, investors);
  a.n_lev = n_lev;
  a.value_0 = value_0;
  // lev_exp.py:163-167: the range negated when -down_r > up_r; 1 + lev * r in f32
  for (int l = 0; l < n_lev; ++l) {
    const float lev = -down_r > up_r ? -levs_host[l] : levs_host[l];
    a.lev[l] = lev;
    a.gu[l] = 1.0f + lev * up_r;
    a.gd[l] = 1.0f + lev * down_r;
    RLMD_CHECK(a.gu[l] >= 0.f && a.gd[l] >= 0.f,
               "leverage outside the supported domain: 1 + lev*up_r and 1 + lev*down_r must be >= 0 "
               "(a negative factor flips the value order; see rlmd_abi.h)");
  }
  const int64_t pre_bytes = (chunks_of(horizon) * investors * 2 + 255) / 256 * 256;
  a.pre = static_cast<uint16_t*>(workspace_dev);
  a.hist = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace_dev) + pre_bytes);
  a.data = data_dev;
  a.data_T = data_T_dev;
  RLMD_HIP(hipMemsetAsync(a.hist, 0, (size_t)horizon * (horizon + 1) * 4, s));
  const dim3 gi((unsigned)((investors + 255) / 256));
#define RLMD_LEV_PRE(NL) \
  hipLaunchKernelGGL(lev_prefix_kernel<NL>, gi, dim3(256), 0, s, a)
  if (!data_T_dev) RLMD_LEV_PRE(0);
  else if (n_lev <= 4) RLMD_LEV_PRE(4);
  else if (n_lev <= 10) RLMD_LEV_PRE(10);
  else if (n_lev <= 16) RLMD_LEV_PRE(16);
  else RLMD_LEV_PRE(32);
#undef RLMD_LEV_PRE
  RLMD_LAUNCH_CHECK();
  const unsigned ib = (unsigned)((investors + kHistThreads * kInvPerThread - 1) / (kHistThreads * kInvPerThread));
  hipLaunchKernelGGL(lev_hist_kernel, dim3(ib, (unsigned)chunks_of(horizon)), dim3(kHistThreads), 0, s, a);
  RLMD_LAUNCH_CHECK();
  hipLaunchKernelGGL(lev_stats_kernel, dim3((unsigned)(horizon - 1), (unsigned)n_lev), dim3(256),
                     (size_t)stats_lds, s, a);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
