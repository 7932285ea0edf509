// lev_sort.hip — fixed-leverage sweeps whose order statistics need the values
// themselves (gfx950).
//
// Replaces dice_smart_lev (lev/lev_exp.py:586-705), gbm_smart_lev (:1008-1119)
// and dice_sh_smart_lev (:1209-1332) — and, statistics of the final values only,
// the *_fixed_final_lev family (:56-127, :508-585, :935-1007, :1121-1208) — and
// the big-brain investors (coin_big_brain_lev :270-452, dice_big_brain_lev
// :741-932): for every leverage l each investor's value is multiplied step by
// step by its gamble factor (float32, as the reference's torch tensors), and
// after each step t >= 1 the reference SORTS the values descending: the first
// `top` form the top group, the rest the adjusted group, and the table column
// [mean, mean_top, mean_adj, mad x3, std x3, median x3, lev] is stored (std
// unbiased=False, median = the lower middle element, torch.median).
//
// Unlike the coin flip (lev.hip: the value is monotone in one up-count, so
// histograms of counts replace the sorts) a die's value depends on two counts
// and a GBM path's on a continuous sum.  But the column needs only FOUR order
// statistics of each step's values — the top group's boundary (descending rank
// top - 1) and the three lower medians — plus group sums, and group membership
// follows from the boundary value vk alone (v > vk: top; v < vk: adjusted; the
// top - #(v > vk) copies of vk that the sort puts in the top group are added
// analytically).  So no sort runs: the four ranks are found together by an
// 11-bit-digit radix SELECT over order-preserving integer keys (3 passes for
// f32, 6 for f64), each pass one streaming read:
//   lev_window_kernel    outcome steps [t0, t0 + 32) transposed to [step][investor]
//                        once per 32 steps (the per-step column read coalesces)
//   lev_advance_kernel   values *= factor(outcome[t][i]) for every (lev, investor),
//                        fused with the select's first digit histogram
//   sel_hist_kernel      later digits: LDS histograms of the keys whose higher
//                        bits match a target's prefix (one per distinct prefix)
//   sel_scan_kernel      per (array, target): the digit bin holding the target
//                        rank (wave scan of the histogram), the next prefix
//   sel_sums_kernel      group sums in f64 (pass 0), then |v - mean| and
//                        (v - mean)^2 (pass 1); fixed chunk order: deterministic
//   sel_fold_kernel      per array: fold the chunks, write the column
#include <hip/hip_runtime.h>
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

constexpr int kChunks = 128;    // partial-sum chunks per array
constexpr int kT = 256;
constexpr int kSelB = 11;       // radix-select digit bits
constexpr int kSelBins = 1 << kSelB;
constexpr int kSelBlocks = 128;  // histogram / advance workgroups per array
constexpr int kW = 32;          // outcome steps per transposed window

// ---- order-preserving integer keys of f32 / f64 (ascending) ----------------
__device__ __forceinline__ uint32_t okey(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ uint64_t okey(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}
__device__ __forceinline__ float kval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ double kval(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & ~(1ull << 63)) : ~k));
}
template <typename VT>
struct KeyT {
  typedef uint32_t K;
};
template <>
struct KeyT<double> {
  typedef uint64_t K;
};

// digit of pass p (most significant first): bits [shift, shift + width)
__host__ __device__ inline void sel_digit(int bits, int p, int& shift, int& width) {
  const int hi = bits - kSelB * p;
  width = hi < kSelB ? hi : kSelB;
  shift = hi - width;
}
inline int sel_passes(int bits) { return (bits + kSelB - 1) / kSelB; }

// per (array, target q): q 0 the top group's boundary (ascending rank N - top),
// 1 the median of all ((N - 1) / 2), 2 of the top group (N - top + (top - 1) / 2),
// 3 of the adjusted group ((N - top - 1) / 2).  prefix: the key bits decided so
// far; rank: the rank left inside that prefix; src: the target whose histogram
// serves this one in the next pass (equal prefixes share one).
struct SelState {
  unsigned long long prefix;
  long long rank;
  int valid, src;
};

// arrays of N values are stored with a stride of pad4(N) (16-B aligned rows)
__host__ __device__ inline int64_t pad4(int64_t n) { return (n + 3) & ~3ll; }

// chunk c of n_chunks over [0, N), chunk starts at multiples of 4
__device__ __forceinline__ void chunk_range(int64_t N, int c, int n_chunks, int64_t& b0, int64_t& b1) {
  const int64_t per = pad4((N + n_chunks - 1) / n_chunks);
  b0 = (int64_t)c * per;
  b1 = b0 + per < N ? b0 + per : N;
  if (b0 > N) b0 = N;
}

// f(v) for every value of [b0, b1) (b0 a multiple of 4), 16-B loads, two in
// flight per thread; loads past b1 stay inside the padded row and are masked
template <typename VT, typename F>
__device__ __forceinline__ void for_vals(const VT* v, int64_t b0, int64_t b1, F f) {
  constexpr int V = 16 / sizeof(VT);
  typedef VT vec_t __attribute__((ext_vector_type(V)));
  const int64_t step = (int64_t)V * blockDim.x;
  for (int64_t i = b0 + (int64_t)V * threadIdx.x; i < b1; i += 2 * step) {
    const vec_t x0 = *reinterpret_cast<const vec_t*>(v + i);
    const bool two = i + step < b1;
    vec_t x1;
    if (two) x1 = *reinterpret_cast<const vec_t*>(v + i + step);
#pragma unroll
    for (int e = 0; e < V; ++e)
      if (i + e < b1) f(x0[e]);
    if (two) {
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (i + step + e < b1) f(x1[e]);
    }
  }
}

// LDS histogram slots flushed into the array's global slots (non-zero bins only)
__device__ __forceinline__ void flush_hist(const unsigned* h, int n, unsigned* g) {
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    if (h[i]) atomicAdd(&g[i], h[i]);
}

// pass p >= 1: histogram of digit p over the keys matching a target's prefix
// On the last pass also the block's sums [all values, values whose key lies
// above the boundary target's bucket, their count] (part2, fixed order)
template <typename VT>
__global__ void __launch_bounds__(kT) sel_hist_kernel(const VT* vals, int64_t N, int p, int last, const SelState* sel,
                                                      unsigned* hist, double* part2) {
  typedef typename KeyT<VT>::K K;
  constexpr int bits = 8 * sizeof(VT);
  int shift, width;
  sel_digit(bits, p, shift, width);
  const int l = blockIdx.y;
  __shared__ unsigned h[4 * kSelBins];
  K pre[4];
  bool on[4];
  const bool top_on = sel[l * 4].valid != 0;
  const K pre0 = (K)sel[l * 4].prefix;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const SelState s = sel[l * 4 + q];
    on[q] = s.valid && s.src == q;
    pre[q] = (K)s.prefix;
    if (on[q])
      for (int i = threadIdx.x; i < kSelBins; i += kT) h[q * kSelBins + i] = 0;
  }
  __syncthreads();
  int64_t b0, b1;
  chunk_range(N, blockIdx.x, gridDim.x, b0, b1);
  const K mask = ((K)1 << width) - 1;
  double sa = 0.0, sab = 0.0, cab = 0.0;
  for_vals(vals + (int64_t)l * pad4(N), b0, b1, [&](VT x) {
    const K key = okey(x);
    const unsigned d = (unsigned)((key >> shift) & mask);
    const K hi = key >> (shift + width);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (on[q] && hi == pre[q]) atomicAdd(&h[q * kSelBins + d], 1u);
    if (last) {
      sa += (double)x;
      if (top_on && hi > pre0) {
        sab += (double)x;
        cab += 1.0;
      }
    }
  });
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (on[q]) flush_hist(h + q * kSelBins, kSelBins, hist + ((int64_t)l * 4 + q) * kSelBins);
  if (!last) return;
  __shared__ double red[3][kT];
  red[0][threadIdx.x] = sa;
  red[1][threadIdx.x] = sab;
  red[2][threadIdx.x] = cab;
  __syncthreads();
  for (int hh = kT / 2; hh > 0; hh >>= 1) {
    if ((int)threadIdx.x < hh)
      for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + hh];
    __syncthreads();
  }
  if ((int)threadIdx.x < 3) part2[((int64_t)l * gridDim.x + blockIdx.x) * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// per array (one workgroup, wave q = target q): the bin of digit p that holds
// the target's rank; then the array's histogram slots are zeroed for the next
// pass and equal prefixes are pointed at one histogram
// On the last pass wave 0 also forms the groups' means from the hist blocks'
// sums and the boundary bucket's histogram (every bin of the last digit is one
// value): means[l][0..4] = mean all, top, adjusted, and the boundary value's
// copies in the top and the adjusted group.
template <typename VT>
__global__ void __launch_bounds__(256) sel_scan_kernel(int p, int last, int64_t N, int64_t top, SelState* sel,
                                                       unsigned* hist, const double* part2, double* means) {
  typedef typename KeyT<VT>::K K;
  constexpr int bits = 8 * sizeof(VT);
  const int l = blockIdx.x, q = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int shift, width;
  sel_digit(bits, p, shift, width);
  const int per = (1 << width) / 64;
  SelState s = sel[l * 4 + q];
  if (p == 0) {
    const int64_t tp = top;
    const int64_t ranks[4] = {N - tp, (N - 1) / 2, N - tp + (tp - 1) / 2, (N - tp - 1) / 2};
    const bool valid[4] = {tp >= 1, N >= 1, tp >= 1, N - tp >= 1};
    s.prefix = 0;
    s.rank = ranks[q];
    s.valid = valid[q] ? 1 : 0;
    s.src = q;
  }
  unsigned* base = hist + (int64_t)l * 4 * kSelBins;
  double gsum = 0.0, gcnt = 0.0, ceq = 0.0;  // last pass, wave 0: the boundary bucket above / at the boundary
  if (s.valid) {
    const unsigned* h = base + (p == 0 ? 0 : s.src) * kSelBins;
    unsigned cb[kSelBins / 64];
#pragma unroll
    for (int j = 0; j < kSelBins / 64; ++j) cb[j] = j < per ? h[lane * per + j] : 0u;
    unsigned long long mine = 0;
#pragma unroll
    for (int j = 0; j < kSelBins / 64; ++j) mine += cb[j];
    unsigned long long incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    const unsigned long long m = __ballot(incl > (unsigned long long)s.rank);
    if (m == 0) {
      s.valid = 0;  // (the counts do not reach the rank: never for consistent input)
    } else {
      const int L = __ffsll(m) - 1;
      int bin = 0;
      unsigned long long below = 0;
      if (lane == L) {
        unsigned long long cum = incl - mine;
        bool found = false;
#pragma unroll
        for (int j = 0; j < kSelBins / 64; ++j) {
          const unsigned c = cb[j];
          if (!found && j < per && cum + c > (unsigned long long)s.rank) {
            bin = lane * per + j;
            below = cum;
            found = true;
          }
          cum += c;
        }
      }
      bin = __shfl(bin, L, 64);
      below = __shfl(below, L, 64);
      if (last && q == 0) {
#pragma unroll
        for (int j = 0; j < kSelBins / 64; ++j) {
          const int bj = lane * per + j;
          if (j < per && bj > bin) {
            gsum += (double)cb[j] * (double)kval((K)((s.prefix << width) | (unsigned long long)bj));
            gcnt += (double)cb[j];
          }
          if (j < per && bj == bin) ceq = (double)cb[j];
        }
      }
      s.prefix = (s.prefix << width) | (unsigned long long)bin;
      s.rank -= (long long)below;
    }
  }
  if (last && q == 0) {
    double sa = 0.0, sab = gsum, cab = gcnt;
    for (int b = lane; b < kSelBlocks; b += 64) {
      sa += part2[((int64_t)l * kSelBlocks + b) * 3];
      sab += part2[((int64_t)l * kSelBlocks + b) * 3 + 1];
      cab += part2[((int64_t)l * kSelBlocks + b) * 3 + 2];
    }
    for (int o = 32; o > 0; o >>= 1) {
      sa += __shfl_xor(sa, o, 64);
      sab += __shfl_xor(sab, o, 64);
      cab += __shfl_xor(cab, o, 64);
      ceq += __shfl_xor(ceq, o, 64);
    }
    if (lane == 0) {
      const bool has_top = s.valid != 0;
      const double vk = has_top ? (double)kval((K)s.prefix) : 0.0;
      const double nt = (double)top;
      const double tie_top = has_top ? nt - cab : 0.0;
      const double sum_top = has_top ? sab + tie_top * vk : 0.0;
      double* m = means + l * 8;
      m[0] = sa / (double)N;
      m[1] = sum_top / nt;
      m[2] = N > top ? (sa - sum_top) / (double)(N - top) : NAN;
      m[3] = tie_top;
      m[4] = has_top ? ceq - tie_top : 0.0;
    }
  }
  __shared__ SelState ss[4];
  if (lane == 0) ss[q] = s;
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * kSelBins; i += 256) base[i] = 0;
  if (lane == 0) {
    int src = q;
    for (int r = 0; r < q; ++r)
      if (ss[r].valid && ss[r].prefix == s.prefix) {
        src = r;
        break;
      }
    s.src = src;
    sel[l * 4 + q] = s;
  }
}

// group sums over the array's values: pass 0 [sum all, sum v > vk, #(v > vk),
// #(v == vk)], pass 1 [|v - m_all|, (v - m_all)^2, top |.|, top ^2, adj |.|,
// adj ^2] (v == vk excluded: the fold adds those copies)
template <typename VT>
__global__ void __launch_bounds__(kT) sel_sums_kernel(const VT* vals, int64_t N, const SelState* sel,
                                                      const double* means, int pass, double* part) {
  typedef typename KeyT<VT>::K K;
  const int l = blockIdx.y, c = blockIdx.x;
  const VT* s = vals + (int64_t)l * pad4(N);
  const bool has_top = sel[l * 4].valid != 0;
  const double vk = has_top ? (double)kval((K)sel[l * 4].prefix) : 0.0;
  int64_t b0, b1;
  chunk_range(N, c, kChunks, b0, b1);
  double acc[6] = {0, 0, 0, 0, 0, 0};
  const double ma = pass ? means[l * 8 + 0] : 0.0, mt = pass ? means[l * 8 + 1] : 0.0,
               md = pass ? means[l * 8 + 2] : 0.0;
  for_vals(s, b0, b1, [&](VT x) {
    const double v = (double)x;
    const bool gt = has_top && v > vk, lt = !has_top || v < vk;
    if (!pass) {
      acc[0] += v;
      if (gt) {
        acc[1] += v;
        acc[2] += 1.0;
      }
      if (has_top && v == vk) acc[3] += 1.0;
    } else {
      const double da = v - ma;
      acc[0] += fabs(da);
      acc[1] += da * da;
      if (gt) {
        const double d = v - mt;
        acc[2] += fabs(d);
        acc[3] += d * d;
      }
      if (lt) {
        const double d = v - md;
        acc[4] += fabs(d);
        acc[5] += d * d;
      }
    }
  });
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

// pass 0: the three groups' means (and the boundary's copies per group); pass 1:
// the table column at step t.  rows: table rows per array; row0: where the 12
// statistics go; the n_extra constants extra[l][*] fill rows row0 + 12 ... (the
// sweeps' lev row, the big-brain stop / roll rows)
template <typename VT>
__global__ void sel_fold_kernel(int64_t N, int64_t top, int n_arr, const SelState* sel, const double* part, int pass,
                                double* means, const float* extra, int n_extra, float* data, int rows, int row0,
                                int steps, int t) {
  typedef typename KeyT<VT>::K K;
  const int l = blockIdx.x;  // one wave per array: lane c folds chunks c, c + 64, ..., then a fixed butterfly
  double s[6] = {0, 0, 0, 0, 0, 0};
  for (int c = threadIdx.x; c < kChunks; c += 64)
    for (int q = 0; q < 6; ++q) s[q] += part[((int64_t)l * kChunks + c) * 6 + q];
#pragma unroll
  for (int q = 0; q < 6; ++q)
    for (int o = 32; o > 0; o >>= 1) s[q] += __shfl_xor(s[q], o, 64);
  if (threadIdx.x != 0) return;
  const double na = (double)N, nt = (double)top, nd = (double)(N - top);
  const bool has_top = sel[l * 4].valid != 0;
  const double vk = has_top ? (double)kval((K)sel[l * 4].prefix) : 0.0;
  double* m = means + l * 8;
  if (!pass) {
    const double tie_top = has_top ? nt - s[2] : 0.0;  // copies of vk in the top group
    const double tie_adj = has_top ? s[3] - tie_top : 0.0;
    const double sum_top = has_top ? s[1] + tie_top * vk : 0.0;
    m[0] = s[0] / na;
    m[1] = sum_top / nt;
    m[2] = N > top ? (s[0] - sum_top) / nd : NAN;
    m[3] = tie_top;
    m[4] = tie_adj;
    return;
  }
  const double tie_top = m[3], tie_adj = m[4];
  const double dt = vk - m[1], dd = vk - m[2];
  auto med = [&](int q) -> double {
    const SelState& x = sel[l * 4 + q];
    return x.valid ? (double)kval((K)x.prefix) : NAN;
  };
  const float col[12] = {(float)m[0],
                         (float)m[1],
                         (float)m[2],
                         (float)(s[0] / na),
                         (float)((s[2] + tie_top * fabs(dt)) / nt),
                         (float)((s[4] + tie_adj * fabs(dd)) / nd),
                         (float)sqrt(s[1] / na),
                         (float)sqrt((s[3] + tie_top * dt * dt) / nt),
                         (float)sqrt((s[5] + tie_adj * dd * dd) / nd),
                         (float)med(1),
                         (float)med(2),
                         (float)med(3)};
  for (int r = 0; r < 12; ++r) data[((int64_t)l * rows + row0 + r) * steps + t] = col[r];
  for (int e = 0; e < n_extra; ++e) data[((int64_t)l * rows + row0 + 12 + e) * steps + t] = extra[l * n_extra + e];
}

struct SelWork {
  unsigned* hist;  // [n_arr][4][kSelBins], zero between passes
  SelState* sel;   // [n_arr][4]
  double* part;    // [n_arr][kChunks][6]
  double* part2;   // [n_arr][kSelBlocks][3]
  double* means;   // [n_arr][8]
};

size_t sel_work_bytes(int64_t n_arr) {
  return (size_t)n_arr * (4 * kSelBins * 4 + 4 * sizeof(SelState) + kChunks * 6 * 8 + kSelBlocks * 3 * 8 + 8 * 8) +
         1024;
}

SelWork sel_work(unsigned char* p, int64_t n_arr) {
  SelWork w;
  w.hist = reinterpret_cast<unsigned*>(p);
  w.sel = reinterpret_cast<SelState*>(p + n_arr * 4 * kSelBins * 4);
  w.part = reinterpret_cast<double*>(w.sel + n_arr * 4);
  w.part2 = w.part + n_arr * kChunks * 6;
  w.means = w.part2 + n_arr * kSelBlocks * 3;
  return w;
}

// the column of every array at step t: the select passes (the first digit's
// histogram already built when hist0_done), then the two sum passes
template <typename VT>
int sel_stats(const VT* vals, int64_t N, int64_t top, int n_arr, const SelWork& w, bool hist0_done, const float* extra,
              int n_extra, float* data, int rows, int row0, int steps, int t, hipStream_t st) {
  constexpr int bits = 8 * sizeof(VT);
  const int P = sel_passes(bits);
  RLMD_CHECK(hist0_done, "select: first digit histogram missing");
  for (int p = 0; p < P; ++p) {
    const int last = p == P - 1 ? 1 : 0;
    if (p > 0) {
      hipLaunchKernelGGL(sel_hist_kernel<VT>, dim3(kSelBlocks, n_arr), dim3(kT), 0, st, vals, N, p, last, w.sel,
                         w.hist, w.part2);
      RLMD_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(sel_scan_kernel<VT>, dim3(n_arr), dim3(256), 0, st, p, last, N, top, w.sel, w.hist, w.part2,
                       w.means);
    RLMD_LAUNCH_CHECK();
  }
  // the deviations from the means, then the column
  hipLaunchKernelGGL(sel_sums_kernel<VT>, dim3(kChunks, n_arr), dim3(kT), 0, st, vals, N, w.sel, w.means, 1, w.part);
  RLMD_LAUNCH_CHECK();
  hipLaunchKernelGGL(sel_fold_kernel<VT>, dim3(n_arr), dim3(64), 0, st, N, top, n_arr, w.sel, w.part, 1, w.means,
                     extra, n_extra, data, rows, row0, steps, t);
  RLMD_LAUNCH_CHECK();
  return 0;
}

// ---- outcome windows ---------------------------------------------------------
// win[s][i] = src[i][t0 + s] for s < ns (64 investors x 32 steps per workgroup
// through an LDS tile: row reads of 32 consecutive steps, coalesced column writes)
template <typename T>
__global__ void __launch_bounds__(256) lev_window_kernel(const T* src, int64_t inv, int64_t ld, int t0, int ns,
                                                         T* win) {
  __shared__ T tile[64][kW + 1];
  const int64_t i0 = (int64_t)blockIdx.x * 64;
  for (int e = threadIdx.x; e < 64 * kW; e += 256) {
    const int r = e / kW, c = e - r * kW;
    if (i0 + r < inv && c < ns) tile[r][c] = src[(i0 + r) * ld + t0 + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * kW; e += 256) {
    const int c = e / 64, r = e - c * 64;
    if (i0 + r < inv && c < ns) win[(int64_t)c * pad4(inv) + i0 + r] = tile[r][c];
  }
}

// ---- the sweeps ----------------------------------------------------------------
struct SortedArgs {
  int kind;              // 0 categorical (u8 outcomes 0/1/2), 1 GBM (f32 outcomes)
  const uint8_t* wcat;   // this window's outcomes [kW][investors]
  const float* wgbm;
  int64_t investors;
  int n_lev;
  const float* table;  // [n_lev][3] (categorical)
  const float* levs;   // [n_lev]
  float* val;          // [n_lev][investors]
};

// t == 0: val = value_0 * factor(t = 0); else val *= factor(t); with hist, the
// new values' first select digit histogrammed on the way (key bits [21, 32))
__global__ void __launch_bounds__(kT) lev_advance_kernel(SortedArgs a, int t, int s, float value_0, int hist,
                                                         unsigned* hist_out) {
  const int l = blockIdx.y;
  __shared__ unsigned h[kSelBins];
  if (hist)
    for (int i = threadIdx.x; i < kSelBins; i += kT) h[i] = 0;
  __syncthreads();
  int64_t b0, b1;
  chunk_range(a.investors, blockIdx.x, gridDim.x, b0, b1);
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const int64_t P4 = pad4(a.investors);
  float* v = a.val + (int64_t)l * P4;
  const float lv = a.levs[l];
  float tab[3] = {0.f, 0.f, 0.f};
  if (a.kind == 0)
    for (int q = 0; q < 3; ++q) tab[q] = a.table[l * 3 + q];
  // 4 investors per thread: 16-B value loads / stores, 4-B (codes) or 16-B
  // (GBM) outcome loads; lanes past N sit in the row padding
  for (int64_t i = b0 + 4 * threadIdx.x; i < b1; i += 4 * kT) {
    f32x4 x = t == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(v + i);
    float g[4];
    if (a.kind == 0) {
      const uchar4 o = *reinterpret_cast<const uchar4*>(a.wcat + (int64_t)s * P4 + i);
      const int oc[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = oc[e] == 0 ? tab[0] : (oc[e] == 1 ? tab[1] : tab[2]);
    } else {
      const f32x4 o = *reinterpret_cast<const f32x4*>(a.wgbm + (int64_t)s * P4 + i);
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = expf(lv * o[e]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[e] = t == 0 ? value_0 * g[e] : x[e] * g[e];
      if (hist && i + e < b1) atomicAdd(&h[okey(x[e]) >> (32 - kSelB)], 1u);
    }
    *reinterpret_cast<f32x4*>(v + i) = x;
  }
  if (!hist) return;
  __syncthreads();
  flush_hist(h, kSelBins, hist_out + (int64_t)l * 4 * kSelBins);
}

// ---------------------------------------------------------------------------
// big-brain investors (coin_big_brain_lev :270-452, dice_big_brain_lev :741-932):
// configuration c = (roll, stop) sets each investor's leverage from its own
// value every step — lev = lev_factor (1 - L / v) with L the stop-loss floor
// stop * value_0, or, when roll > 0 and v > value_0, the rolling floor
// value_0 + roll (v - value_0) (coin_optimal_lev :240-267, dice_optimal_lev
// :704-738) — in the reference's arithmetic (coin f32; dice f64 values, see
// optimal_lev; this file compiles with FP contraction off).  Per step: the
// leverages' statistics (rows 12-23, then stop and roll), the value step
// v = v (1 + lev r), the new leverages, the values' statistics (rows 0-11).
// ---------------------------------------------------------------------------
struct BrainArgs {
  const uint8_t* wcat;  // this window's outcome codes [kW][investors]
  int64_t investors;
  double ret[3];        // return per outcome code (f32 values for coin, f64 for dice)
  float value_0, lev_factor;
  const float* cfg;     // [n_cfg][5]: stop floor value_min, roll, initial leverage, roll > 0, stop level
  void* val;            // [n_cfg][investors] VT
  void* lev;            // [n_cfg][investors] VT
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

// t == 0: v = value_0 (1 + lev0 r[0]); else v = v (1 + lev r[t]); then lev =
// optimal(v); the first select digit of the new leverages (hist_lev) and, when
// hist_val, of the new values histogrammed on the way
template <typename VT>
__global__ void __launch_bounds__(kT) lev_brain_advance_kernel(BrainArgs a, int t, int s, unsigned* hist_lev,
                                                               unsigned* hist_val) {
  constexpr int bits = 8 * sizeof(VT);
  const int c = blockIdx.y;
  __shared__ unsigned hl[kSelBins], hv[kSelBins];
  for (int i = threadIdx.x; i < kSelBins; i += kT) {
    hl[i] = 0;
    hv[i] = 0;
  }
  __syncthreads();
  const float* k = a.cfg + 5 * c;
  const float vmin = k[0], roll = k[1], lev0 = k[2];
  const bool rolling = k[3] != 0.f;
  const int64_t P4 = pad4(a.investors);
  VT* val = static_cast<VT*>(a.val) + (int64_t)c * P4;
  VT* lev = static_cast<VT*>(a.lev) + (int64_t)c * P4;
  const uint8_t* wc = a.wcat + (int64_t)s * P4;
  int64_t b0, b1;
  chunk_range(a.investors, blockIdx.x, gridDim.x, b0, b1);
  for (int64_t i = b0 + threadIdx.x; i < b1; i += kT) {
    const int o = wc[i];
    const VT r = (VT)a.ret[o > 2 ? 2 : o];
    const VT v = t == 0 ? (VT)a.value_0 * ((VT)1 + (VT)lev0 * r) : val[i] * ((VT)1 + lev[i] * r);
    const VT l = optimal_lev<VT>(v, a.value_0, vmin, roll, rolling, a.lev_factor);
    val[i] = v;
    lev[i] = l;
    atomicAdd(&hl[(unsigned)(okey(l) >> (bits - kSelB))], 1u);
    if (hist_val) atomicAdd(&hv[(unsigned)(okey(v) >> (bits - kSelB))], 1u);
  }
  __syncthreads();
  flush_hist(hl, kSelBins, hist_lev + (int64_t)c * 4 * kSelBins);
  if (hist_val) flush_hist(hv, kSelBins, hist_val + (int64_t)c * 4 * kSelBins);
}

}  // namespace

extern "C" {

int64_t rlmd_lev_sorted_workspace_bytes(int64_t investors, int32_t n_lev) {
  if (investors <= 0 || investors > INT32_MAX || n_lev <= 0) return -1;
  const int64_t vals = (int64_t)n_lev * pad4(investors) * 4;
  const int64_t win = (int64_t)kW * pad4(investors) * 4;  // f32 or u8 outcome window
  const int64_t small = (int64_t)n_lev * 16 * 4;
  return ((vals + 255) & ~255ll) + ((win + 255) & ~255ll) + (int64_t)sel_work_bytes(n_lev) + small + 256;
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
  const int64_t vals = (int64_t)n_lev * pad4(investors) * 4;
  const int64_t winb = (int64_t)kW * pad4(investors) * 4;
  float* val = reinterpret_cast<float*>(w);
  void* win = w + ((vals + 255) & ~255ll);
  unsigned char* ws = static_cast<unsigned char*>(win) + ((winb + 255) & ~255ll);
  const SelWork sw = sel_work(ws, n_lev);
  float* small = reinterpret_cast<float*>(ws + sel_work_bytes(n_lev));  // levs [n_lev] | table [n_lev][3]
  RLMD_HIP(hipMemsetAsync(sw.hist, 0, (size_t)n_lev * 4 * kSelBins * 4, st));
  RLMD_HIP(hipMemcpyAsync(small, levs_host, sizeof(float) * n_lev, hipMemcpyHostToDevice, st));
  if (kind == 0)
    RLMD_HIP(hipMemcpyAsync(small + n_lev, table_host, sizeof(float) * 3 * n_lev, hipMemcpyHostToDevice, st));
  SortedArgs a{};
  a.kind = kind;
  a.wcat = static_cast<const uint8_t*>(win);
  a.wgbm = static_cast<const float*>(win);
  a.investors = investors;
  a.n_lev = n_lev;
  a.levs = small;
  a.table = small + n_lev;
  a.val = val;
  const int steps = final_only ? 1 : horizon - 1;
  const dim3 grid_win((unsigned)((investors + 63) / 64));
  for (int t = 0; t < horizon; ++t) {
    if (t % kW == 0) {
      const int ns = std::min(kW, horizon - t);
      if (kind == 0)
        hipLaunchKernelGGL(lev_window_kernel<uint8_t>, grid_win, dim3(256), 0, st,
                           static_cast<const uint8_t*>(outcomes_dev), investors, ld, t, ns,
                           static_cast<uint8_t*>(win));
      else
        hipLaunchKernelGGL(lev_window_kernel<float>, grid_win, dim3(256), 0, st,
                           static_cast<const float*>(outcomes_dev), investors, ld, t, ns, static_cast<float*>(win));
      RLMD_LAUNCH_CHECK();
    }
    const bool stats = final_only ? t == horizon - 1 : t > 0;
    hipLaunchKernelGGL(lev_advance_kernel, dim3(kSelBlocks, n_lev), dim3(kT), 0, st, a, t, t % kW, value_0,
                       stats ? 1 : 0, sw.hist);
    RLMD_LAUNCH_CHECK();
    if (!stats) continue;
    RLMD_TRY_INT(sel_stats<float>(val, investors, tp, n_lev, sw, true, small, 1, data_dev, 13, 0, steps,
                                  final_only ? 0 : t - 1, st));
  }
  if (data_T_dev)
    RLMD_HIP(hipMemcpy2DAsync(data_T_dev, sizeof(float) * investors, val, sizeof(float) * pad4(investors),
                              sizeof(float) * investors, n_lev, hipMemcpyDeviceToDevice, st));
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
  const int64_t vals = 2 * (int64_t)n_cfg * pad4(investors) * 8;  // values, leverages (f64 at most)
  const int64_t win = (int64_t)kW * pad4(investors);
  const int64_t small = (int64_t)n_cfg * 8 * 4;
  return ((vals + 255) & ~255ll) + ((win + 255) & ~255ll) + 2 * (int64_t)sel_work_bytes(n_cfg) + small + 256;
}

}  // extern "C"

template <typename VT>
static int lev_brain(const uint8_t* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld, int64_t top,
                     float value_0, const double* rets3, float lev_factor, const float* cfg_host, int32_t n_cfg,
                     void* workspace, float* data_dev, hipStream_t st) {
  const int64_t tp = top < investors ? (top > 0 ? top : 0) : investors;
  unsigned char* w = static_cast<unsigned char*>(workspace);
  const int64_t NC = (int64_t)n_cfg * pad4(investors);
  VT* val = reinterpret_cast<VT*>(w);
  VT* lev = val + NC;
  uint8_t* win = w + ((2 * NC * 8 + 255) & ~255ll);
  unsigned char* ws = win + (((int64_t)kW * pad4(investors) + 255) & ~255ll);
  const SelWork wl = sel_work(ws, n_cfg), wv = sel_work(ws + sel_work_bytes(n_cfg), n_cfg);  // leverages, values
  float* cfg = reinterpret_cast<float*>(ws + 2 * sel_work_bytes(n_cfg));  // [n_cfg][5] | extra [n_cfg][2]
  float* extra = cfg + 5 * n_cfg;
  std::vector<float> ex(2 * (size_t)n_cfg);
  for (int c = 0; c < n_cfg; ++c) {  // rows 24 / 25: stop level and roll
    ex[2 * c] = cfg_host[5 * c + 4];
    ex[2 * c + 1] = cfg_host[5 * c + 1];
  }
  RLMD_HIP(hipMemsetAsync(wl.hist, 0, (size_t)n_cfg * 4 * kSelBins * 4, st));
  RLMD_HIP(hipMemsetAsync(wv.hist, 0, (size_t)n_cfg * 4 * kSelBins * 4, st));
  RLMD_HIP(hipMemcpyAsync(cfg, cfg_host, sizeof(float) * 5 * n_cfg, hipMemcpyHostToDevice, st));
  RLMD_HIP(hipMemcpyAsync(extra, ex.data(), sizeof(float) * 2 * n_cfg, hipMemcpyHostToDevice, st));
  BrainArgs a{};
  a.wcat = win;
  a.investors = investors;
  for (int q = 0; q < 3; ++q) a.ret[q] = rets3[q];
  a.value_0 = value_0;
  a.lev_factor = lev_factor;
  a.cfg = cfg;
  a.val = val;
  a.lev = lev;
  const dim3 grid_adv(kSelBlocks, (unsigned)n_cfg);
  const dim3 grid_win((unsigned)((investors + 63) / 64));
  const int steps = horizon - 1;
  // the advance histograms both arrays' first digit (the values' from step 1 on)
  auto stats = [&](const VT* src, const SelWork& sw, int row0, const float* ext, int n_ext, int t) -> int {
    return sel_stats<VT>(src, investors, tp, n_cfg, sw, true, ext, n_ext, data_dev, 26, row0, steps, t, st);
  };
  auto advance = [&](int t) -> int {
    if (t % kW == 0) {
      hipLaunchKernelGGL(lev_window_kernel<uint8_t>, grid_win, dim3(256), 0, st, outcomes_dev, investors, ld, t,
                         std::min(kW, (int)horizon - t), win);
      RLMD_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(lev_brain_advance_kernel<VT>, grid_adv, dim3(kT), 0, st, a, t, t % kW, wl.hist,
                       t > 0 ? wv.hist : nullptr);
    RLMD_LAUNCH_CHECK();
    return 0;
  };
  RLMD_TRY_INT(advance(0));
  for (int t = 0; t < steps; ++t) {
    RLMD_TRY_INT(stats(lev, wl, 12, extra, 2, t));
    RLMD_TRY_INT(advance(t + 1));
    RLMD_TRY_INT(stats(val, wv, 0, nullptr, 0, t));
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
