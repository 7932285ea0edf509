// rows.hip — row-block kernels of the SAC / TD3 update (gfx950, wave64).
//
// learn() (algos/algo_sac.py:300-615, algos/algo_td3.py:302-560) is a chain of
// small per-row MLP evaluations separated by a few batch-wide reductions.  Every
// per-row stretch of that chain runs here inside ONE 16-row workgroup (4 waves),
// so the intermediate activations never round-trip through a kernel boundary:
//   layer 1      VALU, one thread per hidden unit, x rows broadcast from LDS
//   layer 2      v_mfma_f32_16x16x32_bf16 (bf16) / v_mfma_f32_16x16x4f32 (fp32):
//                A = the 16 activation rows in LDS, B = fc2.weight fragments read
//                16 bytes per lane straight from the zero-padded compute copy
//                (L2-resident, shared by every workgroup), prefetched a register
//                group ahead; wave w owns output column blocks w, w+4, ...
//   heads        LDS dot products, split over up to 64 lanes per dot
//   sampling     tanh-Gaussian / TD3 noise per row (networks_sac.py:101-178)
// Backward data paths use the transposed compute copy with the same MFMA loop.
// Weight gradients (batch reductions) are left to gemm.hip's BWD_W launch.
#include <math.h>

#include "learn_kernels.h"
#include "rlmd_common.h"

namespace rlmd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int R = kRowBlock;
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
constexpr int kHeadsMax = 2 * RLMD_MAX_ACTION;

__device__ __forceinline__ unsigned short to_bf16(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

template <int PREC>
struct CT;
template <>
struct CT<RLMD_BF16> {
  using T = unsigned short;
  using Frag = bf16x8;
  static constexpr int KS = 32;  // k covered by one 16-byte fragment per lane
  static constexpr int PAD = 8;  // LDS row pad (elements): 16-B aligned rows
  __device__ static T cvt(float f) { return to_bf16(f); }
  __device__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct CT<RLMD_FP32> {
  using T = float;
  using Frag = f32x4;
  static constexpr int KS = 16;
  static constexpr int PAD = 4;
  __device__ static T cvt(float f) { return f; }
  // lane group q = lane >> 4 holds k = k0 + 4q + j in element j: four 16x16x4
  // MFMAs cover k0 .. k0 + 15 (a permutation of the k order, same products)
  __device__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  }
};

// LDS carve-up, identical on host (launch size) and device.
struct Lds {
  int xs, a1, aT, h2s, h1s, hout, ghs, rowv, total;  // byte offsets
  int ldx, lda1, ldaT, ldh2, ldh1;                   // row pitches (elements)
};
__host__ __device__ inline Lds lds_layout(const RowDims& d) {
  const int ts = d.prec == RLMD_BF16 ? 2 : 4;
  const int pad = d.prec == RLMD_BF16 ? 8 : 4;
  Lds l{};
  auto up = [](int v) { return (v + 15) & ~15; };
  int o = 0;
  l.ldx = d.X;
  l.xs = o;
  o = up(o + R * d.X * 4);
  l.lda1 = d.H1p + pad;
  l.a1 = o;
  o = up(o + R * l.lda1 * ts);
  l.ldaT = d.H2p + pad;
  l.aT = o;
  o = up(o + R * l.ldaT * ts);
  l.ldh2 = d.H2p + 4;
  l.h2s = o;
  o = up(o + R * l.ldh2 * 4);
  l.ldh1 = d.H1p + 4;
  l.h1s = o;
  o = up(o + R * l.ldh1 * 4);
  l.hout = o;
  o = up(o + R * kHeadsMax * 4);
  l.ghs = o;
  o = up(o + R * kHeadsMax * 4);
  l.rowv = o;
  o = up(o + R * 4 * 4);
  l.total = o;
  return l;
}

template <int PREC, int NBW, int G>
__device__ __forceinline__ void frag_load(typename CT<PREC>::Frag (&bf)[G][NBW], const typename CT<PREC>::T* Bg,
                                          uint32_t boff, int ldb, int s0, int nsteps, int nblk) {
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < NBW; ++i)
      if (wave + 4 * i < nblk && s0 + g < nsteps)
        bf[g][i] = *reinterpret_cast<const typename CT<PREC>::Frag*>(
            Bg + boff + (uint32_t)(64 * i * ldb) + (uint32_t)((s0 + g) * CT<PREC>::KS));
}

template <int PREC, int NBW, int G>
__device__ __forceinline__ void frag_mfma(const typename CT<PREC>::Frag (&bf)[G][NBW], const typename CT<PREC>::T* As,
                                          uint32_t aoff, int s0, int nsteps, int nblk, f32x4 (&acc)[NBW]) {
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (s0 + g < nsteps) {
      const typename CT<PREC>::Frag a =
          *reinterpret_cast<const typename CT<PREC>::Frag*>(As + aoff + (s0 + g) * CT<PREC>::KS);
#pragma unroll
      for (int i = 0; i < NBW; ++i)
        if (wave + 4 * i < nblk) CT<PREC>::mfma(a, bf[g][i], acc[i]);
    }
  }
}

// acc[i] (i < NBW) = A[16 x K] * B^T for output column block nb = wave + 4 i:
// As: LDS rows of the A operand (pitch lda elements); Bg: compute copy with one
// row of K elements per output column (pitch ldb), zero-padded.  B fragments are
// double-buffered in registers, G K-steps (G * NBW 16-byte loads per lane) ahead.
template <int PREC, int NBW>
__device__ __forceinline__ void mfma_rows(const typename CT<PREC>::T* As, int lda,
                                          const typename CT<PREC>::T* Bg, int ldb, int K, int nblk,
                                          f32x4 (&acc)[NBW]) {
  using C = CT<PREC>;
  using Frag = typename C::Frag;
  constexpr int EPF = 16 / sizeof(typename C::T);
  constexpr int G = NBW >= 8 ? 1 : 8 / NBW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ko = EPF * (lane >> 4);
#pragma unroll
  for (int i = 0; i < NBW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = K / C::KS;
  const uint32_t boff = (uint32_t)((wave * 16 + (lane & 15)) * ldb + ko);
  const uint32_t aoff = (uint32_t)((lane & 15) * lda + ko);
  Frag b0[G][NBW], b1[G][NBW];
  frag_load<PREC, NBW, G>(b0, Bg, boff, ldb, 0, nsteps, nblk);
  for (int s0 = 0; s0 < nsteps; s0 += 2 * G) {
    frag_load<PREC, NBW, G>(b1, Bg, boff, ldb, s0 + G, nsteps, nblk);
    frag_mfma<PREC, NBW, G>(b0, As, aoff, s0, nsteps, nblk, acc);
    frag_load<PREC, NBW, G>(b0, Bg, boff, ldb, s0 + 2 * G, nsteps, nblk);
    frag_mfma<PREC, NBW, G>(b1, As, aoff, s0 + G, nsteps, nblk, acc);
  }
}

// h1 = relu(x W1^T + b1) for the block's rows; x rows in LDS (pitch ldx, first
// `in` columns).  Writes the MFMA operand copy (T, zero-padded to H1p) and the
// f32 activations to HBM (nullable) for the weight gradients / masks.
template <int PREC>
__device__ void layer1(const float* p, const NetOff& o, const float* xs, int ldx, int in,
                       typename CT<PREC>::T* a1, int lda1, float* h1_out, int row0, int B) {
  const int H1 = o.h1, H1p = pad32(H1);
  for (int c = threadIdx.x; c < H1p; c += blockDim.x) {
    if (c < H1) {
      float acc[R];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = 0.f;
      const float* w = p + o.w1 + (int64_t)c * in;
      for (int k = 0; k < in; ++k) {
        const float wk = w[k];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fmaf(xs[r * ldx + k], wk, acc[r]);
      }
      const float bb = p[o.b1 + c];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float v = fmaxf(acc[r] + bb, 0.f);
        a1[r * lda1 + c] = CT<PREC>::cvt(v);
        if (h1_out && row0 + r < B) h1_out[(int64_t)(row0 + r) * H1 + c] = v;
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) a1[r * lda1 + c] = CT<PREC>::cvt(0.f);
    }
  }
}

// h2 = relu(h1 W2^T + b2) -> LDS f32 rows (zero beyond H2) and HBM (nullable).
template <int PREC, int NBW>
__device__ void layer2(const RowNet& net, const NetOff& o, const typename CT<PREC>::T* a1, int lda1,
                       float* h2s, int ldh2, float* h2_out, int row0, int B) {
  using T = typename CT<PREC>::T;
  const int H1p = pad32(o.h1), H2 = o.h2, H2p = pad32(H2);
  f32x4 acc[NBW];
  mfma_rows<PREC, NBW>(a1, lda1, static_cast<const T*>(net.wc), H1p, H1p, H2p / 16, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int nb = wave + 4 * i;
    if (nb < H2p / 16) {
      const int col = nb * 16 + (lane & 15);
      const bool cin = col < H2;
      const float bias = cin ? net.p[o.b2 + col] : 0.f;
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int r = 4 * (lane >> 4) + rg;
        const float v = cin ? fmaxf(acc[i][rg] + bias, 0.f) : 0.f;
        h2s[r * ldh2 + col] = v;
        if (h2_out && cin && row0 + r < B) h2_out[(int64_t)(row0 + r) * H2 + col] = v;
      }
    }
  }
}

// out[r][h] (+)= sum_c src[r][c] * w_h[c * cstride], h < nh, where w_h = wa + h*ldw
// for h < na and wb + (h - na)*ldw beyond.  A dot is split over P lanes of one wave.
__device__ void row_dots(const float* src, int lds, int ncols, int nh, const float* wa, const float* wb,
                         int na, int64_t ldw, int cstride, float* out, int ldo, bool accumulate) {
  const int nd = R * nh;
  int P = 64;
  while (P > 1 && nd * P > (int)blockDim.x) P >>= 1;
  const int part = threadIdx.x % P;
  for (int d0 = threadIdx.x / P; d0 < nd; d0 += blockDim.x / P) {
    const int h = d0 / R, r = d0 % R;
    const float* w = h < na ? wa + (int64_t)h * ldw : wb + (int64_t)(h - na) * ldw;
    float acc = 0.f;
    for (int c = part; c < ncols; c += P) acc = fmaf(src[r * lds + c], w[(int64_t)c * cstride], acc);
    for (int off = P >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (part == 0) out[r * ldo + h] = accumulate ? out[r * ldo + h] + acc : acc;
  }
}

// Full critic forward for the block's rows: x in LDS -> q (no head bias).
template <int PREC, int NBW>
__device__ void critic_rows(const RowNet& net, const NetOff& co, const float* xs, int ldx, int X,
                            unsigned char* smem, const Lds& L, float* h1_out, float* h2_out, float* q_out,
                            int row0, int B) {
  using T = typename CT<PREC>::T;
  T* a1 = reinterpret_cast<T*>(smem + L.a1);
  float* h2s = reinterpret_cast<float*>(smem + L.h2s);
  float* hout = reinterpret_cast<float*>(smem + L.hout);
  layer1<PREC>(net.p, co, xs, ldx, X, a1, L.lda1, h1_out, row0, B);
  __syncthreads();
  layer2<PREC, NBW>(net, co, a1, L.lda1, h2s, L.ldh2, h2_out, row0, B);
  __syncthreads();
  row_dots(h2s, L.ldh2, co.h2, 1, net.p + co.w3, nullptr, 1, co.h2, 1, hout, kHeadsMax, false);
  __syncthreads();
  if (threadIdx.x < R && row0 + (int)threadIdx.x < B) q_out[row0 + threadIdx.x] = hout[threadIdx.x * kHeadsMax];
  __syncthreads();
}

// Policy forward + sample for the block's rows: state in xs[:, :S]; the sampled
// action is written to xs[:, S:S+A] (the critic input) and to xa_out (nullable).
// mode 0: stochastic (SAC tanh-Gaussian / TD3 exploration or smoothing noise),
// mode 1: deterministic.  Same arithmetic as learn.hip's actor_head_kernel.
template <int PREC, int NBW>
__device__ void actor_rows(const RowNet& net, const NetOff& ao, const RowDims& d, const SampleCfg& smp,
                           float* xs, int ldx, unsigned char* smem, const Lds& L, float* h1_out, float* h2_out,
                           int mode, int tag, const float* eps_in, float noise_std, float noise_clip,
                           int clamp_noise, float* logp_out, float* save, float* xa_out, int row0, int B) {
  using T = typename CT<PREC>::T;
  T* a1 = reinterpret_cast<T*>(smem + L.a1);
  float* h2s = reinterpret_cast<float*>(smem + L.h2s);
  float* hout = reinterpret_cast<float*>(smem + L.hout);
  const int S = d.S, A = d.A;
  const bool sac = d.algo == RLMD_SAC;
  layer1<PREC>(net.p, ao, xs, ldx, S, a1, L.lda1, h1_out, row0, B);
  __syncthreads();
  layer2<PREC, NBW>(net, ao, a1, L.lda1, h2s, L.ldh2, h2_out, row0, B);
  __syncthreads();
  row_dots(h2s, L.ldh2, ao.h2, sac ? 2 * A : A, net.p + ao.w3, sac ? net.p + ao.w4 : nullptr, A, ao.h2, 1, hout,
           kHeadsMax, false);
  __syncthreads();
  const int r = threadIdx.x;
  if (r < R) {
    const int b = row0 + r;
    const bool valid = b < B;
    const uint32_t c1 = (uint32_t)*smp.ctr;
    float logp = 0.f;
    for (int j = 0; j < A; ++j) {
      float mu = hout[r * kHeadsMax + j] + net.p[ao.b3 + j];
      float eps = 0.f;
      if (mode == 0 && valid) {
        if (eps_in) {
          eps = eps_in[(int64_t)b * A + j];
        } else {
          double z0, z1;
          rlmd_normal2(rlmd_philox(smp.seed, (uint32_t)b, c1, (uint32_t)tag, (uint32_t)(j >> 1)), z0, z1);
          eps = (float)((j & 1) ? z1 : z0);
        }
      }
      float act;
      if (sac) {
        const float ls_raw = hout[r * kHeadsMax + A + j] + net.p[ao.b4 + j];
        const float ls = fminf(fmaxf(ls_raw, smp.ls_min), smp.ls_max);
        float sigma = expf(ls);
        if (!isfinite(mu)) mu = 0.f;  // NaN scrub (networks_sac.py:131-134)
        if (!isfinite(sigma)) sigma = 3.f;
        if (mode == 1) {
          act = tanhf(mu) * smp.max_action;
        } else {
          const float u = mu + eps * sigma;
          const float dd = u - mu;
          const float lpn = -(dd * dd) / (2.f * (sigma * sigma)) - logf(sigma) - kLogSqrt2Pi;
          act = tanhf(u) * smp.max_action;
          const float an = act / smp.max_action;
          logp += lpn - logf(1.f - an * an + smp.reparam_noise);
          if (save && valid) {
            float* sv = save + (int64_t)b * 5 * A;
            sv[j] = mu;
            sv[A + j] = sigma;
            sv[2 * A + j] = eps;
            sv[3 * A + j] = u;
            sv[4 * A + j] = ls_raw;
          }
        }
      } else {
        act = tanhf(mu) * smp.max_action;
        if (mode == 0) {
          float nz = eps * noise_std;
          if (clamp_noise) nz = fminf(fmaxf(nz, -noise_clip), noise_clip);
          act = fminf(fmaxf(act + nz, -smp.max_action), smp.max_action);
        }
        if (save && valid) save[(int64_t)b * 5 * A + j] = mu;  // pre-tanh for backward
      }
      xs[r * ldx + S + j] = act;
      if (xa_out && valid) xa_out[(int64_t)b * d.X + S + j] = act;
    }
    if (logp_out && valid) logp_out[b] = logp;
  }
  __syncthreads();
}

// Stage rows [row0, row0 + 16) of a [B, in] matrix into xs (pitch ldx), zeros past B.
__device__ void stage_rows(const float* src, int in, float* xs, int ldx, int row0, int B) {
  for (int e = threadIdx.x; e < R * in; e += blockDim.x) {
    const int r = e / in, k = e % in;
    xs[r * ldx + k] = row0 + r < B ? src[(int64_t)(row0 + r) * in + k] : 0.f;
  }
}

template <int PREC, int NBW>
__global__ void __launch_bounds__(256) fwd_rows_kernel(FwdRowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowDims& d = a.d;
  const Lds L = lds_layout(d);
  float* xs = reinterpret_cast<float*>(smem + L.xs);
  const int row0 = blockIdx.x * R, job = blockIdx.y, B = d.B;
  if (job == 0) {  // target path (algo_sac.py:300-367 / algo_td3.py:302-361)
    stage_rows(a.s2, d.S, xs, L.ldx, row0, B);
    __syncthreads();
    actor_rows<PREC, NBW>(a.tactor, a.ao, d, a.smp, xs, L.ldx, smem, L, nullptr, nullptr, 0, a.t_tag, a.eps_next,
                          a.t_noise_std, a.t_noise_clip, a.t_clamp, a.logp_next, nullptr, nullptr, row0, B);
#pragma nounroll
    for (int g = 0; g < 2; ++g)
      critic_rows<PREC, NBW>(a.tcrit[g], a.co, xs, L.ldx, d.X, smem, L, nullptr, nullptr, a.qt[g], row0, B);
  } else if (job <= 2) {  // online critics on (s, a) (algo_sac.py:413-417)
    const int g = job - 1;
    stage_rows(a.xsa, d.X, xs, L.ldx, row0, B);
    __syncthreads();
    critic_rows<PREC, NBW>(a.crit[g], a.co, xs, L.ldx, d.X, smem, L, a.c1[g], a.c2[g], a.q[g], row0, B);
  } else {  // policy on s for the actor update (algo_sac.py:524-535 / algo_td3.py:507-515)
    stage_rows(a.s, d.S, xs, L.ldx, row0, B);
    __syncthreads();
    for (int e = threadIdx.x; e < R * d.S; e += blockDim.x) {
      const int r = e / d.S, k = e % d.S;
      if (row0 + r < B) a.xsan[(int64_t)(row0 + r) * d.X + k] = xs[r * L.ldx + k];
    }
    actor_rows<PREC, NBW>(a.actor, a.ao, d, a.smp, xs, L.ldx, smem, L, a.h1a, a.h2a, a.a_mode, a.a_tag, a.eps_cur,
                          0.f, 0.f, 0, a.logp, a.save, a.xsan, row0, B);
  }
}

template <int PREC, int NBW>
__global__ void __launch_bounds__(256) qeval_rows_kernel(QEvalArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Lds L = lds_layout(a.d);
  float* xs = reinterpret_cast<float*>(smem + L.xs);
  const int row0 = blockIdx.x * R, g = blockIdx.y, B = a.d.B;
  stage_rows(a.x, a.d.X, xs, L.ldx, row0, B);
  __syncthreads();
  critic_rows<PREC, NBW>(a.crit[g], a.co, xs, L.ldx, a.d.X, smem, L, a.e1[g], a.e2[g], a.qn[g], row0, B);
}

// dh1 = (dh2 W2) * [h1 > 0] for the block's rows; dh2 already in the aT operand.
template <int PREC, int NBW>
__device__ void dh1_rows(const RowNet& net, const NetOff& o, const typename CT<PREC>::T* aT, int ldaT,
                         const float* h1, float* dh1_out, float* dh1_lds, int ldl, int row0, int B) {
  using T = typename CT<PREC>::T;
  const int H1 = o.h1, H1p = pad32(H1), H2p = pad32(o.h2);
  f32x4 acc[NBW];
  mfma_rows<PREC, NBW>(aT, ldaT, static_cast<const T*>(net.wt), H2p, H2p, H1p / 16, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int nb = wave + 4 * i;
    if (nb < H1p / 16) {
      const int col = nb * 16 + (lane & 15);
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int r = 4 * (lane >> 4) + rg, b = row0 + r;
        float v = 0.f;
        if (col < H1 && b < B) v = h1[(int64_t)b * H1 + col] > 0.f ? acc[i][rg] : 0.f;
        if (dh1_out && col < H1 && b < B) dh1_out[(int64_t)b * H1 + col] = v;
        if (dh1_lds) dh1_lds[r * ldl + col] = v;
      }
    }
  }
}

// dh2 = dq[b] * w3 * [h2 > 0] -> aT operand (T) and HBM (nullable)
template <int PREC>
__device__ void dh2_from_q(const float* p, const NetOff& o, const float* dq, const float* h2,
                           typename CT<PREC>::T* aT, int ldaT, float* dh2_out, float* rowv, int row0, int B) {
  const int H2 = o.h2, H2p = pad32(H2);
  if (threadIdx.x < R) rowv[threadIdx.x] = row0 + (int)threadIdx.x < B ? dq[row0 + threadIdx.x] : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < H2p; c += blockDim.x) {
    const float w = c < H2 ? p[o.w3 + c] : 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int b = row0 + r;
      float v = 0.f;
      if (c < H2 && b < B) v = h2[(int64_t)b * H2 + c] > 0.f ? rowv[r] * w : 0.f;
      aT[r * ldaT + c] = CT<PREC>::cvt(v);
      if (dh2_out && c < H2 && b < B) dh2_out[(int64_t)b * H2 + c] = v;
    }
  }
  __syncthreads();
}

template <int PREC, int NBW>
__global__ void __launch_bounds__(256) cbwd_rows_kernel(CBwdArgs a) {
  using T = typename CT<PREC>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Lds L = lds_layout(a.d);
  T* aT = reinterpret_cast<T*>(smem + L.aT);
  float* rowv = reinterpret_cast<float*>(smem + L.rowv);
  const int row0 = blockIdx.x * R, g = blockIdx.y, B = a.d.B;
  dh2_from_q<PREC>(a.crit[g].p, a.co, a.dq[g], a.c2[g], aT, L.ldaT, a.dc2[g], rowv, row0, B);
  dh1_rows<PREC, NBW>(a.crit[g], a.co, aT, L.ldaT, a.c1[g], a.dc1[g], nullptr, 0, row0, B);
}

// Actor data-gradients (autograd of algo_sac.py:524-562 through
// networks_sac.py:163-178; algo_td3.py:507-523 through networks_td3.py:91).
template <int PREC, int NBW>
__global__ void __launch_bounds__(256) abwd_rows_kernel(ABwdArgs a) {
  using T = typename CT<PREC>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowDims& d = a.d;
  const Lds L = lds_layout(d);
  T* aT = reinterpret_cast<T*>(smem + L.aT);
  float* h1s = reinterpret_cast<float*>(smem + L.h1s);
  float* hout = reinterpret_cast<float*>(smem + L.hout);  // dL/da per row
  float* ghs = reinterpret_cast<float*>(smem + L.ghs);
  float* rowv = reinterpret_cast<float*>(smem + L.rowv);
  const int row0 = blockIdx.x * R, B = d.B, S = d.S, A = d.A, X = d.X;
  const bool sac = d.algo == RLMD_SAC;
  // dL/da = sum over critics of (dq_g through critic g to its action inputs)
  for (int g = 0; g < a.nq; ++g) {
    dh2_from_q<PREC>(a.crit[g].p, a.co, a.dqn[g], a.e2[g], aT, L.ldaT, nullptr, rowv, row0, B);
    dh1_rows<PREC, NBW>(a.crit[g], a.co, aT, L.ldaT, a.e1[g], nullptr, h1s, L.ldh1, row0, B);
    __syncthreads();
    row_dots(h1s, L.ldh1, d.H1, A, a.crit[g].p + a.co.w1 + S, nullptr, A, 1, X, hout, kHeadsMax, g > 0);
    __syncthreads();
  }
  // through the sampling and the heads
  const int r = threadIdx.x;
  if (r < R) {
    const int b = row0 + r;
    if (b < B) {
      const float* sv = a.save + (int64_t)b * 5 * A;
      for (int j = 0; j < A; ++j) {
        const float da = hout[r * kHeadsMax + j];
        if (sac) {
          const float mu = sv[j], sigma = sv[A + j], eps = sv[2 * A + j], u = sv[3 * A + j];
          const float ls_raw = sv[4 * A + j];
          const float dlp = a.dlogp[b];
          const float t = tanhf(u);
          const float om = 1.f - t * t;
          const float dd = u - mu;
          const float dlogp_du = -dd / (sigma * sigma) + 2.f * t * om / (om + a.smp.reparam_noise);
          const float du = da * a.smp.max_action * om + dlp * dlogp_du;
          const float dmu = du + dlp * (dd / (sigma * sigma));
          const float dsig = du * eps + dlp * ((dd * dd) / (sigma * sigma * sigma) - 1.f / sigma);
          const bool live = ls_raw >= a.smp.ls_min && ls_raw <= a.smp.ls_max;
          const float dls = live ? dsig * sigma : 0.f;
          ghs[r * kHeadsMax + j] = dmu;
          ghs[r * kHeadsMax + A + j] = dls;
          a.gh[(int64_t)b * 2 * A + j] = dmu;
          a.gh[(int64_t)b * 2 * A + A + j] = dls;
        } else {
          const float t = tanhf(sv[j]);
          const float dpre = da * a.smp.max_action * (1.f - t * t);
          ghs[r * kHeadsMax + j] = dpre;
          a.gh[(int64_t)b * 2 * A + j] = dpre;
        }
      }
    } else {
      for (int j = 0; j < 2 * A; ++j) ghs[r * kHeadsMax + j] = 0.f;
    }
  }
  __syncthreads();
  // dh2 = (gh . [W_pi; W_ls]) * [h2 > 0]
  const NetOff& ao = a.ao;
  const int H2 = ao.h2, H2p = pad32(H2);
  const float* P = a.actor.p;
  for (int c = threadIdx.x; c < H2p; c += blockDim.x) {
    float acc[R];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) acc[rr] = 0.f;
    if (c < H2) {
      for (int j = 0; j < A; ++j) {
        const float wp = P[ao.w3 + (int64_t)j * H2 + c];
        const float wl = sac ? P[ao.w4 + (int64_t)j * H2 + c] : 0.f;
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
          acc[rr] = fmaf(ghs[rr * kHeadsMax + j], wp, acc[rr]);
          if (sac) acc[rr] = fmaf(ghs[rr * kHeadsMax + A + j], wl, acc[rr]);
        }
      }
    }
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      const int b = row0 + rr;
      float v = 0.f;
      if (c < H2 && b < B) v = a.h2a[(int64_t)b * H2 + c] > 0.f ? acc[rr] : 0.f;
      aT[rr * L.ldaT + c] = CT<PREC>::cvt(v);
      if (c < H2 && b < B) a.dh2[(int64_t)b * H2 + c] = v;
    }
  }
  __syncthreads();
  dh1_rows<PREC, NBW>(a.actor, ao, aT, L.ldaT, a.h1a, a.dh1, nullptr, 0, row0, B);
}

struct CopyJobs {
  CopyJob j[6];
};

template <int PREC>
__global__ void __launch_bounds__(256) w2_copy_kernel(CopyJobs jobs, int H1, int H2) {
  using T = typename CT<PREC>::T;
  const CopyJob j = jobs.j[blockIdx.y];
  const int H1p = pad32(H1), H2p = pad32(H2);
  T* wc = static_cast<T*>(j.wc);
  T* wt = static_cast<T*>(j.wt);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < H1 * H2; i += gridDim.x * blockDim.x) {
    const int n = i / H1, k = i - n * H1;
    const T v = CT<PREC>::cvt(j.w2[i]);
    wc[(int64_t)n * H1p + k] = v;
    wt[(int64_t)k * H2p + n] = v;
  }
}

template <int PREC>
int launch_all(const RowDims& d, int kind, const void* args, int ny, hipStream_t st) {
  const int H = d.H1p > d.H2p ? d.H1p : d.H2p;
  const dim3 grid((d.B + R - 1) / R, ny);
  const size_t lds = (size_t)lds_layout(d).total;
#define RLMD_ROWS_CASE(NBW)                                                                                     \
  switch (kind) {                                                                                               \
    case 0: hipLaunchKernelGGL((fwd_rows_kernel<PREC, NBW>), grid, dim3(256), lds, st,                          \
                               *static_cast<const FwdRowsArgs*>(args)); break;                                  \
    case 1: hipLaunchKernelGGL((qeval_rows_kernel<PREC, NBW>), grid, dim3(256), lds, st,                        \
                               *static_cast<const QEvalArgs*>(args)); break;                                    \
    case 2: hipLaunchKernelGGL((cbwd_rows_kernel<PREC, NBW>), grid, dim3(256), lds, st,                         \
                               *static_cast<const CBwdArgs*>(args)); break;                                     \
    default: hipLaunchKernelGGL((abwd_rows_kernel<PREC, NBW>), grid, dim3(256), lds, st,                        \
                                *static_cast<const ABwdArgs*>(args)); break;                                    \
  }
  if (H <= 64) {
    RLMD_ROWS_CASE(1)
  } else if (H <= 128) {
    RLMD_ROWS_CASE(2)
  } else if (H <= 256) {
    RLMD_ROWS_CASE(4)
  } else {
    RLMD_ROWS_CASE(8)
  }
#undef RLMD_ROWS_CASE
  RLMD_LAUNCH_CHECK();
  return 0;
}

int launch_rows(const RowDims& d, int kind, const void* args, int ny, hipStream_t st) {
  RLMD_CHECK(d.H1 <= 512 && d.H2 <= 512, "row kernels: hidden widths up to 512");
  RLMD_CHECK(d.A <= RLMD_MAX_ACTION, "row kernels: too many actions");
  if (d.B <= 0) return 0;
  return d.prec == RLMD_BF16 ? launch_all<RLMD_BF16>(d, kind, args, ny, st)
                             : launch_all<RLMD_FP32>(d, kind, args, ny, st);
}

}  // namespace

size_t rows_lds_bytes(const RowDims& d) { return (size_t)lds_layout(d).total; }

int fwd_rows_launch(const FwdRowsArgs& a, hipStream_t st) {
  return launch_rows(a.d, 0, &a, a.with_actor ? 4 : 3, st);
}
int qeval_rows_launch(const QEvalArgs& a, int nq, hipStream_t st) { return launch_rows(a.d, 1, &a, nq, st); }
int cbwd_rows_launch(const CBwdArgs& a, hipStream_t st) { return launch_rows(a.d, 2, &a, 2, st); }
int abwd_rows_launch(const ABwdArgs& a, hipStream_t st) { return launch_rows(a.d, 3, &a, 1, st); }

int w2_copies_launch(const CopyJob* jobs, int n, const RowDims& d, hipStream_t st) {
  RLMD_CHECK(n >= 1 && n <= 6, "bad copy job count");
  CopyJobs j{};
  for (int i = 0; i < 6; ++i) j.j[i] = jobs[i < n ? i : 0];
  const int blocks = (d.H1 * d.H2 + 255) / 256;
  const dim3 grid((unsigned)(blocks < 64 ? blocks : 64), (unsigned)n);
  if (d.prec == RLMD_BF16)
    hipLaunchKernelGGL(w2_copy_kernel<RLMD_BF16>, grid, dim3(256), 0, st, j, d.H1, d.H2);
  else
    hipLaunchKernelGGL(w2_copy_kernel<RLMD_FP32>, grid, dim3(256), 0, st, j, d.H1, d.H2);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd
