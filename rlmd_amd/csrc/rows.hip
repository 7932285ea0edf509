// rows.hip — row-block kernels of the SAC / TD3 update (gfx950, wave64).
//
// learn() (algos/algo_sac.py:300-615, algos/algo_td3.py:302-560) is a chain of
// small per-row MLP evaluations separated by a few batch-wide reductions.  Every
// per-row stretch of that chain runs here inside ONE 16-row workgroup of 8 waves,
// so intermediate activations never round-trip through a kernel boundary:
//   layer 1   VALU: thread = (hidden unit, row group), x rows broadcast from LDS
//   layer 2   v_mfma_f32_16x16x32_bf16 (bf16) / v_mfma_f32_16x16x4f32 (fp32):
//             A = the 16 activation rows in LDS, B = fc2.weight fragments read
//             16 bytes per lane straight from the zero-padded compute copy
//             (L2-resident, shared by every workgroup); wave w owns output column
//             blocks w, w + 8, ...
//   heads     reduced from the MFMA accumulators (lane shuffles + one LDS pass)
//   sampling  tanh-squashed N / Laplace / MVN policy, TD3 noise per row (rlmd_policy.h)
// Latency is the whole cost at these sizes (a few MFLOP per workgroup), so every
// load that does not depend on computed data — both nets' fc2 fragments, biases,
// head weights, fc1 rows, ReLU masks — is issued in ONE round at kernel start.
// Backward data paths use the transposed compute copy with the same MFMA loop.
// Weight gradients (batch reductions) are gemm.hip's BWD_W launch.
#include <math.h>

#include "learn_kernels.h"
#include "rlmd_block.h"
#include "rlmd_loss.h"
#include "rlmd_policy.h"
#include "rlmd_common.h"

namespace rlmd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int R = kRowBlock;  // rows per workgroup
constexpr int NT = 512;       // threads per workgroup
constexpr int NW = NT / 64;   // waves
constexpr int NHF = 4;        // heads reduced in the MFMA epilogue (more -> LDS dot products)
constexpr int W1P = 8;        // fc1 inputs preloaded per thread (more -> read in the loop)
constexpr int kHeadsMax = 2 * RLMD_MAX_ACTION;
#ifndef RLMD_FWD_DEFER
#define RLMD_FWD_DEFER 1  // fwd_rows: a job's second fragment stream issued after its first net's layer 2
#endif
#ifndef RLMD_L1_BATCH
#define RLMD_L1_BATCH 1  // row kernels' layer 1: a batch of rows' inputs read from LDS together
#endif
#ifndef RLMD_SAMPLE_NL
#define RLMD_SAMPLE_NL 1  // fwd_rows: load-free policy sampling on the production path (sample_rows<true>)
#endif

#ifdef RLMD_TIMING
// experiment builds only (tools/ts_probe.py): thread-0 s_memtime checkpoints of
// workgroup (0, y) — slots [16 y, 16 y + 16) for fwd jobs, 96.. for abwd
__device__ unsigned long long g_ts_rows[128];
#define RLMD_TSR(i)                                                                      \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_ts_rows[i] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// job windows (constant-rate clock, comparable across workgroups): block x = 0
#define RLMD_TSJ(i)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_ts_rows[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define RLMD_TSJ(i) \
  do {              \
  } while (0)
#define RLMD_TSR(i) \
  do {              \
  } while (0)
#endif

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
  __device__ __forceinline__ static T cvt(float f) { return to_bf16(f); }
  __device__ __forceinline__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct CT<RLMD_FP32> {
  using T = float;
  using Frag = f32x4;
  static constexpr int KS = 16;
  __device__ __forceinline__ static T cvt(float f) { return f; }
  // lane group q = lane >> 4 holds k = k0 + 4q + j in element j: four 16x16x4
  // MFMAs cover k0 .. k0 + 15 (a permutation of the k order, same products)
  __device__ __forceinline__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  }
};

// ---------------------------------------------------------------------------
// LDS carve-up, identical on host (launch size) and device.
// ---------------------------------------------------------------------------
struct Lds {
  int xs, a1, aT, h2s, part, hout, ghs, rowv, vkey, vval, runs, rank, red, aU, m1s, total;  // byte offsets
  int ldx, lda1, ldaT, ldh2;                                    // row pitches (elements)
};
__host__ __device__ inline Lds lds_layout(const RowDims& d) {
  const int ts = d.prec == RLMD_BF16 ? 2 : 4;
  const int pad = d.prec == RLMD_BF16 ? 8 : 4;  // rows stay 16-B aligned, banks staggered
  const int hmax = d.H1p > d.H2p ? d.H1p : d.H2p;
  Lds l{};
  auto up = [](int v) { return (v + 15) & ~15; };
  int o = 0;
  l.ldx = d.X > W1P ? d.X : W1P;  // >= W1P: layer 1 reads W1P columns unconditionally (zero padded)
  l.xs = o;
  o = up(o + R * l.ldx * 4);
  l.lda1 = hmax + pad;  // A operand of the forward (h1) and backward (dh2) MFMAs
  l.a1 = o;
  o = up(o + R * l.lda1 * ts);
  l.ldaT = l.lda1;
  l.aT = l.a1;
  l.ldh2 = hmax + 4;  // f32 rows for LDS dot products (many heads / actions)
  l.h2s = o;
  o = up(o + R * l.ldh2 * 4);
  l.part = o;  // per-wave head partials [NW][R][NHF]
  o = up(o + NW * R * NHF * 4);
  l.hout = o;  // [R][kHeadsMax]
  o = up(o + R * kHeadsMax * 4);
  l.ghs = o;  // [R][kHeadsMax]
  o = up(o + R * kHeadsMax * 4);
  l.rowv = o;  // [R][4]
  o = up(o + R * 4 * 4);
  l.vkey = o;  // actor loss: every row's ranking key [B] (abwd)
  o = up(o + d.B * 8);
  l.vval = o;  // and its objective v [B]
  o = up(o + d.B * 4);
  l.runs = o;  // loss workgroups: block_rank runs [NT], ranks [3][NT], reductions
  o = up(o + NT * 8);
  l.rank = o;
  o = up(o + 3 * NT * 4);
  l.red = o;
  o = up(o + 16 * 9 * 4);
  l.aU = o;  // A operand of the backward-basis pass (fwd U = (m2 w3) W2), pitch lda1
  o = up(o + R * l.lda1 * ts);
  l.m1s = o;  // layer-1 ReLU mask bytes [R][hmax] (f32 h1 > 0)
  o = up(o + R * hmax);
  l.total = o;
  return l;
}

// ---------------------------------------------------------------------------
// fc2 fragments: Pre holds K-steps [0, G) of one net, issued early; mfma_rows
// consumes it (and streams the rest in G-step groups when MULTI).
// ---------------------------------------------------------------------------
template <int PREC, int NBW, bool MULTI>
struct Pre {
  // 16 fragments (64 VGPRs) per lane when one group covers K; 8 per group (two
  // groups in flight) when the K loop streams
  static constexpr int G = (MULTI ? 8 : 16) / NBW;
  typename CT<PREC>::Frag f[G][NBW];
};

template <int PREC, int NBW, bool MULTI>
using FragArr = typename CT<PREC>::Frag[Pre<PREC, NBW, MULTI>::G][NBW];

template <int PREC, int NBW, bool MULTI>
__device__ __forceinline__ void frag_load(FragArr<PREC, NBW, MULTI>& f,
                                          const typename CT<PREC>::T* Bg, int ldb, int s0, int nsteps, int nblk,
                                          int nb0 = 0) {
  constexpr int G = Pre<PREC, NBW, MULTI>::G;
  constexpr int EPF = 16 / sizeof(typename CT<PREC>::T);
  constexpr int TS = sizeof(typename CT<PREC>::T);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // fragment-major copy (frag_index): block (band nb, step s) at ((nb * nS + s) * 64 + lane) * EPF;
  // this workgroup's bands are nb0 .. nb0 + nblk - 1 (a column split of the output)
  const int nS = ldb / CT<PREC>::KS;
  const uint32_t base = (uint32_t)(((nb0 + wave) * nS * 64 + lane) * EPF);
  const __amdgpu_buffer_rsrc_t rs = rlmd_rsrc(Bg, (int64_t)(nb0 + nblk) * 16 * ldb * TS);
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const bool ok = wave + NW * i < nblk && s0 + g < nsteps;
      const uint32_t e = base + (uint32_t)((NW * i * nS + s0 + g) * 64 * EPF);
      f[g][i] = __builtin_bit_cast(typename CT<PREC>::Frag,
                                   __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (int)(e * TS) : 0x7fffffff, 0, 0));
    }
}

// K-steps [ks0, K / KS) of output bands nb0 .. nb0 + nblk - 1 (a K split: ks0 > 0
// with K short of the full depth; a column split: nb0 > 0 with fewer bands)
template <int PREC, int NBW, bool MULTI>
__device__ __forceinline__ void pre_issue(Pre<PREC, NBW, MULTI>& p, const void* Bg, int ldb, int K, int nblk,
                                          int nb0 = 0, int ks0 = 0) {
  frag_load<PREC, NBW, MULTI>(p.f, static_cast<const typename CT<PREC>::T*>(Bg), ldb, ks0, K / CT<PREC>::KS, nblk,
                              nb0);
}

template <int PREC, int NBW, bool MULTI>
__device__ __forceinline__ void frag_mfma(const FragArr<PREC, NBW, MULTI>& f,
                                          const typename CT<PREC>::T* As, int lda, int s0, int nsteps, int nblk,
                                          f32x4 (&acc)[NBW]) {
  constexpr int G = Pre<PREC, NBW, MULTI>::G;
  constexpr int EPF = 16 / sizeof(typename CT<PREC>::T);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int aoff = (lane & 15) * lda + EPF * (lane >> 4);
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (s0 + g < nsteps) {
      const typename CT<PREC>::Frag a =
          *reinterpret_cast<const typename CT<PREC>::Frag*>(As + aoff + (s0 + g) * CT<PREC>::KS);
#pragma unroll
      for (int i = 0; i < NBW; ++i)
        if (wave + NW * i < nblk) CT<PREC>::mfma(a, f[g][i], acc[i]);
    }
  }
}

// acc[i] = A[16 x K] B^T for output column block nb = wave + 8 i (A: LDS rows of
// pitch lda; B: compute copy, one row of K elements per output column, pitch ldb).
// ks0: the first K-step (pre issued with the same origin); K / KS the end
template <int PREC, int NBW, bool MULTI>
__device__ __forceinline__ void mfma_rows(Pre<PREC, NBW, MULTI>& pre, const typename CT<PREC>::T* As, int lda,
                                          const void* Bv, int ldb, int K, int nblk, f32x4 (&acc)[NBW],
                                          int nb0 = 0, int ks0 = 0) {
  constexpr int G = Pre<PREC, NBW, MULTI>::G;
  const auto* Bg = static_cast<const typename CT<PREC>::T*>(Bv);
  const int nsteps = K / CT<PREC>::KS;
#pragma unroll
  for (int i = 0; i < NBW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (!MULTI) {
    (void)Bg;
    frag_mfma<PREC, NBW, MULTI>(pre.f, As, lda, ks0, nsteps, nblk, acc);
  } else {
    FragArr<PREC, NBW, MULTI> b1;
    for (int s = ks0; s < nsteps; s += 2 * G) {
      frag_load<PREC, NBW, MULTI>(b1, Bg, ldb, s + G, nsteps, nblk, nb0);
      frag_mfma<PREC, NBW, MULTI>(pre.f, As, lda, s, nsteps, nblk, acc);
      frag_load<PREC, NBW, MULTI>(pre.f, Bg, ldb, s + 2 * G, nsteps, nblk, nb0);
      frag_mfma<PREC, NBW, MULTI>(b1, As, lda, s + G, nsteps, nblk, acc);
    }
  }
}

// ---------------------------------------------------------------------------
// element maps
// ---------------------------------------------------------------------------
// [16 x Hp] elementwise work: thread -> (column c, rows [r0, r1))
struct ElemMap {
  int c, r0, r1;
};
__device__ __forceinline__ ElemMap elem_map(int Hp) {
  const int tpc = NT / Hp > 0 ? NT / Hp : 1;
  const int nr = (R + tpc - 1) / tpc;
  const int grp = threadIdx.x / Hp;
  ElemMap m;
  m.c = threadIdx.x % Hp;
  m.r0 = grp < tpc ? grp * nr : R;
  m.r1 = m.r0 + nr < R ? m.r0 + nr : R;
  return m;
}

// rows per thread of a [16 x Hp] elementwise map, Hp <= 128 NBW: 16 / (512 / Hp) <= 4 NBW
template <int NBW>
constexpr int kMR = 4 * NBW < R ? 4 * NBW : R;

// MFMA accumulator element (i, rg) of this lane: column and row
__device__ __forceinline__ int acc_col(int i, int nb0 = 0) {
  return (nb0 + (threadIdx.x >> 6) + NW * i) * 16 + (threadIdx.x & 15);
}
__device__ __forceinline__ int acc_row(int rg) { return 4 * ((threadIdx.x & 63) >> 4) + rg; }

// ---------------------------------------------------------------------------
// forward pieces
// ---------------------------------------------------------------------------
// per-thread constants of one net's forward, loaded before any compute
template <int NBW>
struct FwdConst {
  float w1[W1P], b1;    // fc1 row of this thread's hidden unit
  float b2[NBW];        // fc2 bias of this lane's accumulator columns
  float hw[NBW][NHF];   // head weights of those columns (nh <= NHF)
};

template <int NBW>
__device__ __forceinline__ void fwd_const(FwdConst<NBW>& k, const float* p, const NetOff& o, int in, int nh,
                                          const float* wa, const float* wb, int na, int nb0 = 0) {
  const ElemMap m = elem_map(pad32(o.h1));
  const bool own = m.c < o.h1 && m.r0 < R;
  const __amdgpu_buffer_rsrc_t rp = rlmd_rsrc(p, o.size * 4);
  // j < in and h < nh are uniform: skipped loads are not issued (a wave holds at
  // most 63 loads in flight, and the first load round is at that limit)
  // the fc1 row (in <= 8 contiguous floats) as one or two 16-B loads: a wave's
  // 64 consecutive units are one 1.5 KB span, and per-float loads touched its
  // cache lines once per input (the load round is bound by line accesses)
  {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int off = (int)((o.w1 + (int64_t)m.c * in) * 4);
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rp, own ? off : 0x7fffffff, 0, 0);
    u32x4 hi = u32x4{0u, 0u, 0u, 0u};
    if (in > 4) hi = __builtin_amdgcn_raw_buffer_load_b128(rp, own ? off + 16 : 0x7fffffff, 0, 0);
#pragma unroll
    for (int j = 0; j < W1P; ++j)
      k.w1[j] = j < in ? __builtin_bit_cast(float, j < 4 ? lo[j & 3] : hi[j & 3]) : 0.f;
  }
  k.b1 = rlmd_ldf(rp, o.b1 + m.c, own);
  const int64_t oa = wa - p, ob = (wb ? wb : wa) - p;  // head rows relative to p
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int col = acc_col(i, nb0);
    const bool cin = col < o.h2;
    k.b2[i] = rlmd_ldf(rp, o.b2 + col, cin);
#pragma unroll
    for (int h = 0; h < NHF; ++h) {
      const int64_t row = h < na ? oa + (int64_t)h * o.h2 : ob + (int64_t)(h - na) * o.h2;
      k.hw[i][h] = h < nh ? rlmd_ldf(rp, row + col, cin) : 0.f;
    }
  }
}

// ReLU masks as bytes in the layouts their consumers read (one wide load each):
//   m1 [row block][band][lane][4]: the MFMA accumulator layout over H1p (dh1) —
//      a lane's 4 rows of one column are one 4-byte word;
//   m2 [row block][column][16 rows]: the elementwise map over H2p (dh2) — a
//      thread's kMR consecutive rows are kMR contiguous bytes.
__device__ __forceinline__ int64_t m1_index(int rb, int H1p, int row, int col) {
  return ((((int64_t)rb * (H1p >> 4) + (col >> 4)) * 64 + (col & 15) + 16 * ((row & 15) >> 2)) << 2) + (row & 3);
}
__device__ __forceinline__ int64_t m2_index(int rb, int H2p, int row, int col) {
  return (((int64_t)rb * H2p + col) << 4) + (row & 15);
}

// Row-packed operands of the weight-gradient tiles (update.hip): element (b, c)
// of a [B x Hp] matrix at ((b / 16) * Hp + c) * 16 + b % 16, so the 8 (bf16) or
// 4 (f32) consecutive mini-batch rows an MFMA fragment lane holds along K are
// one contiguous 16-byte run.
__device__ __forceinline__ int64_t rp_index(int rb, int Hp, int row, int col) {
  return (((int64_t)rb * Hp + col) << 4) + (row & 15);
}

// Extra outputs of one net's forward for the fused update kernels (nullable
// members: not written): h1 / h2 row-packed in the compute type; the layer-1
// mask bytes (LDS) and the A operand of the backward-basis pass (LDS).
template <int PREC>
struct FwdExtra {
  typename CT<PREC>::T* hp1;
  typename CT<PREC>::T* hp2;
  uint8_t* m1s;
  typename CT<PREC>::T* aU;  // critic basis pass A operand ([h2 > 0] w3), written in the epilogue
};

// A thread's nr consecutive rows [r0, r0 + nr) of one column, contiguous in the
// row-packed layout (element idx = rp_index(rb, Hp, r0, c); r0 a multiple of nr,
// nr in {1, 2, 4, 8, 16}): stored with the widest buffer stores that cover them.
template <int PREC, int MR>
__device__ __forceinline__ void store_rp_rows(typename CT<PREC>::T* base, int64_t idx, const typename CT<PREC>::T (&v)[MR],
                                              int nr) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  constexpr int TS = sizeof(typename CT<PREC>::T);
  const __amdgpu_buffer_rsrc_t rs = rlmd_rsrc_wave(base, 0x7fffffff);
  const int off = (int)(idx * TS);
  uint32_t w[(MR * TS + 3) / 4];
  if constexpr (PREC == RLMD_BF16) {
#pragma unroll
    for (int k = 0; k < (MR + 1) / 2; ++k) w[k] = (uint32_t)v[2 * k] | (2 * k + 1 < MR ? (uint32_t)v[2 * k + 1] << 16 : 0u);
  } else {
#pragma unroll
    for (int k = 0; k < MR; ++k) w[k] = __float_as_uint(v[k]);
  }
  const int nw = nr * TS / 4;  // whole words (0: one bf16 row)
  if (nw >= 4) {
#pragma unroll
    for (int q = 0; q < (MR * TS) / 16; ++q)
      if (4 * q < nw)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]}, rs, off + 16 * q,
                                               0, RLMD_WT_AUX);
  } else if (nw == 2) {
    if constexpr ((MR * TS) / 4 >= 2) __builtin_amdgcn_raw_buffer_store_b64(u32x2{w[0], w[1]}, rs, off, 0, RLMD_WT_AUX);
  } else if (nw == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(w[0], rs, off, 0, RLMD_WT_AUX);
  } else {
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)w[0], rs, off, 0, RLMD_WT_AUX);
  }
}

// h1 = relu(x W1^T + b1): A operand (T, zero-padded to H1p) + f32 to HBM (nullable)
template <int PREC, int NBW>
__device__ __forceinline__ void layer1(const FwdConst<NBW>& k, const float* p, const NetOff& o, const float* xs,
                                       int ldx, int in, typename CT<PREC>::T* a1, int lda1, float* h1_out,
                                       uint8_t* m1_out, int row0, int B, const FwdExtra<PREC>* ex = nullptr) {
  constexpr int MR = kMR<NBW>;
  const int H1 = o.h1, H1p = pad32(H1);
  const ElemMap m = elem_map(H1p);
  const int nr = m.r1 - m.r0;
  const float* w = p + o.w1 + (int64_t)m.c * in;
  uint64_t mk[(MR + 7) / 8] = {};  // the thread's mask bytes, row r0 + rr at byte rr
  // row r0 + rr's unit: relu(acc + b1) into the A operand, h1_out, the mask bytes
  auto emit = [&](int rr, float acc) {
    const int r = m.r0 + rr;
    float v = 0.f;
    if (m.c < H1) {
      v = fmaxf(acc + k.b1, 0.f);
      if (h1_out && row0 + r < B) h1_out[(int64_t)(row0 + r) * H1 + m.c] = v;
    }
    a1[r * lda1 + m.c] = CT<PREC>::cvt(v);
    if (ex && ex->m1s) ex->m1s[r * H1p + m.c] = v > 0.f ? 1 : 0;
    const uint64_t bit = (uint64_t)(v > 0.f ? 1u : 0u) << (8 * (rr & 7));
    if constexpr (MR > 8) {
      if (rr < 8) mk[0] |= bit;
      else mk[1] |= bit;
    } else {
      mk[0] |= bit;
    }
  };
  if (RLMD_L1_BATCH && in <= W1P && (ldx & 3) == 0) {
    // every input in registers (k.w1, zero past in): a batch of rows' xs as 16-byte
    // LDS reads issued together, then their dots (j ascending, as below).  The
    // per-row loop waited one LDS round trip per row, its bounds being run-time.
    constexpr int LB = MR < 8 ? MR : 8;
    static_assert(W1P == 8, "the batched dots below read 8 inputs per row");
#pragma unroll
    for (int b0 = 0; b0 < MR; b0 += LB) {
      float4 xv[LB][2];
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        const int r = m.r0 + b0 + i < R ? m.r0 + b0 + i : R - 1;  // rows past this thread's: read, unused
        xv[i][0] = *reinterpret_cast<const float4*>(xs + r * ldx);
        xv[i][1] = *reinterpret_cast<const float4*>(xs + r * ldx + 4);
      }
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        if (b0 + i < nr) {
          float acc = 0.f;
          acc = fmaf(xv[i][0].x, k.w1[0], acc);
          acc = fmaf(xv[i][0].y, k.w1[1], acc);
          acc = fmaf(xv[i][0].z, k.w1[2], acc);
          acc = fmaf(xv[i][0].w, k.w1[3], acc);
          acc = fmaf(xv[i][1].x, k.w1[4], acc);
          acc = fmaf(xv[i][1].y, k.w1[5], acc);
          acc = fmaf(xv[i][1].z, k.w1[6], acc);
          acc = fmaf(xv[i][1].w, k.w1[7], acc);
          emit(b0 + i, acc);
        }
      }
    }
  } else {
    for (int r = m.r0; r < m.r1; ++r) {
      float acc = 0.f;
      if (m.c < H1) {
        // xs rows are zero padded to ldx >= W1P and k.w1[j] = 0 for j >= in: no branch
        // between the LDS reads, so a row's W1P reads issue together
#pragma unroll
        for (int j = 0; j < W1P; ++j) acc = fmaf(xs[r * ldx + j], k.w1[j], acc);
        for (int j = W1P; j < in; ++j) acc = fmaf(xs[r * ldx + j], w[j], acc);
      }
      emit(r - m.r0, acc);
    }
  }
  if (m.r0 < R) {
    // the mask bytes: one word per 4 rows (m1_index keeps rows 4q..4q+3 of a column together)
    if (m1_out) {
      if (nr >= 4) {
#pragma unroll
        for (int q = 0; q < MR / 4; ++q)
          if (4 * q < nr)
            rlmd_st_wt(reinterpret_cast<uint32_t*>(m1_out + m1_index(row0 / R, H1p, m.r0 + 4 * q, m.c)),
                       (uint32_t)(mk[q / 2] >> (32 * (q & 1))));
      } else {
#pragma unroll
        for (int rr = 0; rr < (MR < 2 ? MR : 2); ++rr)
          if (rr < nr) m1_out[m1_index(row0 / R, H1p, m.r0 + rr, m.c)] = (uint8_t)(mk[0] >> (8 * rr));
      }
    }
    if (ex && ex->hp1) {
      // h1 in the compute type as the A operand holds it (this thread's own LDS
      // writes), rows past B zero, packed into the row-packed layout
      typename CT<PREC>::T hz[MR];
#pragma unroll
      for (int rr = 0; rr < MR; ++rr)
        hz[rr] = (rr < nr && row0 + m.r0 + rr < B) ? a1[(m.r0 + rr) * lda1 + m.c] : typename CT<PREC>::T(0);
      store_rp_rows<PREC, MR>(ex->hp1, rp_index(row0 / R, H1p, m.r0, m.c), hz, nr);
    }
  }
}

// relu(acc + b2) -> HBM (nullable), LDS rows (nullable) and the per-wave head
// partials part[wave][row][h] (nh <= NHF).
template <int NBW, int PREC = RLMD_BF16>
__device__ __forceinline__ void fwd_epilogue(const f32x4 (&acc)[NBW], const FwdConst<NBW>& k, const NetOff& o,
                                             int nh, float* h2_out, uint8_t* m2_out, float* h2s, int ldh2,
                                             float* part, int row0, int B, const FwdExtra<PREC>* ex = nullptr,
                                             int lda1 = 0, int nb0 = 0, int nbw = 0) {
  // output bands nb0 .. nb0 + nbw - 1 (a column split; nbw = 0: all of them)
  const int H2 = o.h2, nblk = nbw ? nbw : pad32(H2) / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float ph[4][NHF];
#pragma unroll
  for (int rg = 0; rg < 4; ++rg)
#pragma unroll
    for (int h = 0; h < NHF; ++h) ph[rg][h] = 0.f;
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    if (wave + NW * i < nblk) {
      const int col = acc_col(i, nb0);
      const bool cin = col < H2;
      uint32_t mw = 0;
      typename CT<PREC>::T hz[4];
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int r = acc_row(rg);
        const float v = cin ? fmaxf(acc[i][rg] + k.b2[i], 0.f) : 0.f;
        if (h2_out && cin && row0 + r < B) h2_out[(int64_t)(row0 + r) * H2 + col] = v;
        if (h2s) h2s[r * ldh2 + col] = v;
        // critic basis pass A operand: [h2 > 0] * w3 (the head weight of this column)
        if (ex && ex->aU) ex->aU[r * lda1 + col] = CT<PREC>::cvt(v > 0.f ? k.hw[i][0] : 0.f);
        hz[rg] = CT<PREC>::cvt(row0 + r < B ? v : 0.f);
        mw |= (v > 0.f ? 1u : 0u) << (8 * rg);
#pragma unroll
        for (int h = 0; h < NHF; ++h) ph[rg][h] = fmaf(v, k.hw[i][h], ph[rg][h]);
      }
      if (m2_out) rlmd_st_wt(reinterpret_cast<uint32_t*>(m2_out + m2_index(row0 / R, pad32(H2), acc_row(0), col)), mw);
      // the lane's 4 rows of h2, contiguous in the row-packed layout
      if (ex && ex->hp2) store_rp_rows<PREC, 4>(ex->hp2, rp_index(row0 / R, pad32(H2), acc_row(0), col), hz, 4);
    }
  }
  if (nh <= NHF) {
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
      for (int h = 0; h < NHF; ++h) {
        if (h < nh) {
          const float c = rlmd_row16_sum(ph[rg][h]);
          if ((lane & 15) == 0) part[(wave * R + acc_row(rg)) * NHF + h] = c;
        }
      }
  }
}

// sum of the per-wave head partials of row r, head h
__device__ __forceinline__ float head_sum(const float* part, int r, int h) {
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) s += part[(w * R + r) * NHF + h];
  return s;
}

// out[r][h] (+)= sum_c src[r][c] * w_h[c * cstride], h < nh, w_h = wa + h*ldw for
// h < na, wb + (h - na)*ldw beyond.  A dot is split over P lanes of one wave.
__device__ void row_dots(const float* src, int lds, int ncols, int nh, const float* wa, const float* wb, int na,
                         int64_t ldw, int cstride, float* out, int ldo, bool accumulate) {
  const int nd = R * nh;
  int P = 64;
  while (P > 1 && nd * P > NT) P >>= 1;
  const int part = threadIdx.x % P;
  for (int d0 = threadIdx.x / P; d0 < nd; d0 += NT / P) {
    const int h = d0 / R, r = d0 % R;
    const float* w = h < na ? wa + (int64_t)h * ldw : wb + (int64_t)(h - na) * ldw;
    float acc = 0.f;
    for (int c = part; c < ncols; c += P) acc = fmaf(src[r * lds + c], w[(int64_t)c * cstride], acc);
    for (int off = P >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (part == 0) out[r * ldo + h] = accumulate ? out[r * ldo + h] + acc : acc;
  }
}

struct NoHook {
  __device__ void operator()() const {}
};

// One 2-hidden-layer MLP forward over the block's rows (x in LDS), heads left in
// hout[r][h] (no head bias).  pre: this net's fc2 fragments, already issued.
// after_l2 runs right after layer 2's MFMAs, once pre's registers are free: a
// job issues its NEXT fragment stream there, under this net's epilogue, instead
// of with the first load round, where it queued behind (and delayed) this one.
template <int PREC, int NBW, bool MULTI, typename Hook = NoHook>
__device__ __forceinline__ void mlp_rows(const RowNet& net, const NetOff& o, const FwdConst<NBW>& k, Pre<PREC, NBW, MULTI>& pre,
                         const float* xs, int ldx, int in, int nh, const float* wa, const float* wb, int na,
                         unsigned char* smem, const Lds& L, float* h1_out, float* h2_out, int row0, int B,
                         uint8_t* m1_out = nullptr, uint8_t* m2_out = nullptr, const FwdExtra<PREC>* ex = nullptr,
                         int nb0 = 0, int nbw = 0, Hook after_l2 = Hook(), int ts = -1) {
  using T = typename CT<PREC>::T;
  T* a1 = reinterpret_cast<T*>(smem + L.a1);
  float* part = reinterpret_cast<float*>(smem + L.part);
  float* hout = reinterpret_cast<float*>(smem + L.hout);
  float* h2s = reinterpret_cast<float*>(smem + L.h2s);
  (void)ts;  // job 0's stamps (RLMD_TIMING builds): slots ts .. ts + 4
  layer1<PREC, NBW>(k, net.p, o, xs, ldx, in, a1, L.lda1, h1_out, m1_out, row0, B, ex);
  if (blockIdx.y == 2) RLMD_TSR(63);
  if (blockIdx.y == 4) RLMD_TSR(87);
  if (blockIdx.y == 0 && ts >= 0) RLMD_TSR(ts);
  __syncthreads();
  if (blockIdx.y == 2) RLMD_TSR(64);
  if (blockIdx.y == 4) RLMD_TSR(88);
  if (blockIdx.y == 0 && ts >= 0) RLMD_TSR(ts + 1);
  f32x4 acc[NBW];
  const int H1p = pad32(o.h1);
  mfma_rows<PREC, NBW, MULTI>(pre, a1, L.lda1, net.wc, H1p, H1p, nbw ? nbw : pad32(o.h2) / 16, acc, nb0);
  after_l2();
  if (blockIdx.y == 2) RLMD_TSR(65);
  if (blockIdx.y == 4) RLMD_TSR(89);
  if (blockIdx.y == 0 && ts >= 0) RLMD_TSR(ts + 2);
  const bool fused = nh <= NHF;
  fwd_epilogue<NBW, PREC>(acc, k, o, nh, h2_out, m2_out, fused ? nullptr : h2s, L.ldh2, part, row0, B, ex, L.lda1,
                          nb0, nbw);
  if (blockIdx.y == 2) RLMD_TSR(66);
  if (blockIdx.y == 4) RLMD_TSR(90);
  if (blockIdx.y == 0 && ts >= 0) RLMD_TSR(ts + 3);
  __syncthreads();
  if (blockIdx.y == 2) RLMD_TSR(67);
  if (blockIdx.y == 4) RLMD_TSR(91);
  if (blockIdx.y == 0 && ts >= 0) RLMD_TSR(ts + 4);
  if (fused) {
    if ((int)threadIdx.x < R * nh) {
      const int r = threadIdx.x % R, h = threadIdx.x / R;
      hout[r * kHeadsMax + h] = head_sum(part, r, h);
    }
  } else {
    row_dots(h2s, L.ldh2, o.h2, nh, wa, wb, na, o.h2, 1, hout, kHeadsMax, false);
  }
  __syncthreads();
}

// Head biases of the policy for A <= 2, loaded by the sampling threads with the
// kernel's first load round: read at sampling time they would wait behind the
// whole fragment stream (vmcnt retires in issue order).
struct HeadBias {
  float mu[2], ls[2];
};
__device__ __forceinline__ HeadBias head_bias(const float* p, const NetOff& ao, const RowDims& d) {
  HeadBias hb{{0.f, 0.f}, {0.f, 0.f}};
  if ((int)threadIdx.x < R) {
    const __amdgpu_buffer_rsrc_t rp = rlmd_rsrc(p, ao.size * 4);
    const bool sac = d.algo == RLMD_SAC;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      hb.mu[j] = rlmd_ldf(rp, ao.b3 + j, j < d.A);
      hb.ls[j] = rlmd_ldf(rp, ao.b4 + j, sac && j < d.A);
    }
  }
  return hb;
}

// The policy noise of a row's first two components (Philox -> f64 Box-Muller /
// Laplace uniform), drawn at kernel start: it depends on nothing computed, and
// its f64 log / sincospi chain then overlaps the fragment loads instead of
// sitting between the two MLPs of the target path.
struct Noise2 {
  float v[2];
};
__device__ __forceinline__ Noise2 noise_pre(const SampleCfg& smp, const RowDims& d, int tag, int row0) {
  Noise2 n{{0.f, 0.f}};
  const int r = threadIdx.x;
  if (r < R && row0 + r < d.B) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      if (j < d.A) n.v[j] = policy_draw(smp.dist, smp.seed, (uint32_t)(row0 + r), smp.ctr, (uint32_t)tag, j);
  }
  return n;
}

// Policy sample per row from hout (mu | log_scale without biases): writes the
// action into xs[:, S:S+A] and xa_out (nullable).  Same arithmetic as
// learn.hip's actor_head_kernel.  mode 0 stochastic, 1 deterministic.  hb: the
// head biases preloaded (A <= 2) when has_hb, else read here.
// NL (no loads): the caller guarantees has_hb, A <= 2, eps_in == nullptr and has_nz
// (or mode 1): the body then issues no global load.  A load here is waited on
// with vmcnt(0) at its branch's merge, and vmcnt also counts every load and
// store issued before it — a deferred fragment stream (fwd_rows' target critic,
// issued under the policy's epilogue) or the write-through row-packed stores of
// the policy's h1 / h2 — so the sampling waited for all of them.
template <bool NL = false>
__device__ __forceinline__ void sample_rows(const float* p, const NetOff& ao, const RowDims& d, const SampleCfg& smp, float* xs,
                            int ldx, const float* hout, int mode, int tag, const float* eps_in, float noise_std,
                            float noise_clip, int clamp_noise, float* logp_out, float* save, float* xa_out, int row0,
                            int B, HeadBias hbv = HeadBias{{0.f, 0.f}, {0.f, 0.f}}, bool has_hb = false,
                            Noise2 nz2 = Noise2{{0.f, 0.f}}, bool has_nz = false) {
  const int r = threadIdx.x;
  if (r >= R) return;
  const int S = d.S, A = d.A, b = row0 + r;
  const bool valid = b < B, sac = d.algo == RLMD_SAC;
  const uint32_t c1 = smp.ctr;
  float lp_sum = 0.f, m2_sum = 0.f, hld_sum = 0.f, jac_sum = 0.f;
  const bool pre = NL || (has_hb && A <= 2);
  for (int j = 0; j < (NL ? 2 : A); ++j) {
    if (NL && j >= A) break;
    const float mu = hout[r * kHeadsMax + j] + (pre ? (j == 0 ? hbv.mu[0] : hbv.mu[1]) : (NL ? 0.f : p[ao.b3 + j]));
    float noise = 0.f;
    if (mode == 0 && valid) {
      if constexpr (NL)
        noise = j == 0 ? nz2.v[0] : nz2.v[1];
      else
        noise = eps_in ? eps_in[(int64_t)b * A + j]
                       : (has_nz && A <= 2 ? (j == 0 ? nz2.v[0] : nz2.v[1])
                                           : policy_draw(smp.dist, smp.seed, (uint32_t)b, c1, (uint32_t)tag, j));
    }
    float act;
    if (sac) {
      const float ls_raw =
          hout[r * kHeadsMax + A + j] + (pre ? (j == 0 ? hbv.ls[0] : hbv.ls[1]) : (NL ? 0.f : p[ao.b4 + j]));
      const PolicyComp pc = policy_comp(smp.dist, mu, ls_raw, noise, smp.ls_min, smp.ls_max);
      if (mode == 1) {
        act = tanhf(pc.mu) * smp.max_action;
      } else {
        act = tanhf(pc.u) * smp.max_action;
        const float an = act / smp.max_action;
        lp_sum += pc.lp;
        m2_sum += pc.m2;
        hld_sum += pc.hld;
        jac_sum += logf(1.f - an * an + smp.reparam_noise);
        if (save && valid) {
          float* sv = save + (int64_t)b * 5 * A;
          sv[j] = pc.mu;
          sv[A + j] = pc.sigma;
          sv[2 * A + j] = pc.c;
          sv[3 * A + j] = pc.u;
          sv[4 * A + j] = ls_raw;
        }
      }
    } else {
      act = tanhf(mu) * smp.max_action;
      if (mode == 0) {
        float nz = noise * noise_std;
        if (clamp_noise) nz = fminf(fmaxf(nz, -noise_clip), noise_clip);
        act = fminf(fmaxf(act + nz, -smp.max_action), smp.max_action);
      }
      if (save && valid) save[(int64_t)b * 5 * A + j] = mu;  // pre-tanh for backward
    }
    xs[r * ldx + S + j] = act;
    if (xa_out && valid) xa_out[(int64_t)b * d.X + S + j] = act;
  }
  if (logp_out && valid) logp_out[b] = policy_logp(smp.dist, A, lp_sum, m2_sum, hld_sum, jac_sum);
}

// Stage rows [row0, row0 + 16) of a [B, in] matrix into xs (pitch ldx), zeros
// past B and in columns [in, ldx) (layer 1 reads the first W1P columns of every
// row without a bound check).
__device__ __forceinline__ void stage_rows(const float* src, int in, float* xs, int ldx, int row0, int B) {
  const __amdgpu_buffer_rsrc_t rs = rlmd_rsrc(src, (int64_t)B * in * 4);
  for (int e = threadIdx.x; e < R * ldx; e += NT) {
    const int r = e / ldx, k = e % ldx;
    xs[r * ldx + k] = rlmd_ldf(rs, (int64_t)(row0 + r) * in + k, k < in && row0 + r < B);
  }
}

// stage_rows in two halves around the parameter prefetch: the row load is issued
// first, its LDS store after the prefetch is issued, so the store waits on the
// row load only (vmcnt retires in order) and layer 1 overlaps the fragment flight.
struct StageReg {
  float v;
  int e;
};
__device__ __forceinline__ StageReg stage_issue(const float* src, int in, int ldx, int row0, int B) {
  StageReg sr{0.f, (int)threadIdx.x};
  if (R * ldx <= NT) {
    const __amdgpu_buffer_rsrc_t rs = rlmd_rsrc(src, (int64_t)B * in * 4);
    const int r = sr.e / ldx, k = sr.e - r * ldx;
    sr.v = rlmd_ldf(rs, (int64_t)(row0 + r) * in + k, sr.e < R * ldx && k < in && row0 + r < B);
  }
  return sr;
}
__device__ __forceinline__ void stage_commit(const StageReg& sr, const float* src, int in, float* xs, int ldx, int row0,
                                             int B) {
  if (R * ldx <= NT) {
    if (sr.e < R * ldx) xs[sr.e] = sr.v;  // element e = r * ldx + k
  } else {
    stage_rows(src, in, xs, ldx, row0, B);
  }
}

template <int NBW>
__device__ __forceinline__ void actor_const(FwdConst<NBW>& k, const RowNet& n, const NetOff& ao, const RowDims& d) {
  const bool sac = d.algo == RLMD_SAC;
  fwd_const<NBW>(k, n.p, ao, d.S, sac ? 2 * d.A : d.A, n.p + ao.w3, sac ? n.p + ao.w4 : n.p + ao.w3, d.A);
}
template <int NBW>
__device__ __forceinline__ void critic_const(FwdConst<NBW>& k, const RowNet& n, const NetOff& co, const RowDims& d,
                                             int nb0 = 0) {
  fwd_const<NBW>(k, n.p, co, d.X, 1, n.p + co.w3, n.p + co.w3, 1, nb0);
}

// The backward-basis pass of one net over the block's rows: acc = aU (LDS,
// [R][H2p]) times fc2.weight through the transposed compute copy, masked by
// [h1 > 0] (m1s) and stored row-packed in f32 (u, [nrb][H1p][16]).
// K-steps [ks0, ke / KS) of the contraction (a column split: this half's fc2 columns).
template <int PREC, int NBW, bool MULTI>
__device__ __forceinline__ void basis_pass(Pre<PREC, NBW, MULTI>& pw, const typename CT<PREC>::T* aU, int lda,
                                           const void* wt, int H1p, int H2p, const uint8_t* m1s, float* u, int row0,
                                           int B, int ks0 = 0, int ke = 0) {
  f32x4 acc[NBW];
  mfma_rows<PREC, NBW, MULTI>(pw, aU, lda, wt, H2p, ke ? ke : H2p, H1p / 16, acc, 0, ks0);
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    if (wave + NW * i < H1p / 16) {
      const int col = acc_col(i);
      f32x4 v;
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int r = acc_row(rg);
        v[rg] = (m1s[r * H1p + col] && row0 + r < B) ? acc[i][rg] : 0.f;
      }
      rlmd_st_wt16(u + rp_index(row0 / R, H1p, acc_row(0), col), v[0], v[1], v[2], v[3]);
    }
  }
}

// y = 0, 1: target path with target critic y (the policy sample is recomputed
// per critic: same Philox draws, the logp written once); y = 2, 3: online
// critic y - 2 on (s, a); y = 4: policy on s for the actor step.
template <int PREC, int NBW, bool MULTI>
__global__ void __launch_bounds__(NT) fwd_rows_kernel(FwdRowsArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowDims& d = a.d;
  const Lds L = lds_layout(d);
  float* xs = reinterpret_cast<float*>(smem + L.xs);
  const float* hout = reinterpret_cast<const float*>(smem + L.hout);
  const int row0 = blockIdx.x * R, B = d.B;
  // jobs y0 .. nj - 1 of this update, then (npair) the next update's target jobs
  const int nj = a.with_actor ? 5 : 4;
  int job = (int)blockIdx.y + a.y0;
  const bool nxt = job >= nj;
  if (nxt) job -= nj;
  const bool sac = d.algo == RLMD_SAC;
  const int H1p = pad32(d.H1), H2p = pad32(d.H2);
  const int na = sac ? 2 * d.A : d.A;
  // column split of the critics' fc2 (gridDim.z = P <= 2, as qeval_rows): the
  // workgroup of half p streams half of each critic's fc2 copies and writes
  // partial q / target q / U1 at offset p, summed in half order by the critic
  // step.  The policy (target path, job 4) is not split: its heads need every
  // column before tanh; job 4's second half has nothing to do.
  const int P = (int)gridDim.z, p = (int)blockIdx.z;
  const int nbw = H2p / 16 / P, nb0 = p * nbw;              // this half's fc2 output bands
  const int ks0 = p * (H2p / P) / CT<PREC>::KS, ke = (p + 1) * (H2p / P);  // and its basis K-steps
  const int64_t ustr = (int64_t)((B + R - 1) / R) * H1p * R;  // one U1 slab
  if (job == 4 && p > 0) return;
  RLMD_TSJ(40 + job);
  if (job <= 1) {  // target path (algo_sac.py:300-367 / algo_td3.py:302-361)
    RLMD_TSR(16 * job + 0);
    const RowNet& an = a.tactor;
    const RowNet& cn = a.tcrit[job];
    const float* s2 = nxt ? a.s2n : a.s2;
    const float* eps_next = nxt ? nullptr : a.eps_next;
    SampleCfg smp = a.smp;
    if (nxt) smp.ctr = a.ctrn;  // the next update's learn_step_cntr (its target noise draws)
    const StageReg sr = stage_issue(s2, d.S, L.ldx, row0, B);
    const HeadBias hb = head_bias(an.p, a.ao, d);
    const bool pre_nz = eps_next == nullptr;
    FwdConst<NBW> ka, kc;
    actor_const<NBW>(ka, an, a.ao, d);
    Pre<PREC, NBW, MULTI> pa, pc;
    pre_issue<PREC, NBW, MULTI>(pa, an.wc, H1p, H1p, H2p / 16);
    // the target critic's constants and fc2 stream: issued after the policy's
    // layer 2 (RLMD_FWD_DEFER; 0: with this first round)
    auto issue_critic = [&] {
      critic_const<NBW>(kc, cn, a.co, d, nb0);
      pre_issue<PREC, NBW, MULTI>(pc, cn.wc, H1p, H1p, nbw, nb0);
    };
    if constexpr (!RLMD_FWD_DEFER) issue_critic();
    const Noise2 nz = pre_nz ? noise_pre(smp, d, a.t_tag, row0) : Noise2{{0.f, 0.f}};
    RLMD_TSR(16 * job + 1);
    stage_commit(sr, s2, d.S, xs, L.ldx, row0, B);
    __syncthreads();
    RLMD_TSR(16 * job + 2);
    if constexpr (RLMD_FWD_DEFER)
      mlp_rows<PREC, NBW, MULTI>(an, a.ao, ka, pa, xs, L.ldx, d.S, na, an.p + a.ao.w3, sac ? an.p + a.ao.w4 : nullptr,
                                 d.A, smem, L, nullptr, nullptr, row0, B, nullptr, nullptr, nullptr, 0, 0, issue_critic,
                                 6);
    else
      mlp_rows<PREC, NBW, MULTI>(an, a.ao, ka, pa, xs, L.ldx, d.S, na, an.p + a.ao.w3, sac ? an.p + a.ao.w4 : nullptr,
                                 d.A, smem, L, nullptr, nullptr, row0, B);
    RLMD_TSR(16 * job + 3);
    // load-free sampling on the production path (no injected noise): see sample_rows
    if (RLMD_SAMPLE_NL && pre_nz && d.A <= 2)
      sample_rows<true>(an.p, a.ao, d, smp, xs, L.ldx, hout, 0, a.t_tag, nullptr, a.t_noise_std, a.t_noise_clip,
                        a.t_clamp, job == 0 && !nxt && p == 0 ? a.logp_next : nullptr, nullptr, nullptr, row0, B, hb,
                        true, nz, true);
    else
      sample_rows(an.p, a.ao, d, smp, xs, L.ldx, hout, 0, a.t_tag, eps_next, a.t_noise_std, a.t_noise_clip,
                  a.t_clamp, job == 0 && !nxt && p == 0 ? a.logp_next : nullptr, nullptr, nullptr, row0, B, hb, true, nz,
                  pre_nz);
    __syncthreads();
    RLMD_TSR(16 * job + 4);
    mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, nullptr,
                               nullptr, row0, B, nullptr, nullptr, nullptr, nb0, nbw, NoHook(), 22);
    RLMD_TSR(16 * job + 5);
    float* qt = (nxt ? a.qtn[job] : a.qt[job]) + p * B;
    if ((int)threadIdx.x < R && row0 + (int)threadIdx.x < B) qt[row0 + threadIdx.x] = hout[threadIdx.x * kHeadsMax];
    if (!nxt && a.bsnap && blockIdx.x == 0 && p == 0 && threadIdx.x == 0) a.bsnap[2 + job] = cn.p[a.co.b3];
  } else if (job <= 3) {  // online critics on (s, a) (algo_sac.py:413-417)
    if (job == 2) RLMD_TSR(60);
    const int g = job - 2;
    const RowNet& cn = a.crit[g];
    const bool upd = a.u1[0] != nullptr;
    const StageReg sr = stage_issue(a.xsa, d.X, L.ldx, row0, B);
    FwdConst<NBW> kc;
    critic_const<NBW>(kc, cn, a.co, d, nb0);
    Pre<PREC, NBW, MULTI> pc, pw;
    pre_issue<PREC, NBW, MULTI>(pc, cn.wc, H1p, H1p, nbw, nb0);
    // the basis pass's stream (the transposed copy): after the forward's layer 2
    auto issue_basis = [&] {
      if (upd) pre_issue<PREC, NBW, MULTI>(pw, cn.wt, H2p, ke, H1p / 16, 0, ks0);
    };
    if constexpr (!RLMD_FWD_DEFER) issue_basis();
    stage_commit(sr, a.xsa, d.X, xs, L.ldx, row0, B);
    __syncthreads();
    if (job == 2) RLMD_TSR(61);
    if (!upd) {
      mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, a.c1[g],
                                 a.c2[g], row0, B, a.cm1[g], a.cm2[g], nullptr, nb0, nbw);
    } else {
      using T = typename CT<PREC>::T;
      T* aU = reinterpret_cast<T*>(smem + L.aU);
      uint8_t* m1s = reinterpret_cast<uint8_t*>(smem + L.m1s);
      // h1 is the same in both halves: half 0 writes it
      const FwdExtra<PREC> ex{p == 0 ? static_cast<T*>(a.hp1[g]) : nullptr, static_cast<T*>(a.hp2[g]), m1s, aU};
      if constexpr (RLMD_FWD_DEFER)
        mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, nullptr,
                                   nullptr, row0, B, nullptr, a.cm2[g], &ex, nb0, nbw, issue_basis);
      else
        mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, nullptr,
                                   nullptr, row0, B, nullptr, a.cm2[g], &ex, nb0, nbw);
      // the backward basis of these rows: U1 = [h1 > 0] * (([h2 > 0] w3) W2), so
      // that the critic update forms dh1 = dq * U1 once dq is known (update.hip);
      // a half's partial U1 over its fc2 columns
      basis_pass<PREC, NBW, MULTI>(pw, aU, L.lda1, cn.wt, H1p, H2p, m1s, a.u1[g] + p * ustr, row0, B, ks0, ke);
      if (blockIdx.x == 0 && p == 0) {  // snapshots of what the update reads while stepping it
        for (int c = threadIdx.x; c < d.H2; c += NT) a.w3s[g][c] = cn.p[a.co.w3 + c];
        if (threadIdx.x == 0) a.bsnap[g] = cn.p[a.co.b3];
      }
    }
    if (job == 2) RLMD_TSR(62);
    if ((int)threadIdx.x < R && row0 + (int)threadIdx.x < B) a.q[g][p * B + row0 + threadIdx.x] = hout[threadIdx.x * kHeadsMax];
  } else {  // policy on s for the actor update (algo_sac.py:524-535 / algo_td3.py:507-515)
    RLMD_TSR(80);
    const RowNet& an = a.actor;
    const StageReg sr = stage_issue(a.s, d.S, L.ldx, row0, B);
    const HeadBias hb = head_bias(an.p, a.ao, d);
    FwdConst<NBW> ka;
    actor_const<NBW>(ka, an, a.ao, d);
    Pre<PREC, NBW, MULTI> pa;
    pre_issue<PREC, NBW, MULTI>(pa, an.wc, H1p, H1p, H2p / 16);
    const bool pre_nz = a.eps_cur == nullptr && a.a_mode == 0;
    const Noise2 nz = pre_nz ? noise_pre(a.smp, d, a.a_tag, row0) : Noise2{{0.f, 0.f}};
    stage_commit(sr, a.s, d.S, xs, L.ldx, row0, B);
    __syncthreads();
    RLMD_TSR(81);
    for (int e = threadIdx.x; e < R * d.S; e += NT) {
      const int r = e / d.S, k = e % d.S;
      if (row0 + r < B) a.xsan[(int64_t)(row0 + r) * d.X + k] = xs[r * L.ldx + k];
    }
    // fused actor update (hp1a set): h1 / h2 row-packed for its weight-gradient
    // tiles instead of the launch chain's f32 rows
    using T = typename CT<PREC>::T;
    const bool fa = a.hp1a != nullptr;
    const FwdExtra<PREC> ex{static_cast<T*>(a.hp1a), static_cast<T*>(a.hp2a), nullptr, nullptr};  // null: not written
    mlp_rows<PREC, NBW, MULTI>(an, a.ao, ka, pa, xs, L.ldx, d.S, na, an.p + a.ao.w3, sac ? an.p + a.ao.w4 : nullptr,
                               d.A, smem, L, fa ? nullptr : a.h1a, fa ? nullptr : a.h2a, row0, B, a.am1, a.am2, &ex);
    RLMD_TSR(82);
    if (RLMD_SAMPLE_NL && (pre_nz || a.a_mode == 1) && a.eps_cur == nullptr && d.A <= 2)
      sample_rows<true>(an.p, a.ao, d, a.smp, xs, L.ldx, hout, a.a_mode, a.a_tag, nullptr, 0.f, 0.f, 0, a.logp, a.save,
                        a.xsan, row0, B, hb, true, nz, true);
    else
      sample_rows(an.p, a.ao, d, a.smp, xs, L.ldx, hout, a.a_mode, a.a_tag, a.eps_cur, 0.f, 0.f, 0, a.logp, a.save,
                  a.xsan, row0, B, hb, true, nz, pre_nz);
    RLMD_TSR(83);
  }
  RLMD_TSJ(45 + job);
}

// per-thread ReLU masks of one net's rows: m2 in the elementwise map over H2p
// (for dh2), m1 in the MFMA accumulator layout over H1p (for dh1)

template <int NBW>
struct BwdMask {
  float m2[kMR<NBW>];
  float m1[NBW][4];
  float w3;  // head weight of this thread's dh2 column
};

template <int NBW>
__device__ __forceinline__ void bwd_mask(BwdMask<NBW>& k, const uint8_t* m1, const uint8_t* m2, const float* w3,
                                         const NetOff& o, int row0, int B, int nb0 = 0) {
  const int H2 = o.h2, H1p = pad32(o.h1), H2p = pad32(o.h2), rb = row0 / R;
  const ElemMap m = elem_map(H2p);
  const bool cin = m.c < H2;
  const int nrb = (B + R - 1) / R;
  const __amdgpu_buffer_rsrc_t r1 = rlmd_rsrc(m1, (int64_t)nrb * H1p * 16),
                               r2 = rlmd_rsrc(m2, (int64_t)nrb * H2p * 16);
  // m2: this thread's kMR consecutive rows of column m.c from kMR / 4 aligned
  // words (+ one when its first row is not word aligned: fewer than 4 rows per
  // thread, H2p < 128)
  constexpr int NWD = kMR<NBW> / 4;
  const int sh = m.r0 & 3, rbase = m.r0 & ~3;
  uint32_t wd[NWD + 1];
#pragma unroll
  for (int w = 0; w <= NWD; ++w) {
    const int64_t e = m2_index(rb, H2p, rbase + 4 * w, m.c);
    const bool need = m.r0 < R && (w < NWD || sh != 0);
    wd[w] = __builtin_amdgcn_raw_buffer_load_b32(r2, need ? (int)e : 0x7fffffff, 0, 0);
  }
#pragma unroll
  for (int rr = 0; rr < kMR<NBW>; ++rr) {
    const int bb = (rr & 3) + sh;
    const uint32_t w = bb < 4 ? wd[rr >> 2] >> (8 * bb) : wd[(rr >> 2) + 1] >> (8 * (bb - 4));
    k.m2[rr] = (w & 0xffu) ? 1.f : 0.f;
  }
  k.w3 = w3 ? rlmd_ldf(rlmd_rsrc(w3, (int64_t)H2 * 4), m.c, cin) : 0.f;
  // m1: one word (this lane's 4 rows) per accumulator band
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    const int col = acc_col(i, nb0);
    const int64_t e = m1_index(rb, H1p, acc_row(0), col);
    const uint32_t word = __builtin_amdgcn_raw_buffer_load_b32(r1, col < H1p ? (int)e : 0x7fffffff, 0, 0);
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) k.m1[i][rg] = (word >> (8 * rg)) & 0xffu ? 1.f : 0.f;
  }
}

template <int PREC, int NBW, bool MULTI>
__global__ void __launch_bounds__(NT) qeval_rows_kernel(QEvalArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowDims& d = a.d;
  const Lds L = lds_layout(d);
  float* xs = reinterpret_cast<float*>(smem + L.xs);
  const float* hout = reinterpret_cast<const float*>(smem + L.hout);
  const int row0 = blockIdx.x * R, B = d.B;
  const int H1p = pad32(d.H1), H2p = pad32(d.H2);
  // column split (a.split = P halves of the fc2 output columns, P <= 2): the
  // critic workgroup of half p streams half of each fc2 copy — the per-workgroup
  // weight stream is this kernel's cost — and writes partial q and dq/da at
  // offset p, which the actor step sums in half order.  The head jobs' stream
  // (the policy's transposed copy) is one copy already, no more than a critic
  // half's two: they are not split (their second half returns at once), so the
  // actor step reads one basis per head.  Grid y: critic g half p at g * P + p,
  // then the head jobs.
  const int P = a.split > 1 ? 2 : 1, y = (int)blockIdx.y;
  const int g = y < a.nq * P ? y / P : y - a.nq * P + a.nq, p = y < a.nq * P ? y % P : 0;
  const int kh = H2p / P, ks0 = p * kh / CT<PREC>::KS, ke = (p + 1) * kh;  // this half's fc2 columns as K-steps
  if (g >= a.nq) {
    // the policy's backward basis of head h over the block's rows (fused actor
    // update): aU = [h2 > 0] * W_head[h] from the forward's masks, times fc2.weight
    // through the transposed copy, masked by [h1 > 0], stored row-packed f32
    using T = typename CT<PREC>::T;
    const int h = g - a.nq, nrb = (B + R - 1) / R;
    const RowNet& an = a.actor;
    Pre<PREC, NBW, MULTI> pw;
    pre_issue<PREC, NBW, MULTI>(pw, an.wt, H2p, H2p, H1p / 16);
    BwdMask<NBW> k;
    bwd_mask<NBW>(k, a.am1, a.am2, nullptr, a.ao, row0, B);
    const ElemMap m = elem_map(H2p);
    const int64_t wrow = h < d.A ? a.ao.w3 + (int64_t)h * d.H2 : a.ao.w4 + (int64_t)(h - d.A) * d.H2;
    const float wk = rlmd_ldf(rlmd_rsrc(an.p, a.ao.size * 4), wrow + m.c, m.c < d.H2);
    if (blockIdx.x == 0 && m.r0 == 0 && m.c < d.H2) a.wheads[(int64_t)h * d.H2 + m.c] = wk;
    T* aU = reinterpret_cast<T*>(smem + L.aU);
#pragma unroll
    for (int rr = 0; rr < kMR<NBW>; ++rr) {
      const int r = m.r0 + rr;
      if (r < m.r1) aU[r * L.lda1 + m.c] = CT<PREC>::cvt(k.m2[rr] > 0.f ? wk : 0.f);
    }
    __syncthreads();
    f32x4 acc[NBW];
    mfma_rows<PREC, NBW, MULTI>(pw, aU, L.lda1, an.wt, H2p, H2p, H1p / 16, acc);
    float* u = a.ua + (int64_t)h * nrb * H1p * R;
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      if (wave + NW * i < H1p / 16) {
        const int col = acc_col(i);
        f32x4 v;
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) v[rg] = (k.m1[i][rg] > 0.f && row0 + acc_row(rg) < B) ? acc[i][rg] : 0.f;
        rlmd_st_wt16(u + rp_index(row0 / R, H1p, acc_row(0), col), v[0], v[1], v[2], v[3]);
      }
    }
    return;
  }
  const RowNet& cn = a.crit[g];
  const bool upd = a.dqda[0] != nullptr;
  const int nbw = H2p / 16 / P, nb0 = p * nbw;  // this half's fc2 output bands
  Pre<PREC, NBW, MULTI> pc, pw;
  pre_issue<PREC, NBW, MULTI>(pc, cn.wc, H1p, H1p, nbw, nb0);
  FwdConst<NBW> kc;
  critic_const<NBW>(kc, cn, a.co, d, nb0);
  float w1a[NBW][NHF];  // W1[c][S + j] of this lane's accumulator columns (fused actor update)
  // the basis pass's stream: after the forward's layer 2 (as fwd_rows' critic jobs)
  auto issue_basis = [&] { pre_issue<PREC, NBW, MULTI>(pw, cn.wt, H2p, ke, H1p / 16, 0, ks0); };
  if (upd) {
    if constexpr (!RLMD_FWD_DEFER) issue_basis();
    const __amdgpu_buffer_rsrc_t rp = rlmd_rsrc(cn.p, a.co.size * 4);
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int col = acc_col(i);
#pragma unroll
      for (int j = 0; j < NHF; ++j)
        w1a[i][j] = j < d.A ? rlmd_ldf(rp, a.co.w1 + (int64_t)col * d.X + d.S + j, col < d.H1) : 0.f;
    }
  }
  stage_rows(a.x, d.X, xs, L.ldx, row0, B);
  __syncthreads();
  if (!upd) {
    mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, a.e1[g],
                               a.e2[g], row0, B, a.em1[g], a.em2[g], nullptr, nb0, nbw);
  } else {
    // the critic on (s, a_new) and its input gradient dq/da per row: the basis
    // pass [h1 > 0] * (([h2 > 0] w3) W2) contracted with W1[:, S:S+A] (the
    // launch-chain path's abwd_rows dh1 with dq = 1; the actor update scales it)
    using T = typename CT<PREC>::T;
    T* aU = reinterpret_cast<T*>(smem + L.aU);
    const uint8_t* m1s = reinterpret_cast<const uint8_t*>(smem + L.m1s);
    float* part = reinterpret_cast<float*>(smem + L.part);
    const FwdExtra<PREC> ex{nullptr, nullptr, reinterpret_cast<uint8_t*>(smem + L.m1s), aU};
    if constexpr (RLMD_FWD_DEFER)
      mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, nullptr,
                                 nullptr, row0, B, nullptr, nullptr, &ex, nb0, nbw, issue_basis);
    else
      mlp_rows<PREC, NBW, MULTI>(cn, a.co, kc, pc, xs, L.ldx, d.X, 1, cn.p + a.co.w3, nullptr, 1, smem, L, nullptr,
                                 nullptr, row0, B, nullptr, nullptr, &ex, nb0, nbw);
    f32x4 acc[NBW];
    mfma_rows<PREC, NBW, MULTI>(pw, aU, L.lda1, cn.wt, H2p, ke, H1p / 16, acc, 0, ks0);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float pd[4][NHF];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
      for (int j = 0; j < NHF; ++j) pd[rg][j] = 0.f;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      if (wave + NW * i < H1p / 16) {
        const int col = acc_col(i);
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const float v = m1s[acc_row(rg) * H1p + col] ? acc[i][rg] : 0.f;
#pragma unroll
          for (int j = 0; j < NHF; ++j) pd[rg][j] = fmaf(v, w1a[i][j], pd[rg][j]);
        }
      }
    }
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
      for (int j = 0; j < NHF; ++j) {
        if (j < d.A) {
          const float c = rlmd_row16_sum(pd[rg][j]);
          if ((lane & 15) == 0) part[(wave * R + acc_row(rg)) * NHF + j] = c;
        }
      }
    __syncthreads();
    if ((int)threadIdx.x < R * d.A) {
      const int r = threadIdx.x % R, j = threadIdx.x / R;
      if (row0 + r < B) a.dqda[g][(int64_t)(p * B + row0 + r) * d.A + j] = head_sum(part, r, j);
    }
  }
  if ((int)threadIdx.x < R && row0 + (int)threadIdx.x < B) a.qn[g][p * B + row0 + threadIdx.x] = hout[threadIdx.x * kHeadsMax];
}

// ---------------------------------------------------------------------------
// backward pieces
// ---------------------------------------------------------------------------
// dh2 = dq[r] * w3 * [h2 > 0] -> A operand (T) and HBM (nullable)
template <int PREC, int NBW>
__device__ __forceinline__ void dh2_from_q(const BwdMask<NBW>& k, const float* dqr, const NetOff& o,
                                           typename CT<PREC>::T* aT, int ldaT, float* dh2_out, int row0, int B) {
  const int H2 = o.h2;
  const ElemMap m = elem_map(pad32(H2));
  // every row's dq read first (clamped row, no branch between the LDS reads)
  float dq[kMR<NBW>];
#pragma unroll
  for (int rr = 0; rr < kMR<NBW>; ++rr) dq[rr] = dqr[m.r0 + rr < R ? m.r0 + rr : R - 1];
#pragma unroll
  for (int rr = 0; rr < kMR<NBW>; ++rr) {
    const int r = m.r0 + rr;
    if (r < m.r1) {
      const float v = k.m2[rr] > 0.f ? dq[rr] * k.w3 : 0.f;
      aT[r * ldaT + m.c] = CT<PREC>::cvt(v);
      if (dh2_out && m.c < H2 && row0 + r < B) dh2_out[(int64_t)(row0 + r) * H2 + m.c] = v;
    }
  }
}

// dh1 = (dh2 W2) * [h1 > 0] (MFMA with the transposed copy) -> HBM (nullable) and,
// for the actor path, per-wave partials of dL/da = sum_c dh1[r][c] W1[c][S + j].
template <int PREC, int NBW, bool MULTI>
__device__ __forceinline__ void dh1_rows(Pre<PREC, NBW, MULTI>& pre, const RowNet& net, const NetOff& o,
                                         const BwdMask<NBW>& k, const typename CT<PREC>::T* aT, int ldaT,
                                         float* dh1_out, const float (*w1a)[NHF], int na, float* part, int row0,
                                         int B, int nb0 = 0, int nbp = 0) {
  // column split: bands nb0 .. nb0 + nbp - 1 of dh1 (nbp = 0: all of them)
  const int H1 = o.h1, H1p = pad32(H1), H2p = pad32(o.h2);
  const int nb = nbp ? nbp : H1p / 16;
  f32x4 acc[NBW];
  mfma_rows<PREC, NBW, MULTI>(pre, aT, ldaT, net.wt, H2p, H2p, nb, acc, nb0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pd[4][NHF];
#pragma unroll
  for (int rg = 0; rg < 4; ++rg)
#pragma unroll
    for (int j = 0; j < NHF; ++j) pd[rg][j] = 0.f;
#pragma unroll
  for (int i = 0; i < NBW; ++i) {
    if (wave + NW * i < nb) {
      const int col = acc_col(i, nb0);
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int b = row0 + acc_row(rg);
        const float v = k.m1[i][rg] > 0.f ? acc[i][rg] : 0.f;
        if (dh1_out && col < H1 && b < B) dh1_out[(int64_t)b * H1 + col] = v;
        if (w1a) {
#pragma unroll
          for (int j = 0; j < NHF; ++j) pd[rg][j] = fmaf(v, w1a[i][j], pd[rg][j]);
        }
      }
    }
  }
  if (w1a) {
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
      for (int j = 0; j < NHF; ++j) {
        if (j < na) {
          const float c = rlmd_row16_sum(pd[rg][j]);
          if ((lane & 15) == 0) part[(wave * R + acc_row(rg)) * NHF + j] = c;
        }
      }
  }
}

template <int PREC, int NBW, bool MULTI>
__global__ void __launch_bounds__(NT) cbwd_rows_kernel(CBwdArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  using T = typename CT<PREC>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const Lds L = lds_layout(a.d);
  T* aT = reinterpret_cast<T*>(smem + L.aT);
  float* rowv = reinterpret_cast<float*>(smem + L.rowv);
  const int row0 = blockIdx.x * R, g = blockIdx.y, B = a.d.B;
  const RowNet& cn = a.crit[g];
  const int H1p = pad32(a.d.H1), H2p = pad32(a.d.H2);
  // dh1 columns split over gridDim.z workgroups (each streams 1/z of W2^T);
  // part 0 also writes the per-row outputs
  const int nbp = (H1p / 16) / gridDim.z, nb0 = blockIdx.z * nbp;
  const bool lead = blockIdx.z == 0;
  if (g == 0 && lead) RLMD_TSR(112);
  CriticLoads cl{};
  if (a.loss.B > 0) cl = critic_row_load(a.loss);
  BwdMask<NBW> k;
  bwd_mask<NBW>(k, a.cm1[g], a.cm2[g], cn.p + a.co.w3, a.co, row0, B, nb0);
  Pre<PREC, NBW, MULTI> pw;
  pre_issue<PREC, NBW, MULTI>(pw, cn.wt, H2p, H2p, nbp, nb0);
  if (g == 0 && lead) RLMD_TSR(113);
  if (a.loss.B > 0) {
    // critic loss gradient of this block's rows (rlmd_loss.h): every row's loss,
    // then the rows' top-k ranks counted against all B keys
    uint64_t* vkey = reinterpret_cast<uint64_t*>(smem + L.vkey);
    float* red = reinterpret_cast<float*>(smem + L.red);
    int* rank16 = reinterpret_cast<int*>(smem + L.part);
    float* dl16 = reinterpret_cast<float*>(smem + L.part) + R;
    CriticRow o;
    critic_row_loss(a.loss, red, o, cl);
    if (g == 0 && lead) RLMD_TSR(114);
    const int t = threadIdx.x;
    if (a.bias_out && lead && blockIdx.x == 0 && g == 0 && t < 4)
      a.bias_out[t] = t < 2 ? a.loss.qb[t][0] : a.loss.tb[t - 2][0];
    if (t < B) vkey[t] = critic_sel_key(o);
    if (t < R) rank16[t] = 0;
    if (t >= row0 && t < row0 + R) dl16[t - row0] = g == 0 ? o.dl[0] : o.dl[1];
    __syncthreads();
    if (g == 0 && lead) RLMD_TSR(115);
    const bool topk = B > a.loss.k;
    if (topk) {
      const int r = t & (R - 1), prt = t / R;
      constexpr int NP = NT / R;
      const uint64_t mine = vkey[row0 + r < B ? row0 + r : 0];
      int c = 0;
      for (int j = prt; j < B; j += NP) c += vkey[j] < mine;
      atomicAdd(&rank16[r], c);
      __syncthreads();
    }
    if (t < R) {
      const int b = row0 + t, kk = topk ? a.loss.k : B;
      const bool sel = b < B && (!topk || rank16[t] < kk);
      const float dq = sel ? a.loss.grad_scale * dl16[t] / (float)kk : 0.f;
      rowv[t] = dq;
      if (lead && b < B) a.loss.dq[g][b] = dq;
    }
  } else if ((int)threadIdx.x < R) {
    rowv[threadIdx.x] = rlmd_ldf(rlmd_rsrc(a.dq[g], (int64_t)B * 4), row0 + threadIdx.x, row0 + (int)threadIdx.x < B);
  }
  __syncthreads();
  if (g == 0 && lead) RLMD_TSR(116);
  dh2_from_q<PREC, NBW>(k, rowv, a.co, aT, L.ldaT, lead ? a.dc2[g] : nullptr, row0, B);
  __syncthreads();
  if (g == 0 && lead) RLMD_TSR(117);
  dh1_rows<PREC, NBW, MULTI>(pw, cn, a.co, k, aT, L.ldaT, a.dc1[g], nullptr, 0, nullptr, row0, B, nb0, nbp);
  if (g == 0 && lead) RLMD_TSR(118);
}

// Actor data-gradients (autograd of algo_sac.py:524-562 through
// networks_sac.py:163-178; algo_td3.py:507-523 through networks_td3.py:91).
// NQ: critics the actor loss reads (SAC min(q1, q2): 2; TD3 q1: 1) — a compile-time
// count, so TD3's instantiations hold no second critic's fragments or masks.
template <int PREC, int NBW, bool MULTI, int NQ>
__global__ void __launch_bounds__(NT) abwd_rows_kernel(ABwdArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  const int nq = NQ == 1 ? 1 : a.nq;  // NQ = 2 keeps the runtime count (its register allocation measured best)
  using T = typename CT<PREC>::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowDims& d = a.d;
  const Lds L = lds_layout(d);
  T* aT = reinterpret_cast<T*>(smem + L.aT);
  float* h2s = reinterpret_cast<float*>(smem + L.h2s);  // dh1 rows when A > NHF
  float* part = reinterpret_cast<float*>(smem + L.part);
  float* hout = reinterpret_cast<float*>(smem + L.hout);  // dL/da per row
  float* ghs = reinterpret_cast<float*>(smem + L.ghs);
  float* rowv = reinterpret_cast<float*>(smem + L.rowv);
  const int row0 = blockIdx.x * R, B = d.B, S = d.S, A = d.A, X = d.X;
  const bool sac = d.algo == RLMD_SAC;
  const int H1p = pad32(d.H1), H2p = pad32(d.H2);
  const NetOff& ao = a.ao;
  const NetOff& co = a.co;
  const bool fused_da = A <= NHF;
  if (a.cstats.B > 0 && blockIdx.x == gridDim.x - 1) {
    // this update's critic statistics (rlmd_loss.h), off the critical path
    critic_loss_block<NT / 64>(a.cstats, reinterpret_cast<uint64_t*>(smem + L.runs), reinterpret_cast<int*>(smem + L.rank),
                      reinterpret_cast<float*>(smem + L.red));
    return;
  }
  RLMD_TSR(96);
  // ---- every independent load up front; what the actor loss reads first and the
  //      weight fragments last (vmcnt retires in issue order)
  const int64_t nB = (int64_t)B * 4;
  const __amdgpu_buffer_rsrc_t rq0 = rlmd_rsrc(a.qn[0], nB), rq1 = rlmd_rsrc(nq > 1 ? a.qn[1] : a.qn[0], nB),
                               rlp = rlmd_rsrc(sac ? a.logp : a.qn[0], nB);
  const int tq = threadIdx.x, bq = row0 + (int)threadIdx.x;
  const float ld_q1 = rlmd_ldf(rq0, tq, tq < B), ld_q2 = rlmd_ldf(rq1, tq, tq < B && nq > 1);
  const float ld_lp = rlmd_ldf(rlp, tq, tq < B && sac);
  const float log_alpha = sac ? a.st->log_alpha[slot_rd((int)a.smp.ctr)] : 0.f;  // scalar loads, issued with the first round
  const float qb0 = a.crit[0].p[co.b3], qb1 = nq > 1 ? a.crit[1].p[co.b3] : 0.f;
  const float row_q1 = rlmd_ldf(rq0, bq, tq < R && bq < B), row_q2 = rlmd_ldf(rq1, bq, tq < R && bq < B && nq > 1);
  // first round: what the loss and critic 1 need (under the 63-load vmcnt cap);
  // critic 2's masks / fragments follow after the key pass, the actor's before
  // the sampling pass
  BwdMask<NBW> k0, k1, ka;
  bwd_mask<NBW>(k0, a.em1[0], a.em2[0], a.crit[0].p + co.w3, co, row0, B);
  float w1a[NQ][NBW][NHF];  // W1_g[c][S + j] for this lane's dh1 columns
#pragma unroll
  for (int g = 0; g < NQ; ++g) {
    const __amdgpu_buffer_rsrc_t rp = rlmd_rsrc(a.crit[g < nq ? g : 0].p, co.size * 4);
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int col = acc_col(i);
#pragma unroll
      for (int j = 0; j < NHF; ++j)
        w1a[g][i][j] = g < nq && j < A ? rlmd_ldf(rp, co.w1 + (int64_t)col * X + S + j, col < d.H1) : 0.f;
    }
  }
  Pre<PREC, NBW, MULTI> p0, p1;
  pre_issue<PREC, NBW, MULTI>(p0, a.crit[0].wt, H2p, H2p, H1p / 16);
  RLMD_TSR(95);
  // ---- actor loss (algo_sac.py:546-562 / algo_td3.py:507-523): every row's
  //      objective and ranking key (SAC sorts descending, TD3 ascending, Q5)
  uint64_t* vkey = reinterpret_cast<uint64_t*>(smem + L.vkey);
  float* vval = reinterpret_cast<float*>(smem + L.vval);
  int* rank16 = reinterpret_cast<int*>(part);  // [R] (part is free until the first dh1)
  const float alpha = sac ? expf(log_alpha) : 0.f;
  for (int j = threadIdx.x; j < B; j += NT) {
    const bool first = j == (int)threadIdx.x;  // preloaded
    const float q1 = (first ? ld_q1 : a.qn[0][j]) + qb0;
    const float q2 = nq > 1 ? (first ? ld_q2 : a.qn[1][j]) + qb1 : q1;
    const float v = sac ? fminf(q1, q2) - alpha * (first ? ld_lp : a.logp[j]) : q1;
    vval[j] = v;
    vkey[j] = ((uint64_t)(sac ? ~f2key(v) : f2key(v)) << 32) | (uint32_t)j;
  }
  if ((int)threadIdx.x < R) rank16[threadIdx.x] = 0;
  const int kk = a.topk ? (B < a.k ? B : a.k) : B;
  const bool ext = a.dqn_ext[0] != nullptr;  // loss from actor_loss_kernel (B > 512)
  __syncthreads();
  RLMD_TSR(97);
  if (nq > 1) {
    bwd_mask<NBW>(k1, a.em1[1], a.em2[1], a.crit[1].p + co.w3, co, row0, B);
    pre_issue<PREC, NBW, MULTI>(p1, a.crit[1].wt, H2p, H2p, H1p / 16);
  }
  if (!ext && blockIdx.x == gridDim.x - 1 - (a.cstats.B > 0 ? 1 : 0)) {
    // the loss workgroup: selection over all rows -> loss value, temperature gradient
    uint64_t* runs = reinterpret_cast<uint64_t*>(smem + L.runs);
    int* rank_of = reinterpret_cast<int*>(smem + L.rank);
    const int t = threadIdx.x;
    bool sel = t < B;
    if (a.topk) {
      block_rank<NT / 64>(t < B ? vkey[t] : ~0ull, runs, rank_of);
      sel = t < B && rank_of[t] < kk;
    }
    float sm[2] = {sel ? vval[t] : 0.f, (t < B && sac) ? -(ld_lp + a.target_entropy) : 0.f};
    float mx[1] = {-INFINITY};
    block_allreduce<2, 0>(sm, mx, reinterpret_cast<float*>(smem + L.red));
    if (t == 0) {
      if (sac) a.st->pad_temp_grad = sm[1] / B * alpha;
      a.stats[10] = -sm[0] / kk;
    }
    return;
  }
  // rank of this block's rows among all B (32 partial counts per row)
  {
    const int r = threadIdx.x & (R - 1), prt = threadIdx.x / R;
    constexpr int NP = NT / R;
    const uint64_t mine = row0 + r < B ? vkey[row0 + r] : ~0ull;
    int c = 0;
    if (!ext)
      for (int j = prt; j < B; j += NP) c += vkey[j] < mine;
    atomicAdd(&rank16[r], c);
  }
  __syncthreads();
  RLMD_TSR(98);
  float* dlogp_r = rowv + 2 * R;  // [R]
  if ((int)threadIdx.x < R) {
    const int r = threadIdx.x, b = row0 + r;
    float dq0 = 0.f, dq1 = 0.f, dlp = 0.f;
    if (ext && b < B) {
      dq0 = a.dqn_ext[0][b];
      dq1 = nq > 1 ? a.dqn_ext[1][b] : 0.f;
      dlp = sac ? a.dlogp_ext[b] : 0.f;
    } else if (b < B) {
      const bool sel = !a.topk || rank16[r] < kk;
      const float dv = sel ? -1.f / (float)kk : 0.f;
      if (sac) {
        // d min(q1, q2): ties split evenly (torch.minimum backward)
        const float q1 = row_q1 + qb0, q2 = row_q2 + qb1;
        const float g1 = q1 < q2 ? 1.f : (q1 > q2 ? 0.f : 0.5f);
        dq0 = dv * g1;
        dq1 = dv * (1.f - g1);
        dlp = -alpha * dv;
      } else {
        dq0 = dv;
      }
    }
    rowv[r] = dq0;
    rowv[R + r] = dq1;
    dlogp_r[r] = dlp;
  }
  __syncthreads();
  // ---- dL/da through each critic: dh2 -> dh1 (MFMA) -> . W1[:, S:S+A]
  for (int g = 0; g < nq; ++g) {
    const BwdMask<NBW>& k = g == 0 ? k0 : k1;
    dh2_from_q<PREC, NBW>(k, rowv + g * R, co, aT, L.ldaT, nullptr, row0, B);
    __syncthreads();
    RLMD_TSR(99 + 4 * g);
    if (fused_da) {
      dh1_rows<PREC, NBW, MULTI>(g == 0 ? p0 : p1, a.crit[g], co, k, aT, L.ldaT, nullptr, w1a[NQ > 1 ? g : 0], A,
                                 part, row0, B);
      RLMD_TSR(100 + 4 * g);
      __syncthreads();
      RLMD_TSR(101 + 4 * g);
      if ((int)threadIdx.x < R * A) {
        const int r = threadIdx.x % R, j = threadIdx.x / R;
        const float s = head_sum(part, r, j);
        hout[r * kHeadsMax + j] = g == 0 ? s : hout[r * kHeadsMax + j] + s;
      }
    } else {
      // many actions: dh1 rows through LDS, then LDS dot products with W1[:, S:]
      f32x4 acc[NBW];
      mfma_rows<PREC, NBW, MULTI>(g == 0 ? p0 : p1, aT, L.ldaT, a.crit[g].wt, H2p, H2p, H1p / 16, acc);
#pragma unroll
      for (int i = 0; i < NBW; ++i)
        if (((int)threadIdx.x >> 6) + NW * i < H1p / 16)
#pragma unroll
          for (int rg = 0; rg < 4; ++rg)
            h2s[acc_row(rg) * L.ldh2 + acc_col(i)] = k.m1[i][rg] > 0.f ? acc[i][rg] : 0.f;
      __syncthreads();
      row_dots(h2s, L.ldh2, d.H1, A, a.crit[g].p + co.w1 + S, nullptr, A, 1, X, hout, kHeadsMax, g > 0);
    }
    __syncthreads();
  }
  RLMD_TSR(108);
  // ---- through the sampling and the heads
  // this thread's head-weight column for the dh2 pass below (A <= 2: registers),
  // issued ahead of the actor's fragments so its first use does not wait on
  // them (vmcnt retires in issue order); loaded once instead of per row (the
  // dh2 stores may alias the parameters for the compiler)
  float wp[2], wl[2];
  {
    const ElemMap m = elem_map(H2p);
    const bool cin = m.c < ao.h2, few = A <= 2;
    const __amdgpu_buffer_rsrc_t rp = rlmd_rsrc(a.actor.p, ao.size * 4);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      wp[j] = few && j < A ? rlmd_ldf(rp, ao.w3 + (int64_t)j * ao.h2 + m.c, cin) : 0.f;
      wl[j] = few && sac && j < A ? rlmd_ldf(rp, ao.w4 + (int64_t)j * ao.h2 + m.c, cin) : 0.f;
    }
  }
  // the sampling save rows (A <= 2: registers) before the masks and fragments, so
  // the sampling backward waits on them alone (vmcnt retires in issue order)
  const int r = threadIdx.x;
  float svr[5][2];  // [mu, sigma, c, u, log_scale] x action j
  {
    const bool few = A <= 2, own = r < R && row0 + r < B;
    const __amdgpu_buffer_rsrc_t rs = rlmd_rsrc(a.save, (int64_t)B * 5 * A * 4);
#pragma unroll
    for (int q = 0; q < 5; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        svr[q][j] = rlmd_ldf(rs, (int64_t)(row0 + r) * 5 * A + q * A + j, few && own && j < A);
  }
  bwd_mask<NBW>(ka, a.am1, a.am2, nullptr, ao, row0, B);
  Pre<PREC, NBW, MULTI>& pa = p0;  // reuse the first critic's fragment registers
  pre_issue<PREC, NBW, MULTI>(pa, a.actor.wt, H2p, H2p, H1p / 16);
  if (r < R) {
    const int b = row0 + r;
    if (b < B) {
      const float* sv = a.save + (int64_t)b * 5 * A;
      auto one = [&](int j, float mu, float sg, float c, float u, float ls) {
        const float da = hout[r * kHeadsMax + j];
        if (sac) {
          float dmu, dls;
          policy_comp_bwd(a.smp.dist, mu, sg, c, u, ls, da, dlogp_r[r], a.smp.max_action, a.smp.reparam_noise,
                          a.smp.ls_min, a.smp.ls_max, dmu, dls);
          ghs[r * kHeadsMax + j] = dmu;
          ghs[r * kHeadsMax + A + j] = dls;
          a.gh[(int64_t)b * 2 * A + j] = dmu;
          a.gh[(int64_t)b * 2 * A + A + j] = dls;
        } else {
          const float t = tanhf(mu);
          const float dpre = da * a.smp.max_action * (1.f - t * t);
          ghs[r * kHeadsMax + j] = dpre;
          a.gh[(int64_t)b * 2 * A + j] = dpre;
        }
      };
      if (A <= 2) {  // the preloaded registers, constant indices
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (j < A) one(j, svr[0][j], svr[1][j], svr[2][j], svr[3][j], svr[4][j]);
      } else {
        for (int j = 0; j < A; ++j) one(j, sv[j], sv[A + j], sv[2 * A + j], sv[3 * A + j], sv[4 * A + j]);
      }
    } else {
      for (int j = 0; j < 2 * A; ++j) ghs[r * kHeadsMax + j] = 0.f;
    }
    // the dh2 pass reads columns 0..3 of every row unconditionally (A <= 2)
    for (int q = sac ? 2 * A : A; q < 4; ++q) ghs[r * kHeadsMax + q] = 0.f;
  }
  __syncthreads();
  RLMD_TSR(109);
  // ---- dh2 = (gh . [W_pi; W_ls]) * [h2 > 0]
  {
    const int H2 = ao.h2;
    const ElemMap m = elem_map(H2p);
    const float* P = a.actor.p;
    const bool cin = m.c < H2, few = A <= 2;
    RLMD_TSR(106);
#pragma unroll
    for (int rr = 0; rr < kMR<NBW>; ++rr) {
      const int rw = m.r0 + rr;
      if (rw < m.r1) {
        float acc = 0.f;
        if (few) {
          // unconditional reads (zero-filled columns, zero weights past A): no
          // branch between them; the log-scale gradients sit at columns A + j
          const float* gr = ghs + rw * kHeadsMax;
          const float g0 = gr[0], g1 = gr[1], g2 = gr[2], g3 = gr[3];
          const float l0 = A == 1 ? g1 : g2, l1 = A == 1 ? g2 : g3;
          acc = fmaf(g0, wp[0], acc);
          acc = fmaf(l0, wl[0], acc);
          acc = fmaf(g1, wp[1], acc);
          acc = fmaf(l1, wl[1], acc);
        } else if (cin) {
          for (int j = 0; j < A; ++j) {
            acc = fmaf(ghs[rw * kHeadsMax + j], P[ao.w3 + (int64_t)j * H2 + m.c], acc);
            if (sac) acc = fmaf(ghs[rw * kHeadsMax + A + j], P[ao.w4 + (int64_t)j * H2 + m.c], acc);
          }
        }
        const float v = ka.m2[rr] > 0.f ? acc : 0.f;
        aT[rw * L.ldaT + m.c] = CT<PREC>::cvt(v);
        if (m.c < H2 && row0 + rw < B) a.dh2[(int64_t)(row0 + rw) * H2 + m.c] = v;
      }
    }
  }
  RLMD_TSR(107);
  __syncthreads();
  RLMD_TSR(110);
  dh1_rows<PREC, NBW, MULTI>(pa, a.actor, ao, ka, aT, L.ldaT, a.dh1, nullptr, 0, nullptr, row0, B);
  RLMD_TSR(111);
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
    wc[frag_index(n, k, H1p, PREC == RLMD_BF16)] = v;
    wt[frag_index(k, n, H2p, PREC == RLMD_BF16)] = v;
  }
}

template <int PREC, int NBW, bool MULTI>
void launch_kind(int kind, const void* args, dim3 grid, size_t lds, hipStream_t st) {
  switch (kind) {
    case 0:
      hipLaunchKernelGGL((fwd_rows_kernel<PREC, NBW, MULTI>), grid, dim3(NT), lds, st,
                         *static_cast<const FwdRowsArgs*>(args));
      break;
    case 1:
      hipLaunchKernelGGL((qeval_rows_kernel<PREC, NBW, MULTI>), grid, dim3(NT), lds, st,
                         *static_cast<const QEvalArgs*>(args));
      break;
    case 2:
      hipLaunchKernelGGL((cbwd_rows_kernel<PREC, NBW, MULTI>), grid, dim3(NT), lds, st,
                         *static_cast<const CBwdArgs*>(args));
      break;
    default:
      if (static_cast<const ABwdArgs*>(args)->nq > 1)
        hipLaunchKernelGGL((abwd_rows_kernel<PREC, NBW, MULTI, 2>), grid, dim3(NT), lds, st,
                           *static_cast<const ABwdArgs*>(args));
      else
        hipLaunchKernelGGL((abwd_rows_kernel<PREC, NBW, MULTI, 1>), grid, dim3(NT), lds, st,
                           *static_cast<const ABwdArgs*>(args));
      break;
  }
}

// NBW = column blocks per wave (8 waves x 16 columns each), MULTI when the K
// loop needs more than the 16 prefetched fragments per lane.
template <int PREC>
int launch_prec(const RowDims& d, int kind, const void* args, int ny, hipStream_t st, int extra_x, int nz) {
  const int H = d.H1p > d.H2p ? d.H1p : d.H2p;
  const dim3 grid((d.B + R - 1) / R + extra_x, ny, nz);
  const size_t lds = (size_t)lds_layout(d).total;
  const int nsteps = H / CT<PREC>::KS;
  if (H <= 128) {
    if (nsteps <= 16) launch_kind<PREC, 1, false>(kind, args, grid, lds, st);
    else launch_kind<PREC, 1, true>(kind, args, grid, lds, st);
  } else if (H <= 256) {
    if (nsteps <= 8) launch_kind<PREC, 2, false>(kind, args, grid, lds, st);
    else launch_kind<PREC, 2, true>(kind, args, grid, lds, st);
  } else {
    launch_kind<PREC, 4, true>(kind, args, grid, lds, st);
  }
  RLMD_LAUNCH_CHECK();
  return 0;
}

int launch_rows(const RowDims& d, int kind, const void* args, int ny, hipStream_t st, int extra_x = 0, int nz = 1) {
  RLMD_CHECK(d.H1 <= 512 && d.H2 <= 512, "row kernels: hidden widths up to 512");
  RLMD_CHECK(d.A <= RLMD_MAX_ACTION, "row kernels: too many actions");
  RLMD_CHECK(lds_layout(d).total <= 160 * 1024, "row kernels: LDS budget exceeded");
  if (d.B <= 0) return 0;
  return d.prec == RLMD_BF16 ? launch_prec<RLMD_BF16>(d, kind, args, ny, st, extra_x, nz)
                             : launch_prec<RLMD_FP32>(d, kind, args, ny, st, extra_x, nz);
}

}  // namespace

size_t rows_lds_bytes(const RowDims& d) { return (size_t)lds_layout(d).total; }

}  // namespace rlmd

#ifdef RLMD_TIMING
extern "C" int rlmd_debug_ts_rows(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlmd::g_ts_rows), sizeof(unsigned long long) * 128) == hipSuccess ? 0 : 2;
}
#endif

namespace rlmd {

int fwd_rows_launch(const FwdRowsArgs& a, hipStream_t st, int split) {
  RLMD_CHECK(a.y0 == 0 || a.y0 == 2, "fwd_rows: y0 is 0 or 2");
  RLMD_CHECK(a.npair == 0 || (a.y0 == 0 && a.s2n && a.qtn[0] && a.qtn[1]), "fwd_rows: target pairing buffers");
  RLMD_CHECK(split == 1 || (split == 2 && a.u1[0] && a.d.H2p % 64 == 0),
             "fwd_rows: a column split needs the fused critic path and H2p a multiple of 64");
  return launch_rows(a.d, 0, &a, (a.with_actor ? 5 : 4) - a.y0 + 2 * a.npair, st, 0, split);
}
int qeval_rows_launch(const QEvalArgs& a, int nq, hipStream_t st, int split) {
  RLMD_CHECK(a.nq == nq && (a.nab == 0 || (a.ua && a.wheads && a.am1 && a.am2)), "qeval_rows: head jobs need their buffers");
  RLMD_CHECK(a.split == split && (split == 1 || (split == 2 && a.dqda[0] && a.d.H2p % 64 == 0)),
             "qeval_rows: a column split needs the fused actor path and H2p a multiple of 64");
  return launch_rows(a.d, 1, &a, nq * split + a.nab, st);
}
// cbwd: dh1 columns in halves when each half is a whole number of column blocks
// per wave (the per-workgroup W2^T stream is the kernel's cost)
int cbwd_rows_launch(const CBwdArgs& a, hipStream_t st) {
  const int nb = a.d.H1p / 16;
  const int nz = (nb % (2 * NW) == 0) ? 2 : 1;
  return launch_rows(a.d, 2, &a, 2, st, 0, nz);
}
int abwd_rows_launch(const ABwdArgs& a, hipStream_t st) {
  const bool ext = a.dqn_ext[0] != nullptr;
  RLMD_CHECK(ext || a.d.B <= NT, "fused actor loss: mini-batch up to 512 rows");
  RLMD_CHECK(a.cstats.B <= NT, "critic statistics workgroup: mini-batch up to 512 rows");
  // + the actor-loss workgroup, + the critic-statistics workgroup
  return launch_rows(a.d, 3, &a, 1, st, (ext ? 0 : 1) + (a.cstats.B > 0 ? 1 : 0));
}

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
