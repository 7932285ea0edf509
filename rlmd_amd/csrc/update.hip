// update.hip — the critic step of learn() as ONE launch (gfx950, wave64).
//
// The reference's critic step (algos/algo_sac.py:413-479, algo_td3.py:395-470)
// is: the loss over the mini-batch (tools/critic_loss.py, top-k of the summed
// losses), autograd through both critics, torch.optim.Adam, the Polyak update
// of the targets.  As separate launches that chain is row backward -> weight-
// gradient GEMM -> Adam, three kernel boundaries and three dependent load
// rounds.  Here every workgroup owns a set of parameters outright and computes
// their gradient over ALL mini-batch rows itself, so it can step them at once:
//
//   * every workgroup forms the loss gradient dq of every row (the loss inputs
//     are B floats per critic; the top-k selection is one block_rank), so no
//     workgroup waits for another;
//   * dh2[b, i] = dq[b] w3[i] [h2 > 0] is elementwise, and dh1 = dq * U1 with the
//     backward basis U1 = [h1 > 0] * (([h2 > 0] w3) W2) that the forward row
//     kernel already produced (rows.hip) — the same contraction with the
//     per-row scalar dq factored out;
//   * dW2 tiles (32 x 32 of fc2.weight, MFMA over the B rows as K), with db2,
//     dW3 / db3 (q_value) on the tiles of the first column; dW1 / db1 blocks of
//     32 fc1 rows (VALU over the rows);
//   * the workgroup then applies Adam, the Polyak target update and the bf16 /
//     f32 compute copies (rlmd_adam.h) to exactly the parameters it owns.
//
// Reductions are in a fixed order (row k-steps per wave, then waves 0..7), so
// the step is deterministic.  Inputs the step also writes (q_value weight and
// biases) are read from the forward kernel's snapshots.
#include "learn_kernels.h"
#include "rlmd_adam.h"
#include "rlmd_block.h"
#include "rlmd_loss.h"
#include "rlmd_policy.h"
#include "rlmd_update.h"

namespace rlmd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int NT = 512;
#ifndef RLMD_W1_HALF
#define RLMD_W1_HALF 1  // the actor step's fc1 blocks 16 units wide (0: 32): twice the blocks, half the bases each
#endif
constexpr int TW = 32;
// the actor step's fc1 block width: its bases (nh x B x TW1 f32) made it the
// launch's last workgroup to finish at 32 (128 KB of loads at C2)
constexpr int TW1 = RLMD_W1_HALF ? 16 : 32;
constexpr int kW1G = NT / TW1;      // row groups of an fc1 block (a thread per unit and group)
constexpr int kW1R = 512 / kW1G;    // rows per group (B <= 512)
constexpr int kW1Q = kW1R / 4;      // f32x4 base loads per thread and head
// timing ablations (experiment builds only, RLMD_EXTRA_FLAGS=-DRLMD_ABL=<bits>; the
// results are wrong): 1 no ranking (rank = row), 2 no optimiser step / copies
#ifndef RLMD_ABL
#define RLMD_ABL 0
#endif
#ifndef RLMD_ROLE_SPLIT
#define RLMD_ROLE_SPLIT 1  // role-specialised update bodies (0: one body, roles' loads predicated off)
#endif
#ifndef RLMD_SPLIT_SPEC
#define RLMD_SPLIT_SPEC 1  // critic step bodies specialised on fwd_rows' column split (0: one body, halves predicated)
#endif
#ifndef RLMD_W1_EARLY
#define RLMD_W1_EARLY 1  // the actor step's fc1 block loads its operands before the ranking (0: after)
#endif
template <int NW>
__device__ __forceinline__ void upd_rank(uint64_t key, uint64_t* runs, int* out) {
  if constexpr ((RLMD_ABL & 1) != 0) {
    out[threadIdx.x] = (int)threadIdx.x;
    __syncthreads();
  } else {
    block_rank<NW>(key, runs, out);
  }
}  // tile edge (fc2.weight tiles TW x TW, fc1 blocks of TW rows)

#ifdef RLMD_TIMING
// experiment builds only (tools/ts_probe.py upd): thread-0 s_memtime stamps of
// three workgroups (slot 0: tile (0, 0), 1: tile (0, 1), 2: the first fc1 block)
__device__ unsigned long long g_ts_upd[128];
__device__ unsigned long long g_ts_aupd[128];
#ifdef RLMD_TIMING_WINDOWS  // entry / exit windows only: the phase stamps perturb the register allocation
#define RLMD_TS_ON(i) ((i) >= 14)
#else
#define RLMD_TS_ON(i) true
#endif
// RLMD_TIMING_DRAIN: the exit stamp waits until the workgroup's stores have completed
#ifdef RLMD_TIMING_DRAIN
#define RLMD_TS_DRAIN(i)                              \
  if ((i) == 15) {                                    \
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    __syncthreads();                                  \
  }
#else
#define RLMD_TS_DRAIN(i)
#endif
#define RLMD_TSU(i)                                                                       \
  do {                                                                                    \
    RLMD_TS_DRAIN(i)                                                                      \
    if (RLMD_TS_ON(i) && threadIdx.x == 0 && ts_slot >= 0)                                \
      g_ts_upd[ts_slot * 16 + (i)] = (i) >= 14 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime(); \
  } while (0)
// actor step: cycles (i < 14) and the constant-rate clock (i = 14, 15: entry / exit)
#define RLMD_TSA(i)                                                                        \
  do {                                                                                     \
    RLMD_TS_DRAIN(i)                                                                       \
    if (RLMD_TS_ON(i) && threadIdx.x == 0 && ts_slot >= 0)                                 \
      g_ts_aupd[ts_slot * 16 + (i)] = (i) >= 14 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define RLMD_TSU(i) \
  do {              \
  } while (0)
#define RLMD_TSA(i) \
  do {              \
  } while (0)
#endif

// f32 -> bf16, round to nearest even: the plain cast lowers to v_cvt_pk_bf16_f32
// (NaN stays NaN; no per-element branch)
__device__ __forceinline__ unsigned short bf16_rne(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}

// The compute copies of one stepped 32 x 32 fc2.weight tile (rows i0.., columns
// j0..; new values in LDS, pcl[(i - i0) * 33 + (j - j0)], the Polyak targets'
// at pcl + 32 * 33): the tile is 2 KB contiguous in each fragment-major copy
// (frag_index: 16-row bands x KS-column steps of 64 lanes x EPF elements), so
// the workgroup writes it as 16-byte chunks, one (copy, block, lane) per job,
// instead of one 2- or 4-byte store per element per copy.
template <int PREC>
__device__ __forceinline__ void tile_copies(const float* pcl, const CopyDst& cd, bool targets, int i0, int j0, int H1p,
                                            int H2p) {
  constexpr bool BF = PREC == RLMD_BF16;
  constexpr int KS = BF ? 32 : 16, EPF = KS / 4, NBLK = 2 * (32 / KS);  // blocks per tile
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int njobs = (targets ? 4 : 2) * NBLK * 64;
  for (int jb = threadIdx.x; jb < njobs; jb += NT) {
    const int lane = jb & 63, blk = (jb >> 6) % NBLK, c = (jb >> 6) / NBLK;  // c: wc, wt, twc, twt
    const bool tr = c & 1;
    const float* src = pcl + (c >= 2 ? 32 * 33 : 0);
    const int rb = blk % 2, st = blk / 2;                 // 16-row band, KS-column step inside the tile
    const int row = 16 * rb + (lane & 15), col0 = st * KS + (lane >> 4) * EPF;  // tile-relative
    float v[EPF];
#pragma unroll
    for (int e = 0; e < EPF; ++e) v[e] = tr ? src[(col0 + e) * 33 + row] : src[row * 33 + col0 + e];
    // global chunk: wc (n = i0 + row, k = j0 + col), wt (k = j0 + row, n = i0 + col)
    const int64_t at = tr ? frag_index(j0 + row, i0 + col0, H2p, BF) : frag_index(i0 + row, j0 + col0, H1p, BF);
    void* dst = c == 0 ? cd.wc : c == 1 ? cd.wt : c == 2 ? cd.twc : cd.twt;
    u32x4 w;
    if constexpr (BF) {
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = (uint32_t)bf16_rne(v[2 * q]) | ((uint32_t)bf16_rne(v[2 * q + 1]) << 16);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = __float_as_uint(v[q]);
    }
    __builtin_amdgcn_raw_buffer_store_b128(w, rlmd_rsrc_wave(dst, 0x7fffffff),
                                           (int)(at * (BF ? 2 : 4)), 0, RLMD_WT_AUX);
  }
}

// Operand fragments of one K-step over rows: bf16 16x16x32 (8 rows per lane) or
// f32 4 x 16x16x4 (4 rows per lane, k = 4 q + j).
template <int PREC>
struct KT;
template <>
struct KT<RLMD_BF16> {
  static constexpr int RPL = 8;   // consecutive rows per lane
  static constexpr int KS = 32;   // rows per K-step
  using T = unsigned short;
  using Frag = bf16x8;
  __device__ __forceinline__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static Frag load_b(__amdgpu_buffer_rsrc_t r, int64_t elem, bool ok) {
    return __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (int)(elem * 2) : 0x7fffffff, 0, 0));
  }
  // 8 mask bytes of this lane's rows
  __device__ __forceinline__ static void load_mask(__amdgpu_buffer_rsrc_t r, int64_t byte, bool ok, uint32_t (&w)[2]) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, ok ? (int)byte : 0x7fffffff, 0, 0));
    w[0] = v[0];
    w[1] = v[1];
  }
  __device__ __forceinline__ static Frag form_a(const uint32_t (&w)[2], const float* dq, float w3) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t byte = (w[e >> 2] >> (8 * (e & 3))) & 0xffu;
      f[e] = (short)bf16_rne(byte ? dq[e] * w3 : 0.f);
    }
    return f;
  }
};
template <>
struct KT<RLMD_FP32> {
  static constexpr int RPL = 4;
  static constexpr int KS = 16;
  using T = float;
  using Frag = f32x4;
  __device__ __forceinline__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  }
  __device__ __forceinline__ static Frag load_b(__amdgpu_buffer_rsrc_t r, int64_t elem, bool ok) {
    return __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (int)(elem * 4) : 0x7fffffff, 0, 0));
  }
  __device__ __forceinline__ static void load_mask(__amdgpu_buffer_rsrc_t r, int64_t byte, bool ok, uint32_t (&w)[2]) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, ok ? (int)byte : 0x7fffffff, 0, 0);
    w[1] = 0;
  }
  __device__ __forceinline__ static Frag form_a(const uint32_t (&w)[2], const float* dq, float w3) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = ((w[0] >> (8 * e)) & 0xffu) ? dq[e] * w3 : 0.f;
    return f;
  }
};

__device__ __forceinline__ int64_t rp_idx(int row, int Hp, int col) {
  return (((int64_t)(row >> 4) * Hp + col) << 4) + (row & 15);
}

// LDS of the critic update (bytes)
struct ULds {
  static constexpr int dq = 0;                  // f32 [512] loss gradient per row
  static constexpr int runs = dq + 512 * 4;     // u64 [512] block_rank runs
  static constexpr int rank = runs + 512 * 8;   // int [512]
  static constexpr int red = rank + 512 * 4;    // block reductions (16 * 9 floats)
  static constexpr int part = red + 16 * 9 * 4; // f32 [8 waves][4 blocks][256] partial tiles / row partials
  static constexpr int xs = part + 8 * 4 * 256 * 4;  // f32 [512][8] critic inputs (fc1 blocks)
  static constexpr int pcl = xs + 512 * 8 * 4;       // f32 [2 halves][2][32][33] stepped tile + targets (copies)
  static constexpr int total = pcl + 2 * 2 * 32 * 33 * 4;
};

// WIDE (mini-batch B <= 256, e.g. TD3's 200): a tile workgroup owns 32 x 64 of
// fc2.weight — waves 0-3 cover the batch's 256 rows for columns [j0, j0 + 32),
// waves 4-7 for [j0 + 32, j0 + 64) — where the 32 x 32 form would leave waves
// 4-7 on rows past B.  Half the tile workgroups: TD3 400/300's 2 x 153 of them
// exceed the 256 CUs at one workgroup per CU (a second dispatch round); 2 x 88 do not.
// Roles of the critic step's workgroups: an fc2.weight tile, an fc1 block, a head
// workgroup (b2 / w3 of 32 fc2 rows, b3 on the first).  The role is a template
// parameter of the body, so each workgroup issues exactly its own role's first
// load round: issued predicated-off, the other roles' loads had cost a third of the
// launch in texture-addresser issue (TA_TA_BUSY, profiles/r06_pmc_ta.json).
enum { kRoleW2 = 0, kRoleW1 = 1, kRoleHead = 2 };

template <int PREC, bool WIDE, int ROLE, bool SPLIT>
__device__ __forceinline__ void critic_update_body(const CritUpdArgs& a, unsigned char* smem, int g, int t);

// SPLIT false (fwd_rows unsplit, a.loss.qsplit == 1): the bodies without the
// second halves' loads of q / target q / U1 — predicated off, each still cost the
// texture addresser a wave-instruction
template <int PREC, bool WIDE, bool SPLIT>
__global__ void __launch_bounds__(NT) critic_update_kernel(CritUpdArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // per critic: fc2.weight tiles, fc1 blocks, then head workgroups (b2 / w3 of 32
  // fc2 rows each, b3 on the first)
  const int per = a.n_w2 + a.n_w1 + a.ti;
  if ((int)blockIdx.x >= 2 * per) {
    // the critic statistics of an update without an actor step (rlmd_loss.h), beside
    // the step: they read the loss scalars' starting slot, part 0 writes the other
    critic_loss_block<NT / 64>(a.cstats, reinterpret_cast<uint64_t*>(smem + ULds::runs),
                               reinterpret_cast<int*>(smem + ULds::part), reinterpret_cast<float*>(smem + ULds::red),
                               (int)blockIdx.x - 2 * per);
    return;
  }
  const int g = blockIdx.x / per, t = blockIdx.x - g * per;
#if RLMD_ROLE_SPLIT
  if (t < a.n_w2) critic_update_body<PREC, WIDE, kRoleW2, SPLIT>(a, smem, g, t);
  else if (t >= a.n_w2 + a.n_w1) critic_update_body<PREC, WIDE, kRoleHead, SPLIT>(a, smem, g, t);
  else critic_update_body<PREC, WIDE, kRoleW1, SPLIT>(a, smem, g, t);
#else
  critic_update_body<PREC, WIDE, -1, SPLIT>(a, smem, g, t);
#endif
}

// ROLE -1: one body for every role, the roles' loads issued predicated-off (the
// round-5 form, RLMD_ROLE_SPLIT=0)
template <int PREC, bool WIDE, int ROLE, bool SPLIT>
__device__ __forceinline__ void critic_update_body(const CritUpdArgs& a, unsigned char* smem, int g, int t) {
  using K = KT<PREC>;
  float* dqs = reinterpret_cast<float*>(smem + ULds::dq);
  float* part = reinterpret_cast<float*>(smem + ULds::part);
  const RowDims& d = a.d;
  const NetOff& co = a.co;
  const int B = d.B, H1 = d.H1, H2 = d.H2, H1p = d.H1p, H2p = d.H2p, X = d.X;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = (B + 15) / 16;
  // this workgroup's role; IS_* = the role's loads are compiled in
  constexpr bool IS_W2 = ROLE < 0 || ROLE == kRoleW2, IS_W1 = ROLE < 0 || ROLE == kRoleW1,
                 IS_HEAD = ROLE < 0 || ROLE == kRoleHead;
  const bool w2tile = ROLE < 0 ? t < a.n_w2 : ROLE == kRoleW2;
  const bool first_col = ROLE < 0 ? t >= a.n_w2 + a.n_w1 : ROLE == kRoleHead;  // first_col: a head workgroup
  constexpr int TJ = WIDE ? 2 * TW : TW;  // fc2.weight columns per tile
  constexpr int NH = WIDE ? 2 : 1;        // 32-column halves per tile
  const int i0 = w2tile ? (t / a.tj) * TW : first_col ? (t - a.n_w2 - a.n_w1) * TW : 0;
  const int j0 = w2tile ? (t % a.tj) * TJ : first_col ? 0 : (t - a.n_w2) * TW;
  const bool w1blk = ROLE < 0 ? !w2tile && !first_col : ROLE == kRoleW1;
  const int wrow = WIDE ? (wave & 3) : wave;     // this wave's 64-row slice of the batch
  const int jw = j0 + (WIDE ? 32 * (wave >> 2) : 0);  // and its 32-column half
  const int64_t pbase = (int64_t)g * co.size;  // this critic's parameters in the Adam base
  const bool polyak = adam_polyak(a.adam);
  const CopyDst cd = copy_dst(a.adam, g);
  // Adam on an element of this critic (fc2.weight elements also refresh the copies)
  auto step = [&](int pi, float gv, const AdamIn& in) {
    const int j = pi - (int)pbase - (int)co.w2;
    if (!(RLMD_ABL & 2)) adam_apply_dst(a.adam, pi, gv, in, polyak, (j >= 0 && j < H1 * H2) ? j : -1, cd);
  };
  const int bx = blockIdx.x, pb = a.n_w2 + a.n_w1 + a.ti;
  const int ts_slot = bx == 0 ? 0 : bx == 1 ? 1 : bx == a.n_w2 ? 2 : bx == a.n_w2 + a.n_w1 ? 3 : bx == pb ? 4
                    : bx == (int)gridDim.x - 1 ? 5 : -1;
  (void)ts_slot;
  RLMD_TSU(14);
  RLMD_TSU(0);

  // ---- first load round: loss inputs, this workgroup's operands, Adam state.
  //      Branch-free: every load is issued by every workgroup, predicated through
  //      the range check on its role (a load inside `if (role)` is copied out of
  //      its registers at the merge, which waits for it on the spot)
  const CriticLoads cl = critic_row_load<SPLIT>(a.loss);
  // (a) dW2 tile: per wave rows [64 w, 64 w + 64), per K-step the A masks (two i
  //     sub-blocks) and B fragments (two j sub-blocks)
  constexpr int NKS = 64 / K::KS;
  uint32_t mw[NKS][2][2];
  typename K::Frag bf[NKS][2];
  const __amdgpu_buffer_rsrc_t rm2 = rlmd_rsrc(a.m2[g], (int64_t)nrb * H2p * 16),
                               rh1 = rlmd_rsrc(a.hp1[g], (int64_t)nrb * H1p * 16 * sizeof(typename K::T));
  float w3l[2];
  if constexpr (IS_W2) {
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int row = 64 * wrow + s * K::KS + K::RPL * (lane >> 4);
    const bool rok = w2tile && row < nrb * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = i0 + 16 * h + (lane & 15), j = jw + 16 * h + (lane & 15);
      K::load_mask(rm2, rp_idx(row, H2p, i), rok && i < H2p, mw[s][h]);
      bf[s][h] = K::load_b(rh1, rp_idx(row, H1p, j), rok && j < H1p);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = i0 + 16 * h + (lane & 15);
    w3l[h] = rlmd_ldf(rlmd_rsrc(a.w3s[g], (int64_t)H2 * 4), i, w2tile && i < H2);
  }
  }
  // (b) Adam state of the owned parameters: 1024 elements per 32-column half, 2
  //     per thread and half
  int pidx[NH][2];
  AdamIn ain[NH][2];
  if constexpr (IS_W2) {
#pragma unroll
  for (int hf = 0; hf < NH; ++hf)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int el = tid * 2 + e, blk = el >> 8, ln = (el >> 2) & 63, rg = el & 3;
      const int i = i0 + 16 * (blk >> 1) + 4 * (ln >> 4) + rg, j = j0 + 32 * hf + 16 * (blk & 1) + (ln & 15);
      pidx[hf][e] = (w2tile && i < H2 && j < H1) ? (int)(pbase + co.w2 + (int64_t)i * H1 + j) : -1;
      ain[hf][e] = adam_load(a.adam, pidx[hf][e], polyak);
    }
  }
  // (c) first-column tiles: this thread's column of h2 and [h2 > 0] over its 32 rows
  //     (thread: column i0 + tid % 32, rows [32 p, 32 p + 32) of part p = tid / 32)
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr int NV = 16 * sizeof(typename K::T) / 16;  // 16-byte loads per 16 rows of h2
  u32x4 fmb[2], fhv[2][NV];
  if constexpr (IS_HEAD) {
    const int ci = tid & 31, p = tid >> 5, i = i0 + ci;
    const __amdgpu_buffer_rsrc_t rh2 = rlmd_rsrc(a.hp2[g], (int64_t)nrb * H2p * 16 * sizeof(typename K::T));
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      const int r0 = 32 * p + 16 * hb;
      const bool ok = first_col && r0 < nrb * 16;
      const int64_t ix = rp_idx(r0, H2p, i);
      fmb[hb] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rm2, ok ? (int)ix : 0x7fffffff, 0, 0));
#pragma unroll
      for (int v = 0; v < NV; ++v)
        fhv[hb][v] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rh2, ok ? (int)(ix * sizeof(typename K::T) + 16 * v) : 0x7fffffff,
                                                   0, 0));
    }
  }
  // (e) Adam state of the parameters stepped after the tile: on the first tile
  //     column b2 / w3 (threads 0..63) and b3 (thread 64 of tile 0), on an fc1
  //     block W1 / b1 (thread c * 32 + jj: input c < X, or c = 8 for the bias)
  int xpi = -1;
  {
    const int c = i0 + (tid & 31);
    if (first_col && tid < 64 && c < H2) xpi = (int)(pbase + (tid < 32 ? co.b2 + c : co.w3 + c));
    if (first_col && tid == 64 && i0 == 0) xpi = (int)(pbase + co.b3);
    const int jj = tid & 31, ci = tid >> 5, jr = j0 + jj;
    if (w1blk && tid < 32 * 9 && (ci < X || ci == 8) && jr < H1)
      xpi = (int)(pbase + (ci == 8 ? co.b1 + jr : co.w1 + (int64_t)jr * X + ci));
  }
  AdamIn xin{};
  if constexpr (IS_W1 || IS_HEAD) xin = adam_load(a.adam, xpi, polyak);
  float w3c = 0.f;
  if constexpr (IS_HEAD) w3c = rlmd_ldf(rlmd_rsrc(a.w3s[g], (int64_t)H2 * 4), i0 + (tid & 31), first_col && tid < 32);
  // (d) fc1 blocks: the critic inputs of this thread's 8 LDS slots and U1 of its
  //     column over its 32 rows
  float* xs = reinterpret_cast<float*>(smem + ULds::xs);
  float xv[8];
  f32x4 u1v[8], u1w[8];  // U1, and its second partial half (fwd_rows column split)
  if constexpr (IS_W1) {
    const __amdgpu_buffer_rsrc_t rx = rlmd_rsrc(a.x, (int64_t)B * X * 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + q * NT, r = e >> 3, c = e & 7;
      xv[q] = rlmd_ldf(rx, (int64_t)r * X + c, w1blk && r < B && c < X);
    }
    const int cj = tid & 31, p = tid >> 5, j = j0 + cj;
    const bool us = SPLIT && a.loss.qsplit > 1;
    const int64_t ustr = (int64_t)nrb * H1p * 16;
    const __amdgpu_buffer_rsrc_t ru = rlmd_rsrc(a.u1[g], ustr * (us ? 2 : 1) * 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = 32 * p + 4 * q;
      const bool ok = w1blk && r < nrb * 16 && j < H1p;
      u1v[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             ru, ok ? (int)(rp_idx(r, H1p, j) * 4) : 0x7fffffff, 0, 0));
      if constexpr (SPLIT)
        u1w[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               ru, (ok && us) ? (int)((ustr + rp_idx(r, H1p, j)) * 4) : 0x7fffffff, 0, 0));
      else
        u1w[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }

  RLMD_TSU(1);
  // ---- the loss gradient of every row (critic g): critic_row_loss, top-k by
  //      rank among all B keys (critic_loss.py:438-453)
  {
    float* red = reinterpret_cast<float*>(smem + ULds::red);
    CriticRow o;
    // the block sums only where the loss itself needs them (CIM kernel, TCAU
    // truncation): the statistics workgroups form the rest (rlmd_loss.h)
#ifndef RLMD_LOSS_BLOCK_ALWAYS
    critic_row_loss(a.loss, red, o, cl, critic_loss_needs_block(a.loss));
#else
    critic_row_loss(a.loss, red, o, cl);
#endif
    RLMD_TSU(2);
    const int kk = B > a.loss.k ? a.loss.k : B;
    bool sel = o.in;
    if (B > a.loss.k) {
      int* rank_of = reinterpret_cast<int*>(smem + ULds::rank);
      upd_rank<NT / 64>(critic_sel_key(o), reinterpret_cast<uint64_t*>(smem + ULds::runs), rank_of);
      sel = o.in && rank_of[tid] < kk;
      if (blockIdx.x == 0 && a.rank_out && o.in) a.rank_out[tid] = rank_of[tid];  // for the statistics
    }
    dqs[tid] = sel ? a.loss.grad_scale * (g == 0 ? o.dl[0] : o.dl[1]) / (float)kk : 0.f;
    // learn_step_cntr; log alpha carried into this update's slot (no temperature here)
    if (blockIdx.x == 0 && tid == 0) adam_scalar_step(a.adam);
  }
  __syncthreads();
  RLMD_TSU(3);

  if (IS_W2 && w2tile) {
    // ---- dW2[i0.., j0..] = sum_b dh2[b, i] h1[b, j] over this wave's rows
    f32x4 acc[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int v = 0; v < 2; ++v) acc[h][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int row = 64 * wrow + s * K::KS + K::RPL * (lane >> 4);
      float dq[K::RPL];
#pragma unroll
      for (int e = 0; e < K::RPL; ++e) dq[e] = dqs[(row + e) & 511];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const typename K::Frag af = K::form_a(mw[s][h], dq, w3l[h]);
#pragma unroll
        for (int v = 0; v < 2; ++v) K::mfma(af, bf[s][v], acc[h][v]);
      }
    }
    // waves' partial tiles -> LDS, summed in wave order
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int v = 0; v < 2; ++v)
        *reinterpret_cast<f32x4*>(part + ((wave * 4 + h * 2 + v) * 64 + lane) * 4) = acc[h][v];
    __syncthreads();
    RLMD_TSU(4);
    float* pcl = reinterpret_cast<float*>(smem + ULds::pcl);
#pragma unroll
    for (int hf = 0; hf < NH; ++hf)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int el = tid * 2 + e, blk = el >> 8, ln = (el >> 2) & 63, rg = el & 3;
        const int ii = 16 * (blk >> 1) + 4 * (ln >> 4) + rg, jj = 16 * (blk & 1) + (ln & 15);
        float gs = 0.f;  // the half's waves in order (WIDE: 4 of 64 rows, else 8)
#pragma unroll
        for (int w = 0; w < 8 / NH; ++w) gs += part[(hf * (8 / NH) + w) * 1024 + el];
        float pn = 0.f, tn = 0.f;  // padding elements: zero in the copies
        if (pidx[hf][e] >= 0 && !(RLMD_ABL & 2)) adam_core(a.adam, pidx[hf][e], gs, ain[hf][e], polyak, pn, tn);
        float* ph = pcl + hf * 2 * 32 * 33;
        ph[ii * 33 + jj] = pn;
        ph[32 * 33 + ii * 33 + jj] = tn;
      }
    __syncthreads();
#pragma unroll
    for (int hf = 0; hf < NH; ++hf)
      if (j0 + 32 * hf < H1p)  // WIDE: the last tile's second half may lie past the padded width
        if (!(RLMD_ABL & 2)) tile_copies<PREC>(pcl + hf * 2 * 32 * 33, cd, polyak && cd.twc, i0, j0 + 32 * hf, H1p, H2p);
    RLMD_TSU(5);
  } else if (IS_HEAD && first_col) {
    {
      // ---- db2[i] = w3[i] sum_b dq[b] [h2 > 0], dW3[i] = sum_b dq[b] h2[b, i]
      //      (thread: column i0 + tid % 32, rows [32 p, 32 p + 32) of part p = tid / 32)
      const int ci = tid & 31, p = tid >> 5;
      float sm = 0.f, sh = 0.f;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {  // the part's two 16-row blocks of column i (prefetched)
        const int r0 = 32 * p + 16 * hb;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float q = dqs[r0 + e];
          const uint32_t byte = (fmb[hb][e >> 2] >> (8 * (e & 3))) & 0xffu;
          float h;
          if constexpr (PREC == RLMD_BF16) {
            const uint32_t w = fhv[hb][e >> 3][(e >> 1) & 3];
            h = __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
          } else {
            h = __uint_as_float(fhv[hb][e >> 2][e & 3]);
          }
          sm += byte ? q : 0.f;
          sh = fmaf(q, h, sh);
        }
      }
      part[p * 64 + ci] = sm;
      part[p * 64 + 32 + ci] = sh;
      __syncthreads();
      if (tid < 64 && xpi >= 0) {
        float v = 0.f;
        for (int q = 0; q < 16; ++q) v += part[q * 64 + tid];
        step(xpi, tid < 32 ? v * w3c : v, xin);
      }
      if (i0 == 0) {  // db3 = sum_b dq[b] (thread 64)
        float s3[1] = {dqs[tid]};
        float mx[1] = {-INFINITY};
        block_allreduce<1, 0>(s3, mx, reinterpret_cast<float*>(smem + ULds::red));
        if (tid == 64) step(xpi, s3[0], xin);
      }
      RLMD_TSU(6);
    }
  } else if (IS_W1) {
    // ---- dW1[j, x] = sum_b dq[b] U1[b, j] x[b, x], db1[j] = sum_b dq[b] U1[b, j]
    //      (thread: fc1 row j0 + tid % 32, rows [32 p, 32 p + 32) of part p)
    const int cj = tid & 31, p = tid >> 5;
#pragma unroll
    for (int q = 0; q < 8; ++q) xs[tid + q * NT] = xv[q];
    __syncthreads();
    const f32x4* u = u1v;
    float acc[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) acc[c] = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 32 * p + 4 * q + e;
        const float du = dqs[r] * (u[q][e] + u1w[q][e]);  // halves in order (u1w = 0 unsplit)
        acc[8] += du;
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = fmaf(du, xs[r * 8 + c], acc[c]);
      }
    RLMD_TSU(4);
    __syncthreads();  // xs / part
#pragma unroll
    for (int c = 0; c < 9; ++c) part[(p * 9 + c) * 32 + cj] = acc[c];
    __syncthreads();
    // 32 rows x (X + 1) outputs, thread c * 32 + jj (Adam state prefetched)
    if (xpi >= 0) {
      const int jj = tid & 31, c = tid >> 5;
      float v = 0.f;
      for (int q = 0; q < 16; ++q) v += part[(q * 9 + c) * 32 + jj];
      step(xpi, v, xin);
    }
    RLMD_TSU(5);
  }
  RLMD_TSU(7);
  RLMD_TSU(15);
}

// ---------------------------------------------------------------------------
// The actor (+ temperature) step in one launch (algos/algo_sac.py:524-595,
// algo_td3.py:503-531).  Every workgroup ranks all B rows' actor objective
// v = min(q1, q2) - alpha log pi (SAC, descending) / q1 (TD3, ascending) itself
// (Q5), forms dL/da = sum_c dL/dq_c dq_c/da with the critics' input gradients
// that qeval_rows produced, back-propagates through the policy's sampling and
// heads per row (gh = dL/d[mu, log_scale] or dL/d pre-tanh), and then, like the
// critic step: fc2.weight tiles with dh2 = [h2 > 0] * (gh . W_head), fc1 blocks
// with dh1 = sum_h gh[., h] U_h (the forward's per-head backward bases), the
// heads on the first tile column, Adam + Polyak + copies of what it owns.  One
// extra workgroup computes this update's critic statistics.  The last workgroup
// to finish reading log_alpha (an arrival counter) steps the temperature.
// ---------------------------------------------------------------------------
constexpr int kHM = 4;  // heads per row held in LDS (2 A; the fused actor step takes A <= 2)
constexpr int kAM = 2;  // actions

// dh2 = sum over the heads of gh[h] W_head[h] in the launch chain's order: mu_j
// then log_scale_j per action j (SAC), mu_j (TD3).  Position q of that order
// holds head head_at(q) (-1 past the nh heads), so that the sum runs over a
// fixed kHM positions with no runtime-indexed register arrays.
__device__ __forceinline__ int head_at(int q, int A, bool sac) {
  const int nh = sac ? 2 * A : A;
  return q >= nh ? -1 : !sac ? q : (q & 1) ? A + (q >> 1) : (q >> 1);
}

struct ALds {
  static constexpr int gh = 0;                      // f32 [512][kHM] head gradients per row (head order)
  static constexpr int ghp = gh + 512 * kHM * 4;    // the same in summation order (head_at), zero padded
  static constexpr int runs = ghp + 512 * kHM * 4;  // u64 [512]
  static constexpr int rank = runs + 512 * 8;       // int [3 * 512] (critic statistics: 3 ranks)
  static constexpr int red = rank + 3 * 512 * 4;    // 16 * 9 floats
  static constexpr int part = red + 16 * 9 * 4;     // f32 [8][4][256]
  // f32 [512][8] states of an fc1 block: read before the barrier ahead of the
  // block's partial sums, so they share part's bytes (68 KB in all: two actor
  // steps of two seeds fit one CU)
  static constexpr int xs = part;
  static constexpr int pcl = part + 8 * 4 * 256 * 4;  // f32 [2][32][33] stepped tile + targets (copies)
  static constexpr int total = pcl + 2 * 32 * 33 * 4;
};

template <int PREC, int ROLE>
__device__ __forceinline__ void actor_update_body(const ActUpdArgs& a, unsigned char* smem);

template <int PREC>
__global__ void __launch_bounds__(NT) actor_update_kernel(ActUpdArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // roles as in critic_update_kernel: tiles, fc1 blocks, head workgroups, then the
  // two critic-statistics workgroups (handled in the body's first branch)
  const int t = blockIdx.x;
#if RLMD_ROLE_SPLIT
  if (t < a.n_w2) actor_update_body<PREC, kRoleW2>(a, smem);
  else if (t < a.n_w2 + a.n_w1) actor_update_body<PREC, kRoleW1>(a, smem);
  else actor_update_body<PREC, kRoleHead>(a, smem);  // heads and the statistics workgroups
#else
  actor_update_body<PREC, -1>(a, smem);
#endif
}

template <int PREC, int ROLE>
__device__ __forceinline__ void actor_update_body(const ActUpdArgs& a, unsigned char* smem) {
  using K = KT<PREC>;
  constexpr bool IS_W2 = ROLE < 0 || ROLE == kRoleW2, IS_W1 = ROLE < 0 || ROLE == kRoleW1,
                 IS_HEAD = ROLE < 0 || ROLE == kRoleHead;
  float* ghs = reinterpret_cast<float*>(smem + ALds::gh);
  float* ghp = reinterpret_cast<float*>(smem + ALds::ghp);
  float* part = reinterpret_cast<float*>(smem + ALds::part);
  float* red = reinterpret_cast<float*>(smem + ALds::red);
  const RowDims& d = a.d;
  const NetOff& ao = a.ao;
  const int B = d.B, H1 = d.H1, H2 = d.H2, H1p = d.H1p, H2p = d.H2p, S = d.S, A = d.A;
  const bool sac = d.algo == RLMD_SAC;
  const int nh = sac ? 2 * A : A;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = (B + 15) / 16;
  const int t = blockIdx.x;
  (void)IS_W1;
  // workgroups: fc2.weight tiles, fc1 blocks, head workgroups (b2 and the heads
  // of 32 fc2 rows each), and two critic-statistics workgroups.  Every reader of
  // log alpha and the Cauchy scales takes the update's starting slot, the
  // temperature step (the last head workgroup) and statistics part 0 write the
  // other one (LearnState): no ordering between the workgroups is needed.
  // learn_cntr already holds this update's count (critic_update_kernel set it).
  const int n_hd = a.ti;
  const int nwg = a.n_w2 + a.n_w1 + n_hd;
  const int sidx = t - (a.n_w2 + a.n_w1 + n_hd);  // >= 0: statistics part
  const int ts_slot = t == 0 ? 0 : t == 1 ? 1 : t == a.n_w2 ? 2 : sidx == 0 ? 3 : t == a.n_w2 + a.n_w1 ? 4 : sidx == 1 ? 5 : -1;
  (void)ts_slot;
  RLMD_TSA(14);
  RLMD_TSA(0);
  LearnState* st = a.st;
  const bool stats_wg = IS_HEAD && sidx >= 0;
  const bool w2tile = ROLE < 0 ? t < a.n_w2 : ROLE == kRoleW2;
  const bool first_col = ROLE < 0 ? !stats_wg && t >= a.n_w2 + a.n_w1 : ROLE == kRoleHead && !stats_wg;  // a head workgroup
  const bool w1blk = ROLE < 0 ? !stats_wg && !w2tile && !first_col : ROLE == kRoleW1;
  const int i0 = w2tile ? (t / a.tj) * TW : first_col ? (t - a.n_w2 - a.n_w1) * TW : 0;
  const int j0 = w2tile ? (t % a.tj) * TW : w1blk ? (t - a.n_w2) * TW1 : 0;
  const bool polyak = adam_polyak(a.adam);
  const CopyDst cd = copy_dst(a.adam, 0);
  auto step = [&](int pi, float gv, const AdamIn& in) {
    const int j = pi - (int)ao.w2;
    if (!(RLMD_ABL & 2)) adam_apply_dst(a.adam, pi, gv, in, polyak, (j >= 0 && j < H1 * H2) ? j : -1, cd);
  };
  float v = 0.f, lpv = 0.f, alpha = 0.f;
  bool sel = false;
  int kk = B;
  // the last head workgroup writes the actor-loss value and steps the
  // temperature into this update's slot (the others read the starting slot)
  auto temperature_step = [&]() {
    if (t == nwg - 1) {
      float sm[2] = {sel ? v : 0.f, (tid < B && sac) ? -(lpv + a.target_entropy) : 0.f};
      float mx[1] = {-INFINITY};
      block_allreduce<2, 0>(sm, mx, red);
      if (tid == 0) {
        if (sac) st->pad_temp_grad = sm[1] / B * alpha;
        a.stats[10] = -sm[0] / kk;
        adam_scalar_step(a.adam);  // learn_step_cntr, temperature Adam, stats[11]
      }
    }
  };
  if (stats_wg) {
    // this update's critic statistics (rlmd_loss.h), off the critical path
    critic_loss_block<NT / 64>(a.cstats, reinterpret_cast<uint64_t*>(smem + ALds::runs),
                               reinterpret_cast<int*>(smem + ALds::rank), red, sidx);
    RLMD_TSA(3);
    RLMD_TSA(4);
    RLMD_TSA(15);
    return;
  }
  float* xs = reinterpret_cast<float*>(smem + ALds::xs);
  RLMD_TSA(1);
  // ---- first load round, branch-free (predicated on the workgroup's role through
  //      the range checks, as in critic_update_kernel): the row's loss inputs, the
  //      tile operands, Adam state, the fc1 block's states and first two bases
  const bool in = tid < B;
  const int64_t nB = (int64_t)B * 4;
  const int QP = a.qsplit > 1 ? 2 : 1;  // partial halves of q / dq/da / bases (qeval_rows column split)
  const bool h2nd = QP > 1;
  const __amdgpu_buffer_rsrc_t rq0 = rlmd_rsrc(a.qn[0], nB * QP), rq1 = rlmd_rsrc(a.qn[1], a.nq > 1 ? nB * QP : 0);
  const float q1r = rlmd_ldf(rq0, tid, in) + rlmd_ldf(rq0, B + tid, in && h2nd);
  const float q2r = rlmd_ldf(rq1, tid, in) + rlmd_ldf(rq1, B + tid, in && h2nd);
  lpv = rlmd_ldf(rlmd_rsrc(a.logp, sac ? nB : 0), tid, in);
  float dqda[2][kAM], sv[5][kAM];
  {
    const bool rin = in && !stats_wg;
    const __amdgpu_buffer_rsrc_t r0 = rlmd_rsrc(a.dqda[0], nB * A * QP),
                                 r1 = rlmd_rsrc(a.dqda[1], a.nq > 1 ? nB * A * QP : 0),
                                 rs = rlmd_rsrc(a.save, nB * 5 * A);
#pragma unroll
    for (int j = 0; j < kAM; ++j) {
      dqda[0][j] = rlmd_ldf(r0, (int64_t)tid * A + j, rin && j < A) +
                   rlmd_ldf(r0, (int64_t)(B + tid) * A + j, rin && h2nd && j < A);
      dqda[1][j] = rlmd_ldf(r1, (int64_t)tid * A + j, rin && j < A) +
                   rlmd_ldf(r1, (int64_t)(B + tid) * A + j, rin && h2nd && j < A);
#pragma unroll
      for (int q = 0; q < 5; ++q) sv[q][j] = rlmd_ldf(rs, (int64_t)tid * 5 * A + q * A + j, rin && j < A);
    }
  }
  constexpr int NKS = 64 / K::KS;
  uint32_t mw[NKS][2][2];
  typename K::Frag bf[NKS][2];
  float wh[2][kHM];
  int pidx[2];
  AdamIn ain[2];
  const __amdgpu_buffer_rsrc_t rm2 = rlmd_rsrc(a.am2, (int64_t)nrb * H2p * 16),
                               rh1 = rlmd_rsrc(a.hp1a, (int64_t)nrb * H1p * 16 * sizeof(typename K::T));
  const __amdgpu_buffer_rsrc_t rw = rlmd_rsrc(a.wheads, (int64_t)nh * H2 * 4);
  if constexpr (IS_W2) {
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int row = 64 * wave + s * K::KS + K::RPL * (lane >> 4);
    const bool rok = w2tile && row < nrb * 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = i0 + 16 * h + (lane & 15), j = j0 + 16 * h + (lane & 15);
      K::load_mask(rm2, rp_idx(row, H2p, i), rok && i < H2p, mw[s][h]);
      bf[s][h] = K::load_b(rh1, rp_idx(row, H1p, j), rok && j < H1p);
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = i0 + 16 * h + (lane & 15);
#pragma unroll
    for (int q = 0; q < kHM; ++q) {  // summation order
      const int hq = head_at(q, A, sac);
      wh[h][q] = rlmd_ldf(rw, (int64_t)(hq < 0 ? 0 : hq) * H2 + i, w2tile && hq >= 0 && i < H2);
    }
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int el = tid * 2 + e, blk = el >> 8, ln = (el >> 2) & 63, rg = el & 3;
    const int i = i0 + 16 * (blk >> 1) + 4 * (ln >> 4) + rg, j = j0 + 16 * (blk & 1) + (ln & 15);
    pidx[e] = (w2tile && i < H2 && j < H1) ? (int)(ao.w2 + (int64_t)i * H1 + j) : -1;
    ain[e] = adam_load(a.adam, pidx[e], polyak);
  }
  }
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr int NV = 16 * sizeof(typename K::T) / 16;  // 16-byte loads per 16 rows of h2
  u32x4 fmb[2], fhv[2][NV];
  float whc[kHM];
  int xpi = -1;
  AdamIn xin;
  float xv[8];
  constexpr int kUP = 2;  // bases prefetched per fc1-block thread (the rest load in the loop)
  f32x4 uv[kUP][kW1Q];
  const int64_t ustride = (int64_t)nrb * H1p * 16;
  const __amdgpu_buffer_rsrc_t ru = rlmd_rsrc(a.ua, ustride * nh * 4);
  // the fc1 block operands: the block's rows of s and its first kUP bases, and the
  // Adam state of W1 / b1 (thread c * 32 + jj)
  auto load_w1 = [&]() {
    const __amdgpu_buffer_rsrc_t rx = rlmd_rsrc(a.s, (int64_t)B * S * 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + q * NT, r = e >> 3, c = e & 7;
      xv[q] = rlmd_ldf(rx, (int64_t)r * S + c, w1blk && r < B && c < S);
    }
    const int j = j0 + tid % TW1, p = tid / TW1;
#pragma unroll
    for (int h = 0; h < kUP; ++h)
#pragma unroll
      for (int q = 0; q < kW1Q; ++q) {
        const int r = kW1R * p + 4 * q;
        const bool ok = w1blk && h < nh && r < nrb * 16 && j < H1p;
        uv[h][q] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(ru, ok ? (int)((h * ustride + rp_idx(r, H1p, j)) * 4) : 0x7fffffff,
                                                         0, 0));
      }
  };
  auto w1_adam = [&]() {
    const int c = tid / TW1, jr = j0 + tid % TW1;
    if (w1blk && tid < TW1 * 9 && (c < S || c == 8) && jr < H1)
      xpi = (int)(c == 8 ? ao.b1 + jr : ao.w1 + (int64_t)jr * S + c);
  };
  // an fc1 block with its own body issues them with the first load round, under
  // the loss and the ranking (the fc1 block is the actor step's last role to finish)
  constexpr bool W1_EARLY = ROLE == kRoleW1 && RLMD_W1_EARLY;
  if constexpr (W1_EARLY) {
    load_w1();
    w1_adam();
    xin = adam_load(a.adam, xpi, polyak);
  }
  {
    const float qb0 = a.qb[0][0], qb1 = a.nq > 1 ? a.qb[1][0] : 0.f;
    const float log_alpha = sac ? st->log_alpha[slot_rd(a.adam.cnt)] : 0.f;

    // ---- actor loss over all rows (algo_sac.py:546-562 / algo_td3.py:507-523)
    alpha = sac ? expf(log_alpha) : 0.f;
    const float q1 = q1r + qb0, q2 = a.nq > 1 ? q2r + qb1 : q1;
    v = sac ? fminf(q1, q2) - alpha * lpv : q1;
    kk = a.topk ? (B < a.k ? B : a.k) : B;
    sel = in;
    if (a.topk) {
      int* rank_of = reinterpret_cast<int*>(smem + ALds::rank);
      upd_rank<NT / 64>(in ? ((uint64_t)(sac ? ~f2key(v) : f2key(v)) << 32) | (uint32_t)tid : ~0ull,
                 reinterpret_cast<uint64_t*>(smem + ALds::runs), rank_of);
      sel = in && rank_of[tid] < kk;
    }
    RLMD_TSA(2);
    // without role bodies, after the ranking, to bound register use
    if constexpr (IS_W1 && !W1_EARLY) load_w1();
    // the first tile column's operands: h2 / [h2 > 0] of its column over the
    // thread's 32 rows, the heads' weights, and the Adam state of b2 / the heads'
    // rows (thread c * 32 + ci: c = 0 b2, 1..nh head c - 1) and biases (thread
    // 288 + h); on an fc1 block the Adam state of W1 / b1 (thread c * 32 + jj)
    if constexpr (IS_HEAD) {
      const int ci = tid & 31, p = tid >> 5, i = i0 + ci;
      const __amdgpu_buffer_rsrc_t rh2 = rlmd_rsrc(a.hp2a, (int64_t)nrb * H2p * 16 * sizeof(typename K::T));
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        const int r0 = 32 * p + 16 * hb;
        const bool ok = first_col && r0 < nrb * 16;
        const int64_t ix = rp_idx(r0, H2p, i);
        fmb[hb] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rm2, ok ? (int)ix : 0x7fffffff, 0, 0));
#pragma unroll
        for (int q = 0; q < NV; ++q)
          fhv[hb][q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rh2, ok ? (int)(ix * sizeof(typename K::T) + 16 * q) : 0x7fffffff,
                                                     0, 0));
      }
#pragma unroll
      for (int q = 0; q < kHM; ++q) {  // summation order
        const int hq = head_at(q, A, sac);
        whc[q] = rlmd_ldf(rw, (int64_t)(hq < 0 ? 0 : hq) * H2 + i, first_col && hq >= 0 && i < H2);
      }
    }
    {
      const int c = tid >> 5, ii = i0 + (tid & 31);
      if (first_col && tid < 32 * 9 && c <= nh && ii < H2)
        xpi = (int)(c == 0 ? ao.b2 + ii : c - 1 < A ? ao.w3 + (int64_t)(c - 1) * H2 + ii
                                                   : ao.w4 + (int64_t)(c - 1 - A) * H2 + ii);
      if (first_col && i0 == 0 && tid >= 288 && tid < 288 + nh)
        xpi = (int)(tid - 288 < A ? ao.b3 + (tid - 288) : ao.b4 + (tid - 288 - A));
      if constexpr (IS_W1 && !W1_EARLY) w1_adam();
      if constexpr ((IS_W1 && !W1_EARLY) || IS_HEAD) xin = adam_load(a.adam, xpi, polyak);
    }
    // ---- dL/da per row, then through the sampling and the heads (rlmd_policy.h)
    const float dv = sel ? -1.f / (float)kk : 0.f;
    float dq0 = dv, dq1 = 0.f, dlp = 0.f;
    if (sac) {
      const float g1 = q1 < q2 ? 1.f : (q1 > q2 ? 0.f : 0.5f);  // torch.minimum backward splits ties
      dq0 = dv * g1;
      dq1 = dv * (1.f - g1);
      dlp = -alpha * dv;
    }
    float gh[kHM];
#pragma unroll
    for (int q = 0; q < kHM; ++q) gh[q] = 0.f;
#pragma unroll
    for (int j = 0; j < kAM; ++j) {
      if (j < A && in) {
        const float da = dq0 * dqda[0][j] + dq1 * dqda[1][j];
        if (sac) {
          float dmu, dls;
          policy_comp_bwd(a.smp.dist, sv[0][j], sv[1][j], sv[2][j], sv[3][j], sv[4][j], da, dlp, a.smp.max_action,
                          a.smp.reparam_noise, a.smp.ls_min, a.smp.ls_max, dmu, dls);
          gh[j] = dmu;
          gh[A + j] = dls;
        } else {
          const float th = tanhf(sv[0][j]);
          gh[j] = da * a.smp.max_action * (1.f - th * th);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kHM; ++q) ghs[tid * kHM + q] = gh[q];
#pragma unroll
    for (int q = 0; q < kHM; ++q) {
      const int hq = head_at(q, A, sac);
      float v = 0.f;
#pragma unroll
      for (int h = 0; h < kHM; ++h) v = h == hq ? gh[h] : v;
      ghp[tid * kHM + q] = v;
    }
  }
  RLMD_TSA(3);
  temperature_step();
  RLMD_TSA(4);

  if (IS_W2 && w2tile) {
    // ---- dW2 = sum_b dh2[b, i] h1[b, j], dh2 = [h2 > 0] (sum_h gh[b, h] W_head[h, i])
    f32x4 acc[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[h][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int row = 64 * wave + s * K::KS + K::RPL * (lane >> 4);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float dh[K::RPL];
#pragma unroll
        for (int e = 0; e < K::RPL; ++e) {
          const float* gr = ghp + ((row + e) & 511) * kHM;
          float acc_h = 0.f;  // the launch-chain order (head_at); padded positions add 0 * 0
#pragma unroll
          for (int q = 0; q < kHM; ++q) acc_h = fmaf(gr[q], wh[h][q], acc_h);
          dh[e] = acc_h;
        }
        const typename K::Frag af = K::form_a(mw[s][h], dh, 1.f);
#pragma unroll
        for (int u = 0; u < 2; ++u) K::mfma(af, bf[s][u], acc[h][u]);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        *reinterpret_cast<f32x4*>(part + ((wave * 4 + h * 2 + u) * 64 + lane) * 4) = acc[h][u];
    __syncthreads();
    RLMD_TSA(5);
    float* pcl = reinterpret_cast<float*>(smem + ALds::pcl);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int el = tid * 2 + e, blk = el >> 8, ln = (el >> 2) & 63, rg = el & 3;
      const int ii = 16 * (blk >> 1) + 4 * (ln >> 4) + rg, jj = 16 * (blk & 1) + (ln & 15);
      float gs = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) gs += part[w * 1024 + el];
      float pn = 0.f, tn = 0.f;
      if (pidx[e] >= 0 && !(RLMD_ABL & 2)) adam_core(a.adam, pidx[e], gs, ain[e], polyak, pn, tn);
      pcl[ii * 33 + jj] = pn;
      pcl[32 * 33 + ii * 33 + jj] = tn;
    }
    __syncthreads();
    if (!(RLMD_ABL & 2)) tile_copies<PREC>(pcl, cd, polyak && cd.twc, i0, j0, H1p, H2p);
    RLMD_TSA(6);
  } else if (IS_HEAD && first_col) {
    {
      // ---- db2[i] = sum_b dh2[b, i]; the heads dW_head[h, i] = sum_b gh[b, h] h2[b, i]
      const int ci = tid & 31, p = tid >> 5;
      float sb = 0.f, sw[kHM];
#pragma unroll
      for (int q = 0; q < kHM; ++q) sw[q] = 0.f;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {  // the part's two 16-row blocks of column i (prefetched)
        const int r0 = 32 * p + 16 * hb;
        const u32x4& mb = fmb[hb];
        const u32x4(&hv)[NV] = fhv[hb];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float* gr = ghs + (r0 + e) * kHM;
          const uint32_t byte = (mb[e >> 2] >> (8 * (e & 3))) & 0xffu;
          float hval;
          if constexpr (PREC == RLMD_BF16) {
            const uint32_t w = hv[e >> 3][(e >> 1) & 3];
            hval = __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
          } else {
            hval = __uint_as_float(hv[e >> 2][e & 3]);
          }
          const float* grp = ghp + (r0 + e) * kHM;
          float acc_h = 0.f;
#pragma unroll
          for (int q = 0; q < kHM; ++q) acc_h = fmaf(grp[q], whc[q], acc_h);
          sb += byte ? acc_h : 0.f;
#pragma unroll
          for (int q = 0; q < kHM; ++q) sw[q] = fmaf(gr[q], hval, sw[q]);
        }
      }
      part[p * 9 * 32 + ci] = sb;
#pragma unroll
      for (int q = 0; q < kHM; ++q) part[(p * 9 + 1 + q) * 32 + ci] = sw[q];
      __syncthreads();
      if (tid < 9 * 32 && xpi >= 0) {
        const int c = tid >> 5;
        float vsum = 0.f;
        for (int q = 0; q < 16; ++q) vsum += part[(q * 9 + c) * 32 + (tid & 31)];
        step(xpi, vsum, xin);
      }
      if (i0 == 0) {  // the heads' biases: sum_b gh[b, h]
        __syncthreads();
        float sg[kHM];
#pragma unroll
        for (int q = 0; q < kHM; ++q) sg[q] = ghs[tid * kHM + q];
        float mx[1] = {-INFINITY};
        block_allreduce<kHM, 0>(sg, mx, red);
        if (tid >= 288 && tid < 288 + nh) {
          float gvb = 0.f;
#pragma unroll
          for (int q = 0; q < kHM; ++q) gvb = tid - 288 == q ? sg[q] : gvb;
          step(xpi, gvb, xin);
        }
      }
    }
  } else if (IS_W1) {
    // ---- dW1[j, x] = sum_b dh1[b, j] s[b, x], db1[j]; dh1 = sum_h gh[b, h] U_h[b, j]
    const int cj = tid % TW1, p = tid / TW1, j = j0 + cj;
#pragma unroll
    for (int q = 0; q < 8; ++q) xs[tid + q * NT] = xv[q];
    __syncthreads();
    // dh1 of the thread's kW1R rows: heads in order, the first from registers
    f32x4 du[kW1Q];
#pragma unroll
    for (int q = 0; q < kW1Q; ++q) {
      const int r = kW1R * p + 4 * q;
      du[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < kUP; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) du[q][e] = fmaf(ghs[(r + e) * kHM + h], uv[h][q][e], du[q][e]);
    }
    for (int h = kUP; h < nh; ++h) {
      f32x4 u[kW1Q];
#pragma unroll
      for (int q = 0; q < kW1Q; ++q) {
        const int r = kW1R * p + 4 * q;
        const bool ok = r < nrb * 16 && j < H1p;
        u[q] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(ru, ok ? (int)((h * ustride + rp_idx(r, H1p, j)) * 4) : 0x7fffffff,
                                                         0, 0));
      }
#pragma unroll
      for (int q = 0; q < kW1Q; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) du[q][e] = fmaf(ghs[(kW1R * p + 4 * q + e) * kHM + h], u[q][e], du[q][e]);
    }
    float acc[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) acc[c] = 0.f;
#pragma unroll 2
    for (int q = 0; q < kW1Q; ++q) {
      const int r = kW1R * p + 4 * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[8] += du[q][e];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = fmaf(du[q][e], xs[(r + e) * 8 + c], acc[c]);
      }
    }
    RLMD_TSA(5);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 9; ++c) part[(p * 9 + c) * TW1 + cj] = acc[c];
    __syncthreads();
    if (xpi >= 0) {  // TW1 rows x (S + 1) outputs, thread c * TW1 + jj (Adam state prefetched)
      const int jj = tid % TW1, c = tid / TW1;
      float vsum = 0.f;
      for (int q = 0; q < kW1G; ++q) vsum += part[(q * 9 + c) * TW1 + jj];
      step(xpi, vsum, xin);
    }
  }
  RLMD_TSA(7);
  RLMD_TSA(15);
}

}  // namespace

#ifdef RLMD_TIMING
extern "C" int rlmd_debug_ts_upd(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ts_upd), sizeof(unsigned long long) * 128) == hipSuccess ? 0 : 2;
}
extern "C" int rlmd_debug_ts_aupd(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ts_aupd), sizeof(unsigned long long) * 128) == hipSuccess ? 0 : 2;
}
#endif

size_t critic_update_lds() { return (size_t)ULds::total; }
int actor_update_n_w1(const RowDims& d) { return d.H1p / TW1; }
int critic_update_tj(const RowDims& d) { return d.B <= 256 ? (d.H1p / TW + 1) / 2 : d.H1p / TW; }

int actor_update_launch(const ActUpdArgs& a, hipStream_t st) {
  const RowDims& d = a.d;
  RLMD_CHECK(d.B <= NT && d.S <= 8 && d.A <= kAM, "actor update: B <= 512, state width <= 8, actions <= 2");
  RLMD_CHECK(a.tj == d.H1p / TW && a.ti * TW >= d.H2p && a.n_w2 == a.ti * a.tj && a.n_w1 == d.H1p / TW1 &&
                 d.H1p % TW1 == 0,
             "actor update: tile grid inconsistent with the widths");
  RLMD_CHECK(a.cstats.B <= NT, "critic statistics workgroup: mini-batch up to 512 rows");
  const dim3 grid(a.n_w2 + a.n_w1 + a.ti + (a.cstats.B > 0 ? 2 : 0));
  if (d.prec == RLMD_BF16)
    hipLaunchKernelGGL(actor_update_kernel<RLMD_BF16>, grid, dim3(NT), ALds::total, st, a);
  else
    hipLaunchKernelGGL(actor_update_kernel<RLMD_FP32>, grid, dim3(NT), ALds::total, st, a);
  RLMD_LAUNCH_CHECK();
  return 0;
}

int critic_update_launch(const CritUpdArgs& a, hipStream_t st) {
  const RowDims& d = a.d;
  RLMD_CHECK(d.B <= NT, "critic update: mini-batch up to 512 rows");
  RLMD_CHECK(d.X <= 8, "critic update: critic input width up to 8");
  const bool wide = d.B <= 256;
  RLMD_CHECK(a.tj == critic_update_tj(d) && a.ti * TW >= d.H2p && a.n_w2 == a.ti * a.tj && a.n_w1 == d.H1p / TW,
             "critic update: tile grid inconsistent with the widths");
  RLMD_CHECK(a.cstats.B <= NT, "critic statistics workgroups: mini-batch up to 512 rows");
  const dim3 grid(2 * (a.n_w2 + a.n_w1 + a.ti) + (a.cstats.B > 0 ? 2 : 0));
  const bool split = !RLMD_SPLIT_SPEC || a.loss.qsplit > 1;
#define CRIT_LAUNCH(P_, W_)                                                                                  \
  do {                                                                                                       \
    if (split) hipLaunchKernelGGL((critic_update_kernel<P_, W_, true>), grid, dim3(NT), ULds::total, st, a);  \
    else hipLaunchKernelGGL((critic_update_kernel<P_, W_, false>), grid, dim3(NT), ULds::total, st, a);      \
  } while (0)
  if (d.prec == RLMD_BF16) {
    if (wide) CRIT_LAUNCH(RLMD_BF16, true);
    else CRIT_LAUNCH(RLMD_BF16, false);
  } else {
    if (wide) CRIT_LAUNCH(RLMD_FP32, true);
    else CRIT_LAUNCH(RLMD_FP32, false);
  }
#undef CRIT_LAUNCH
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd
