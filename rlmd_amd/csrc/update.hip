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
#include "rlmd_update.h"

namespace rlmd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
constexpr int NT = 512;
constexpr int TW = 32;  // tile edge (fc2.weight tiles TW x TW, fc1 blocks of TW rows)

__device__ __forceinline__ unsigned short bf16_rne(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
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
  __device__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static Frag load_b(__amdgpu_buffer_rsrc_t r, int64_t elem, bool ok) {
    return __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (int)(elem * 2) : 0x7fffffff, 0, 0));
  }
  // 8 mask bytes of this lane's rows
  __device__ static void load_mask(__amdgpu_buffer_rsrc_t r, int64_t byte, bool ok, uint32_t (&w)[2]) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, ok ? (int)byte : 0x7fffffff, 0, 0));
    w[0] = v[0];
    w[1] = v[1];
  }
  __device__ static Frag form_a(const uint32_t (&w)[2], const float* dq, float w3) {
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
  __device__ static void mfma(const Frag& a, const Frag& b, f32x4& c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  }
  __device__ static Frag load_b(__amdgpu_buffer_rsrc_t r, int64_t elem, bool ok) {
    return __builtin_bit_cast(Frag, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (int)(elem * 4) : 0x7fffffff, 0, 0));
  }
  __device__ static void load_mask(__amdgpu_buffer_rsrc_t r, int64_t byte, bool ok, uint32_t (&w)[2]) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, ok ? (int)byte : 0x7fffffff, 0, 0);
    w[1] = 0;
  }
  __device__ static Frag form_a(const uint32_t (&w)[2], const float* dq, float w3) {
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
  static constexpr int total = xs + 512 * 8 * 4;
};

template <int PREC>
__global__ void __launch_bounds__(NT) critic_update_kernel(CritUpdArgs a) {
  using K = KT<PREC>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* dqs = reinterpret_cast<float*>(smem + ULds::dq);
  float* part = reinterpret_cast<float*>(smem + ULds::part);
  const RowDims& d = a.d;
  const NetOff& co = a.co;
  const int per = a.n_w2 + a.n_w1;
  const int g = blockIdx.x / per, t = blockIdx.x - g * per;
  const int B = d.B, H1 = d.H1, H2 = d.H2, H1p = d.H1p, H2p = d.H2p, X = d.X;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = (B + 15) / 16;
  const bool w2tile = t < a.n_w2;
  const int i0 = w2tile ? (t / a.tj) * TW : 0, j0 = w2tile ? (t % a.tj) * TW : (t - a.n_w2) * TW;
  const bool first_col = w2tile && (t % a.tj) == 0;
  const int64_t pbase = (int64_t)g * co.size;  // this critic's parameters in the Adam base
  const bool polyak = adam_polyak(a.adam);

  // ---- first load round: loss inputs, this workgroup's operands, Adam state
  const CriticLoads cl = critic_row_load(a.loss);
  // (a) dW2 tile: per wave rows [64 w, 64 w + 64), per K-step the A masks (two i
  //     sub-blocks) and B fragments (two j sub-blocks)
  constexpr int NKS = 64 / K::KS;
  uint32_t mw[NKS][2][2];
  typename K::Frag bf[NKS][2];
  const __amdgpu_buffer_rsrc_t rm2 = rlmd_rsrc(a.m2[g], (int64_t)nrb * H2p * 16),
                               rh1 = rlmd_rsrc(a.hp1[g], (int64_t)nrb * H1p * 16 * sizeof(typename K::T));
  float w3l[2] = {0.f, 0.f};
  if (w2tile) {
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int row = 64 * wave + s * K::KS + K::RPL * (lane >> 4);
      const bool rok = row < nrb * 16;
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
      w3l[h] = rlmd_ldf(rlmd_rsrc(a.w3s[g], (int64_t)H2 * 4), i, i < H2);
    }
  }
  // (b) Adam state of the owned parameters: a dW2 tile's 1024 elements, 2 per thread
  int pidx[2];
  AdamIn ain[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    pidx[e] = -1;
    if (w2tile) {
      const int el = tid * 2 + e, blk = el >> 8, ln = (el >> 2) & 63, rg = el & 3;
      const int i = i0 + 16 * (blk >> 1) + 4 * (ln >> 4) + rg, j = j0 + 16 * (blk & 1) + (ln & 15);
      if (i < H2 && j < H1) pidx[e] = (int)(pbase + co.w2 + (int64_t)i * H1 + j);
    }
    ain[e] = adam_load(a.adam, pidx[e], polyak);
  }
  // (c) fc1 block: the critic inputs of every row into LDS
  float* xs = reinterpret_cast<float*>(smem + ULds::xs);
  if (!w2tile) {
    const __amdgpu_buffer_rsrc_t rx = rlmd_rsrc(a.x, (int64_t)B * X * 4);
    for (int e = tid; e < 512 * 8; e += NT) {
      const int r = e >> 3, c = e & 7;
      xs[e] = rlmd_ldf(rx, (int64_t)r * X + c, r < B && c < X);
    }
  }

  // ---- the loss gradient of every row (critic g): critic_row_loss, top-k by
  //      rank among all B keys (critic_loss.py:438-453)
  {
    float* red = reinterpret_cast<float*>(smem + ULds::red);
    CriticRow o;
    critic_row_loss(a.loss, red, o, cl);
    const int kk = B > a.loss.k ? a.loss.k : B;
    bool sel = o.in;
    if (B > a.loss.k) {
      int* rank_of = reinterpret_cast<int*>(smem + ULds::rank);
      block_rank(critic_sel_key(o), reinterpret_cast<uint64_t*>(smem + ULds::runs), rank_of);
      sel = o.in && rank_of[tid] < kk;
    }
    dqs[tid] = sel ? a.loss.grad_scale * (g == 0 ? o.dl[0] : o.dl[1]) / (float)kk : 0.f;
    if (blockIdx.x == 0 && tid == 0) adam_scalar_step(a.adam);  // learn_step_cntr (no temperature here)
  }
  __syncthreads();

  if (w2tile) {
    // ---- dW2[i0.., j0..] = sum_b dh2[b, i] h1[b, j] over this wave's rows
    f32x4 acc[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int v = 0; v < 2; ++v) acc[h][v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int row = 64 * wave + s * K::KS + K::RPL * (lane >> 4);
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
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int el = tid * 2 + e;
      float gs = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) gs += part[w * 1024 + el];
      if (pidx[e] >= 0) adam_apply(a.adam, pidx[e], gs, ain[e], polyak);
    }
    if (first_col) {
      // ---- db2[i] = w3[i] sum_b dq[b] [h2 > 0], dW3[i] = sum_b dq[b] h2[b, i]
      //      (thread: column i0 + tid % 32, rows [32 p, 32 p + 32) of part p = tid / 32)
      __syncthreads();  // part reused
      const int ci = tid & 31, p = tid >> 5, i = i0 + ci;
      const __amdgpu_buffer_rsrc_t rh2 = rlmd_rsrc(a.hp2[g], (int64_t)nrb * H2p * 16 * sizeof(typename K::T));
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      float sm = 0.f, sh = 0.f;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {  // the part's two 16-row blocks of column i
        const int r0 = 32 * p + 16 * hb;
        const bool ok = r0 < nrb * 16;
        const int64_t ix = rp_idx(r0, H2p, i);
        const u32x4 mb = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rm2, ok ? (int)ix : 0x7fffffff, 0, 0));
        constexpr int NV = 16 * sizeof(typename K::T) / 16;  // 16-byte loads per 16 rows of h2
        u32x4 hv[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v)
          hv[v] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rh2, ok ? (int)(ix * sizeof(typename K::T) + 16 * v) : 0x7fffffff, 0, 0));
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float q = dqs[r0 + e];
          const uint32_t byte = (mb[e >> 2] >> (8 * (e & 3))) & 0xffu;
          float h;
          if constexpr (PREC == RLMD_BF16) {
            const uint32_t w = hv[e >> 3][(e >> 1) & 3];
            h = __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
          } else {
            h = __uint_as_float(hv[e >> 2][e & 3]);
          }
          sm += byte ? q : 0.f;
          sh = fmaf(q, h, sh);
        }
      }
      part[p * 64 + ci] = sm;
      part[p * 64 + 32 + ci] = sh;
      __syncthreads();
      if (tid < 64) {
        float v = 0.f;
        for (int q = 0; q < 16; ++q) v += part[q * 64 + tid];
        const int c = i0 + (tid & 31);
        if (c < H2) {
          const int pi = (int)(pbase + (tid < 32 ? co.b2 + c : co.w3 + c));
          const float gv = tid < 32 ? v * rlmd_ldf(rlmd_rsrc(a.w3s[g], (int64_t)H2 * 4), c, true) : v;
          adam_apply(a.adam, pi, gv, adam_load(a.adam, pi, polyak), polyak);
        }
      }
      if (t == 0) {  // db3 = sum_b dq[b]
        float s3[1] = {dqs[tid]};
        float mx[1] = {-INFINITY};
        block_allreduce<1, 0>(s3, mx, reinterpret_cast<float*>(smem + ULds::red));
        if (tid == 0) {
          const int pi = (int)(pbase + co.b3);
          adam_apply(a.adam, pi, s3[0], adam_load(a.adam, pi, polyak), polyak);
        }
      }
    }
  } else {
    // ---- dW1[j, x] = sum_b dq[b] U1[b, j] x[b, x], db1[j] = sum_b dq[b] U1[b, j]
    //      (thread: fc1 row j0 + tid % 32, rows [32 p, 32 p + 32) of part p)
    const int cj = tid & 31, p = tid >> 5, j = j0 + cj;
    const __amdgpu_buffer_rsrc_t ru = rlmd_rsrc(a.u1[g], (int64_t)nrb * H1p * 16 * 4);
    f32x4 u[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = 32 * p + 4 * q;
      u[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           ru, (r < nrb * 16 && j < H1p) ? (int)(rp_idx(r, H1p, j) * 4) : 0x7fffffff,
                                           0, 0));
    }
    float acc[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) acc[c] = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 32 * p + 4 * q + e;
        const float du = dqs[r] * u[q][e];
        acc[8] += du;
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = fmaf(du, xs[r * 8 + c], acc[c]);
      }
    __syncthreads();  // xs / part
#pragma unroll
    for (int c = 0; c < 9; ++c) part[(p * 9 + c) * 32 + cj] = acc[c];
    __syncthreads();
    // 32 rows x (X + 1) outputs
    for (int o = tid; o < 32 * 9; o += NT) {
      const int jj = o % 32, c = o / 32;
      if (c < X || c == 8) {
        float v = 0.f;
        for (int q = 0; q < 16; ++q) v += part[(q * 9 + c) * 32 + jj];
        const int jr = j0 + jj;
        if (jr < H1) {
          const int pi = (int)(pbase + (c == 8 ? co.b1 + jr : co.w1 + (int64_t)jr * X + c));
          adam_apply(a.adam, pi, v, adam_load(a.adam, pi, polyak), polyak);
        }
      }
    }
  }
}

}  // namespace

size_t critic_update_lds() { return (size_t)ULds::total; }

int critic_update_launch(const CritUpdArgs& a, hipStream_t st) {
  const RowDims& d = a.d;
  RLMD_CHECK(d.B <= NT, "critic update: mini-batch up to 512 rows");
  RLMD_CHECK(d.X <= 8, "critic update: critic input width up to 8");
  RLMD_CHECK(a.tj == d.H1p / TW && a.ti * TW >= d.H2p && a.n_w2 == a.ti * a.tj && a.n_w1 == d.H1p / TW,
             "critic update: tile grid inconsistent with the widths");
  const dim3 grid(2 * (a.n_w2 + a.n_w1));
  if (d.prec == RLMD_BF16)
    hipLaunchKernelGGL(critic_update_kernel<RLMD_BF16>, grid, dim3(NT), ULds::total, st, a);
  else
    hipLaunchKernelGGL(critic_update_kernel<RLMD_FP32>, grid, dim3(NT), ULds::total, st, a);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd
