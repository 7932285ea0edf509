// gemm.hip — MFMA tiles for the actor/critic MLP layers (gfx950, wave64).
//
// The reference's only dense contractions are nn.Linear forward/backward
// (algos/networks_sac.py:120-129, :357-362; algos/networks_td3.py:76-91, :152-168).
// Three layouts cover every layer of forward and backward (torch layout: weight
// W[out, in] row-major):
//   FWD    C[m, n] = act(Σ_k A[m, k] W[n, k] + b[n])                 (y = x Wᵀ + b)
//   BWD_X  C[m, c] = mask(Σ_r G[m, r] W[r, c])                       (dx = g W, ReLU mask)
//   BWD_W  C[n, c] = Σ_m G[m, n] X[m, c];  bgrad[n] = Σ_m G[m, n]     (dW = gᵀ x, db)
// Operands are staged HBM/L2 -> registers -> LDS in 64x64 tiles (range-checked
// buffer loads, next K-step prefetched into registers) and fed to
//   v_mfma_f32_16x16x4_f32   (RLMD_FP32: exact f32 fmaf chain, parity mode) or
//   v_mfma_f32_16x16x32_bf16 (RLMD_BF16: bf16 operands, f32 accumulate).
// 256 threads = 4 waves, each wave owns a 32x32 output sub-tile (2x2 MFMA
// blocks).  Up to six independent problems of different shapes (e.g. every
// weight gradient of both critics) share a launch through blockIdx.x.
#include "rlmd_common.h"
#include "rlmd_gemm.h"

namespace {

// Tile configurations (TM x TM outputs per 256-thread block, BK-deep K steps):
//   TM = 64, BK = 64  for large M (acting over all lanes): 4 waves x 32x32
//   TM = 32, BK = 128 for mini-batch GEMMs (M <= 1024): 4 waves x 16x16, a whole
//                     128-deep K chunk per load round trip, 4x more blocks
constexpr int PAD_F32 = 2;  // f32 rows of BK+2 words: 16 rows x 4 k columns spread over banks
constexpr int PAD_BF = 8;   // bf16 rows of BK+8: 16-B aligned fragment reads

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short f2bf(float f) {
  // round-to-nearest-even (finite inputs; NaN kept NaN)
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// Operand element addressing.  Loads go through buffer resources with the
// hardware range check: an element outside the operand (row >= M or k >= K)
// gets an out-of-range byte offset and reads 0, so no load is conditional and
// the compiler keeps a whole tile of loads in flight (a plain `cond ? x[i] : 0`
// is lowered to exec-masked branches that wait vmcnt(0) per pair of loads).
template <int MODE>
__device__ __forceinline__ int64_t a_off(const rlmd::GemmProblem& p, int i, int r) {
  return MODE == rlmd::GEMM_BWD_W ? (int64_t)r * p.lda + i : (int64_t)i * p.lda + r;
}
template <int MODE>
__device__ __forceinline__ int64_t b_off(const rlmd::GemmProblem& p, int r, int j) {
  return MODE == rlmd::GEMM_FWD ? (int64_t)j * p.ldb + r : (int64_t)r * p.ldb + j;
}
constexpr int kOutOfRange = 0x7fffffff;
constexpr int kSC1 = 16;  // buffer cache-policy bit: sc1 (write-through store / L2-coherent load)

__device__ __forceinline__ float buf_load(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// Epilogue for one accumulator element; bias / ReLU-mask operands are read
// through range-checked buffer loads (unconditional), only the store is guarded.
template <int MODE>
__device__ __forceinline__ float store_c(const rlmd::GemmProblem& p, const rlmd::GemmShape& s, int i,
                                         int j, float v, __amdgpu_buffer_rsrc_t rx) {
  const bool in = i < s.M && j < s.N;
  if (MODE == rlmd::GEMM_FWD) {
    if (p.bias) v += buf_load(rx, in ? j * 4 : kOutOfRange);
    if (s.relu) v = fmaxf(v, 0.f);
    if (in) p.C[(int64_t)i * p.ldc + j] = v;
    return in ? v : 0.f;
  } else if (MODE == rlmd::GEMM_BWD_X) {
    if (p.mask) {
      const float m = buf_load(rx, in ? (int)(((int64_t)i * p.ldm + j) * 4) : kOutOfRange);
      v = m > 0.f ? v : 0.f;
    }
    if (in) p.C[(int64_t)i * p.ldc + j] = v;
  } else {
    if (in) p.C[(int64_t)i * p.ldc + j] = v;
    else if (i < s.M && j == s.N && p.bias_grad) p.bias_grad[i] = v;
  }
  return 0.f;
}


// Register stage of one (A, B) tile pair: issue all global loads of a K-step.
// BWD_W operands are both [K rows][cols] with cols contiguous: each thread takes
// groups of 4 adjacent columns of one row, read as one 16-B buffer load when the
// operand's pitch, width and base allow it (4x fewer memory instructions), else
// as 4 dword loads.  FWD / BWD_X keep one element per load.
template <int MODE, int BM, int BK>
struct TileRegs {
  static constexpr int BN = BM;
  static constexpr int kPerThread = (BM * BK) / 256;  // elements of each operand tile per thread
  static constexpr int kG = BM / 4;                   // BWD_W: 4-column groups per K row
  float a[kPerThread], b[kPerThread];

  // BWD_W: 4 adjacent elements (row gr, columns gc .. gc+3) of a [K][ncols] operand
  __device__ __forceinline__ static void load4(__amdgpu_buffer_rsrc_t rs, bool vec, int ld, int ncols, int gr,
                                               int gc, bool row_ok, float* out) {
    if (vec) {
      const bool ok = row_ok && gc < ncols;  // ncols % 4 == 0: the group is all in or all out
      const f32x4 v = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (gr * ld + gc) * 4 : kOutOfRange, 0, 0));
      out[0] = v[0];
      out[1] = v[1];
      out[2] = v[2];
      out[3] = v[3];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        out[c] = buf_load(rs, (row_ok && gc + c < ncols) ? (gr * ld + gc + c) * 4 : kOutOfRange);
    }
  }

  __device__ __forceinline__ void load(const rlmd::GemmProblem& p, const rlmd::GemmShape& s,
                                       __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int i0,
                                       int j0, int r0, int r_end) {
    const int tid = threadIdx.x;
    if constexpr (MODE == rlmd::GEMM_BWD_W) {
      const bool va = (p.lda & 3) == 0 && (s.M & 3) == 0 && ((uintptr_t)p.A & 15) == 0;
      const bool vb = (p.ldb & 3) == 0 && (s.N & 3) == 0 && ((uintptr_t)p.B & 15) == 0;
#pragma unroll
      for (int e = 0; e < kPerThread / 4; ++e) {
        const int g = e * 256 + tid, c4 = (g % kG) * 4, rr = g / kG;
        const int gr = r0 + rr;
        load4(ra, va, p.lda, s.M, gr, i0 + c4, gr < r_end, &a[4 * e]);
        load4(rb, vb, p.ldb, s.N, gr, j0 + c4, gr < r_end, &b[4 * e]);
        if (p.bias_grad)  // ones column -> db
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (j0 + c4 + c == s.N && gr < r_end) b[4 * e + c] = 1.f;
      }
      return;
    }
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
      const int idx = e * 256 + tid;
      const int rr = idx % BK, ii = idx / BK;
      const int gi = i0 + ii, gr = r0 + rr;
      const bool ok = gi < s.M && gr < r_end;
      a[e] = buf_load(ra, ok ? (int)(a_off<MODE>(p, gi, gr) * 4) : kOutOfRange);
    }
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
      const int idx = e * 256 + tid;
      int jj, rr;
      if (MODE == rlmd::GEMM_FWD) {  // W[j, r]: r fastest
        rr = idx % BK;
        jj = idx / BK;
      } else {  // B[r, j]: j fastest
        jj = idx % BN;
        rr = idx / BN;
      }
      const int gj = j0 + jj, gr = r0 + rr;
      const bool ok = gj < s.N && gr < r_end;
      b[e] = buf_load(rb, ok ? (int)(b_off<MODE>(p, gr, gj) * 4) : kOutOfRange);
    }
  }

  template <typename T, int LD>
  __device__ __forceinline__ void store(T (*As)[LD], T (*Bs)[LD]) const {
    const int tid = threadIdx.x;
    if constexpr (MODE == rlmd::GEMM_BWD_W) {
#pragma unroll
      for (int e = 0; e < kPerThread / 4; ++e) {
        const int g = e * 256 + tid, c4 = (g % kG) * 4, rr = g / kG;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if constexpr (sizeof(T) == 4) {
            As[c4 + c][rr] = a[4 * e + c];
            Bs[c4 + c][rr] = b[4 * e + c];
          } else {
            As[c4 + c][rr] = f2bf(a[4 * e + c]);
            Bs[c4 + c][rr] = f2bf(b[4 * e + c]);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
      const int idx = e * 256 + tid;
      const int ii = idx / BK, rr = idx % BK;
      if constexpr (sizeof(T) == 4) As[ii][rr] = a[e];
      else As[ii][rr] = f2bf(a[e]);
    }
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
      const int idx = e * 256 + tid;
      const int jj = MODE == rlmd::GEMM_FWD ? idx / BK : idx % BN;
      const int rr = MODE == rlmd::GEMM_FWD ? idx % BK : idx / BN;
      if constexpr (sizeof(T) == 4) Bs[jj][rr] = b[e];
      else Bs[jj][rr] = f2bf(b[e]);
    }
  }
};

template <int PREC, int MODE, int BM, int BK>
__global__ void __launch_bounds__(256) gemm_kernel(rlmd::GemmBatch batch) {
  constexpr int BN = BM;
  constexpr int MB = BM / 32;  // 16x16 MFMA blocks per wave per dimension (waves are 2 x 2)
  int pi = 0;
  while (pi + 1 < batch.nprob && (int)blockIdx.x >= batch.tile_begin[pi + 1]) ++pi;
  rlmd::GemmProblem p = batch.prob[pi];
  const rlmd::GemmShape s = batch.shape[pi];
  const int tile = (int)blockIdx.x - batch.tile_begin[pi];
  const int tile_x = tile % batch.tiles_n[pi], tile_y = tile / batch.tiles_n[pi];
  // split-K (weight gradients): blockIdx.z = split `sp` reduces batch rows
  // [sp*chunk, min(K, (sp+1)*chunk)) and publishes its partial: a slab of C /
  // bias_grad (the optimiser sums the slabs in order), or with fuse_adam a
  // private write-through slab, the tile's last arriving split then summing the
  // slabs in order and stepping the parameters (rlmd_adam.h).
  const bool fused = MODE == rlmd::GEMM_BWD_W && batch.fuse_adam;
  const int chunk = (s.K + batch.splits - 1) / batch.splits;
  const int sp0 = (int)blockIdx.z, nsp = 1;
  if (!fused && sp0) {
    p.C += (int64_t)sp0 * batch.split_stride;
    if (p.bias_grad) p.bias_grad += (int64_t)sp0 * batch.split_stride;
  }
  const int i0 = tile_y * BM, j0 = tile_x * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  f32x4 acc[MB][MB], tot[MB][MB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[a][b] = tot[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K-steps per split (every split gets the same count; steps past a split's
  // end read zeros through the range check and add exact zeros)
  const int nkc = (chunk + BK - 1) / BK;
  const int nq = s.K > 0 ? nsp * nkc : 0;
  auto step_rows = [&](int q, int& r0, int& r1) {
    const int sp = sp0 + q / nkc, t = q % nkc;
    const int rb = sp * chunk;
    r0 = rb + t * BK;
    r1 = min(s.K, rb + chunk);
  };
  // operand extents in bytes (range-checked buffer resources)
  const int64_t a_rows = MODE == rlmd::GEMM_BWD_W ? s.K : s.M;
  const int64_t a_cols = MODE == rlmd::GEMM_BWD_W ? s.M : s.K;
  const int64_t b_rows = MODE == rlmd::GEMM_FWD ? s.N : s.K;
  const int64_t b_cols = MODE == rlmd::GEMM_FWD ? s.K : s.N;
  const __amdgpu_buffer_rsrc_t ra = rlmd_rsrc_wave(
      (void*)p.A, (int)(((a_rows - 1) * p.lda + a_cols) * 4));
  const __amdgpu_buffer_rsrc_t rb = rlmd_rsrc_wave(
      (void*)p.B, (int)(((b_rows - 1) * p.ldb + b_cols) * 4));
  // K-steps in flight: D register stages.  One: every split-K workgroup has a
  // single K-step at B <= 512, and a deeper ring (4: a fused tile's whole
  // reduction at once) doubles the VGPRs and halves the resident waves.
  constexpr int D = 1;
  TileRegs<MODE, BM, BK> regs[D];
#pragma unroll
  for (int u = 0; u < D; ++u)
    if (u < nq) {
      int r0, r1;
      step_rows(u, r0, r1);
      regs[u].load(p, s, ra, rb, i0, j0, r0, r1);
    }
  const int row0 = MB * 16 * wr, col0 = MB * 16 * wc;
  // fused optimiser: this thread's parameters and their state, loaded now
  int pidx[MB][MB][4];
  rlmd::AdamIn ain[MB][MB][4];
  bool polyak = false;
  if constexpr (MODE == rlmd::GEMM_BWD_W) {
    if (fused) {
      const rlmd::AdamArgs& ad = batch.adam;
      polyak = rlmd::adam_polyak(ad);
      const int offc = (int)(p.C - ad.g), offb = p.bias_grad ? (int)(p.bias_grad - ad.g) : 0;
#pragma unroll
      for (int mi = 0; mi < MB; ++mi)
#pragma unroll
        for (int ni = 0; ni < MB; ++ni)
#pragma unroll
          for (int rg = 0; rg < 4; ++rg) {
            const int i = i0 + row0 + 16 * mi + 4 * (lane >> 4) + rg;
            const int j = j0 + col0 + 16 * ni + (lane & 15);
            pidx[mi][ni][rg] = (i < s.M && j < s.N) ? offc + i * p.ldc + j
                                                    : ((i < s.M && j == s.N && p.bias_grad) ? offb + i : -1);
            ain[mi][ni][rg] = rlmd::adam_load(ad, pidx[mi][ni][rg], polyak);
          }
    }
  }
  // end of K-step q: fold the split's accumulator into the total when its last step is done
  auto close_step = [&](int q) {
    if (q % nkc != nkc - 1) return;
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        tot[a][b] = q == nkc - 1 ? acc[a][b] : tot[a][b] + acc[a][b];
        acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
  };
  if constexpr (PREC == RLMD_FP32) {
    __shared__ float As[BM][BK + PAD_F32];
    __shared__ float Bs[BN][BK + PAD_F32];
    for (int q0 = 0; q0 < nq; q0 += D)
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int q = q0 + u;
      if (q >= nq) break;
      __syncthreads();
      regs[u].store(As, Bs);
      __syncthreads();
      if (q + D < nq) {  // the stage refills D steps ahead
        int r0, r1;
        step_rows(q + D, r0, r1);
        regs[u].load(p, s, ra, rb, i0, j0, r0, r1);
      }
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        const int kr = kk + (lane >> 4);
        float av[MB], bv[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          av[m] = As[row0 + 16 * m + (lane & 15)][kr];
          bv[m] = Bs[col0 + 16 * m + (lane & 15)][kr];
        }
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
          for (int n = 0; n < MB; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[n], acc[m][n], 0, 0, 0);
      }
      close_step(q);
    }
  } else {
    __shared__ __attribute__((aligned(16))) unsigned short As[BM][BK + PAD_BF];
    __shared__ __attribute__((aligned(16))) unsigned short Bs[BN][BK + PAD_BF];
    for (int q0 = 0; q0 < nq; q0 += D)
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int q = q0 + u;
      if (q >= nq) break;
      __syncthreads();
      regs[u].store(As, Bs);
      __syncthreads();
      if (q + D < nq) {
        int r0, r1;
        step_rows(q + D, r0, r1);
        regs[u].load(p, s, ra, rb, i0, j0, r0, r1);
      }
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        const int kr = kk + 8 * (lane >> 4);
        bf16x8 av[MB], bv[MB];
#pragma unroll
        for (int m = 0; m < MB; ++m) {
          av[m] = *reinterpret_cast<const bf16x8*>(&As[row0 + 16 * m + (lane & 15)][kr]);
          bv[m] = *reinterpret_cast<const bf16x8*>(&Bs[col0 + 16 * m + (lane & 15)][kr]);
        }
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
          for (int n = 0; n < MB; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[m], bv[n], acc[m][n], 0, 0, 0);
      }
      close_step(q);
    }
  }
  if constexpr (MODE == rlmd::GEMM_BWD_W && MB == 1) {
    if (fused) {
      // publish this split's partial write-through (sc1), drain, then one lane
      // takes an arrival ticket on the tile's counter (MI355X_MICROARCH.md,
      // inter-workgroup hand-off: sc1 stores + vmcnt(0) + agent atomic; the
      // last arriver reads with sc1 loads after its add returned / a barrier)
      const int tg = (int)blockIdx.x, ns = batch.splits;
      const rlmd::AdamArgs& ad = batch.adam;
      if (ns == 1) {  // one split owns the whole reduction: step straight from the registers
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
          if (pidx[0][0][rg] >= 0) rlmd::adam_apply(ad, pidx[0][0][rg], tot[0][0][rg], ain[0][0][rg], polyak);
        if (tg == 0 && threadIdx.x == 0) rlmd::adam_scalar_step(ad);
        return;
      }
      // one uniform resource over the tile's slabs; the lane offset in voffset
      const __amdgpu_buffer_rsrc_t rsl = rlmd_rsrc_wave(
          batch.slabs + (int64_t)tg * ns * 256, ns * 256 * 16);
      const int lo = (int)threadIdx.x * 16;
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, tot[0][0]), rsl, lo + sp0 * 4096, 0, kSC1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      __shared__ int s_last;
      if (threadIdx.x == 0) {
        const unsigned prev =
            __hip_atomic_fetch_add(batch.tile_ctr + tg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev % (unsigned)ns) == (unsigned)(ns - 1);
      }
      __syncthreads();
      if (!s_last) return;
      f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int sp = 0; sp < ns; ++sp) {
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsl, lo + sp * 4096, 0, kSC1));
        g = sp == 0 ? v : g + v;  // slab order, as adam_kernel sums them
      }
#pragma unroll
      for (int rg = 0; rg < 4; ++rg)
        if (pidx[0][0][rg] >= 0) rlmd::adam_apply(ad, pidx[0][0][rg], g[rg], ain[0][0][rg], polyak);
      if (tg == 0) {
        if (threadIdx.x == 0) rlmd::adam_scalar_step(ad);
      }
      return;
    }
  }
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[a][b] = tot[a][b];
  // C/D map (16x16 MFMA, every dtype): col = lane & 15, row = 4*(lane >> 4) + reg
  __amdgpu_buffer_rsrc_t rx = ra;
  if (MODE == rlmd::GEMM_FWD && p.bias)
    rx = rlmd_rsrc_wave((void*)p.bias, s.N * 4);
  if (MODE == rlmd::GEMM_BWD_X && p.mask)
    rx = rlmd_rsrc_wave((void*)p.mask, (int)(((int64_t)(s.M - 1) * p.ldm + s.N) * 4));
  float out[MB][MB][4];
#pragma unroll
  for (int mi = 0; mi < MB; ++mi)
#pragma unroll
    for (int ni = 0; ni < MB; ++ni)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int i = i0 + row0 + 16 * mi + 4 * (lane >> 4) + rg;
        const int j = j0 + col0 + 16 * ni + (lane & 15);
        out[mi][ni][rg] = store_c<MODE>(p, s, i, j, acc[mi][ni][rg], rx);
      }
  if constexpr (MODE == rlmd::GEMM_FWD && MB == 1) {
    if (p.head_w) {  // fused q head: per-row partial over this tile's 32 columns
      __shared__ float hp[2][32];
      const int j = j0 + col0 + (lane & 15);
      const float w = buf_load(rlmd_rsrc_wave((void*)p.head_w, s.N * 4),
                               j < s.N ? j * 4 : kOutOfRange);
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const float c = rlmd_row16_sum(out[0][0][rg] * w);
        if ((lane & 15) == 0) hp[wc][row0 + 4 * (lane >> 4) + rg] = c;
      }
      __syncthreads();
      if (threadIdx.x < 32 && i0 + (int)threadIdx.x < s.M)
        p.head_part[(int64_t)tile_x * s.M + i0 + threadIdx.x] = hp[0][threadIdx.x] + hp[1][threadIdx.x];
    }
  }
}

}  // namespace

namespace rlmd {

int gemm_launch(int prec, int mode, const GemmBatch& b_in, hipStream_t stream) {
  RLMD_CHECK(b_in.nprob >= 1 && b_in.nprob <= RLMD_GEMM_MAX_PROBS, "bad GEMM problem count");
  GemmBatch b = b_in;
  if (b.splits < 1) b.splits = 1;
  RLMD_CHECK(mode == GEMM_BWD_W || b.splits == 1, "split-K only for weight gradients");
  RLMD_CHECK(mode == GEMM_BWD_W || !b.fuse_adam, "the optimiser epilogue is for weight gradients");
  bool big = false;
  for (int i = 0; i < b.nprob; ++i) big = big || b.shape[i].M > 1024;
  const int T = big ? 64 : 32;
  int tiles = 0;
  for (int i = 0; i < b.nprob; ++i) {
    RLMD_CHECK(!big || !b.prob[i].head_w, "fused head only on mini-batch GEMMs");
    const int n_out = b.shape[i].N + (mode == GEMM_BWD_W ? 1 : 0);
    const bool empty = b.shape[i].M <= 0 || n_out <= 0;
    b.tiles_n[i] = empty ? 1 : (n_out + T - 1) / T;
    b.tile_begin[i] = tiles;
    tiles += empty ? 0 : b.tiles_n[i] * ((b.shape[i].M + T - 1) / T);
  }
  b.tile_begin[b.nprob] = tiles;
  if (tiles == 0) return 0;
  RLMD_CHECK(!b.fuse_adam || (!big && b.slabs && b.tile_ctr && tiles <= b.max_tiles),
             "fused optimiser epilogue: 32x32 tiles and enough slab space");
  dim3 grid(tiles, 1, b.splits);
#define RLMD_GEMM_CASE(P, M)                                                                  \
  if (prec == P && mode == M) {                                                               \
    if (big) hipLaunchKernelGGL((gemm_kernel<P, M, 64, 64>), grid, dim3(256), 0, stream, b);  \
    else hipLaunchKernelGGL((gemm_kernel<P, M, 32, 128>), grid, dim3(256), 0, stream, b);     \
    RLMD_LAUNCH_CHECK();                                                                      \
    return 0;                                                                                 \
  }
  RLMD_GEMM_CASE(RLMD_FP32, GEMM_FWD)
  RLMD_GEMM_CASE(RLMD_FP32, GEMM_BWD_X)
  RLMD_GEMM_CASE(RLMD_FP32, GEMM_BWD_W)
  RLMD_GEMM_CASE(RLMD_BF16, GEMM_FWD)
  RLMD_GEMM_CASE(RLMD_BF16, GEMM_BWD_X)
  RLMD_GEMM_CASE(RLMD_BF16, GEMM_BWD_W)
#undef RLMD_GEMM_CASE
  RLMD_CHECK(false, "bad GEMM precision/mode");
}

}  // namespace rlmd

extern "C" {

// Test hook: one GEMM of the given mode on caller buffers (tests/test_gemm_gpu.py).
int rlmd_gemm(int32_t prec, int32_t mode, int32_t M, int32_t N, int32_t K, int32_t relu,
              const float* A, int32_t lda, const float* B, int32_t ldb, const float* bias,
              float* C, int32_t ldc, const float* mask, int32_t ldm, float* bias_grad,
              void* stream) {
  rlmd::GemmBatch b{};
  rlmd::gemm_add(b, {M, N, K, relu}, {A, lda, B, ldb, bias, C, ldc, mask, ldm, bias_grad, nullptr, nullptr});
  b.splits = 1;
  return rlmd::gemm_launch(prec, mode, b, (hipStream_t)stream);
}

}  // extern "C"
