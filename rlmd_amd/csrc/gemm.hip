// gemm.hip — MFMA tiles for the actor/critic MLP layers (gfx950, wave64).
//
// The reference's only dense contractions are nn.Linear forward/backward
// (algos/networks_sac.py:120-129, :357-362; algos/networks_td3.py:76-91, :152-168).
// Three layouts cover every layer of forward and backward (torch layout: weight
// W[out, in] row-major):
//   FWD    C[m, n] = act(Σ_k A[m, k] W[n, k] + b[n])                 (y = x Wᵀ + b)
//   BWD_X  C[m, c] = mask(Σ_r G[m, r] W[r, c])                       (dx = g W, ReLU mask)
//   BWD_W  C[n, c] = Σ_m G[m, n] X[m, c];  bgrad[n] = Σ_m G[m, n]     (dW = gᵀ x, db)
// Operands are staged HBM/L2 -> LDS in 64x32 tiles and fed to
//   v_mfma_f32_16x16x4_f32   (RLMD_FP32: exact f32 fmaf chain, parity mode) or
//   v_mfma_f32_16x16x32_bf16 (RLMD_BF16: bf16 operands, f32 accumulate).
// 256 threads = 4 waves, each wave owns a 32x32 output sub-tile (2x2 MFMA
// blocks).  Up to two independent problems (the twin critics) share a launch
// through gridDim.z.
#include "rlmd_common.h"
#include "rlmd_gemm.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int PAD_F32 = 2;  // row stride 34 words: conflict-free column reads by 16 rows x 2 k
constexpr int PAD_BF = 8;   // row stride 80 B: 16-B aligned fragment reads

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short f2bf(float f) {
  // round-to-nearest-even (finite inputs; NaN kept NaN)
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

template <int MODE>
__device__ __forceinline__ float load_a(const rlmd::GemmProblem& p, const rlmd::GemmShape& s,
                                        int i, int r) {
  if (i >= s.M || r >= s.K) return 0.f;
  if (MODE == rlmd::GEMM_BWD_W) return p.A[(int64_t)r * p.lda + i];
  return p.A[(int64_t)i * p.lda + r];
}

template <int MODE>
__device__ __forceinline__ float load_b(const rlmd::GemmProblem& p, const rlmd::GemmShape& s,
                                        int r, int j) {
  if (r >= s.K) return 0.f;
  if (MODE == rlmd::GEMM_BWD_W) {
    if (j < s.N) return p.B[(int64_t)r * p.ldb + j];
    return (j == s.N && p.bias_grad) ? 1.f : 0.f;  // ones column -> bias gradient
  }
  if (j >= s.N) return 0.f;
  if (MODE == rlmd::GEMM_FWD) return p.B[(int64_t)j * p.ldb + r];
  return p.B[(int64_t)r * p.ldb + j];
}

template <int MODE>
__device__ __forceinline__ void store_c(const rlmd::GemmProblem& p, const rlmd::GemmShape& s, int i,
                                        int j, float v) {
  if (i >= s.M) return;
  if (MODE == rlmd::GEMM_FWD) {
    if (j >= s.N) return;
    if (p.bias) v += p.bias[j];
    if (s.relu) v = fmaxf(v, 0.f);
    p.C[(int64_t)i * p.ldc + j] = v;
  } else if (MODE == rlmd::GEMM_BWD_X) {
    if (j >= s.N) return;
    if (p.mask && !(p.mask[(int64_t)i * p.ldm + j] > 0.f)) v = 0.f;
    p.C[(int64_t)i * p.ldc + j] = v;
  } else {
    if (j < s.N) p.C[(int64_t)i * p.ldc + j] = v;
    else if (j == s.N && p.bias_grad) p.bias_grad[i] = v;
  }
}

// Global -> LDS staging of one BMxBK A tile and one BNxBK B tile (both stored
// r-contiguous).  Loop order follows the contiguous global dimension so each
// wave-instruction reads consecutive addresses.
template <int MODE, typename T, int LD>
__device__ __forceinline__ void stage(const rlmd::GemmProblem& p, const rlmd::GemmShape& s, int i0,
                                      int j0, int r0, T (*As)[LD], T (*Bs)[LD]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < (BM * BK) / 256; ++e) {
    const int idx = e * 256 + tid;
    int ii, rr;
    if (MODE == rlmd::GEMM_BWD_W) {  // A element (i, r) at A[r*lda + i]: i fastest
      ii = idx % BM;
      rr = idx / BM;
    } else {
      rr = idx % BK;
      ii = idx / BK;
    }
    const float v = load_a<MODE>(p, s, i0 + ii, r0 + rr);
    if constexpr (sizeof(T) == 4) As[ii][rr] = v;
    else As[ii][rr] = f2bf(v);
  }
#pragma unroll
  for (int e = 0; e < (BN * BK) / 256; ++e) {
    const int idx = e * 256 + tid;
    int jj, rr;
    if (MODE == rlmd::GEMM_FWD) {  // W[j, r]: r fastest
      rr = idx % BK;
      jj = idx / BK;
    } else {  // B[r, j]: j fastest
      jj = idx % BN;
      rr = idx / BN;
    }
    const float v = load_b<MODE>(p, s, r0 + rr, j0 + jj);
    if constexpr (sizeof(T) == 4) Bs[jj][rr] = v;
    else Bs[jj][rr] = f2bf(v);
  }
}

template <int PREC, int MODE>
__global__ void __launch_bounds__(256) gemm_kernel(rlmd::GemmBatch batch) {
  const rlmd::GemmProblem& p = batch.prob[blockIdx.z];
  const rlmd::GemmShape& s = batch.shape;
  const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int Kr = s.K;
  if constexpr (PREC == RLMD_FP32) {
    __shared__ float As[BM][BK + PAD_F32];
    __shared__ float Bs[BN][BK + PAD_F32];
    for (int r0 = 0; r0 < Kr; r0 += BK) {
      __syncthreads();
      stage<MODE, float, BK + PAD_F32>(p, s, i0, j0, r0, As, Bs);
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < BK; kk += 4) {
        const int kr = kk + (lane >> 4);
        float a0 = As[32 * wr + (lane & 15)][kr];
        float a1 = As[32 * wr + 16 + (lane & 15)][kr];
        float b0 = Bs[32 * wc + (lane & 15)][kr];
        float b1 = Bs[32 * wc + 16 + (lane & 15)][kr];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
  } else {
    __shared__ __attribute__((aligned(16))) unsigned short As[BM][BK + PAD_BF];
    __shared__ __attribute__((aligned(16))) unsigned short Bs[BN][BK + PAD_BF];
    for (int r0 = 0; r0 < Kr; r0 += BK) {
      __syncthreads();
      stage<MODE, unsigned short, BK + PAD_BF>(p, s, i0, j0, r0, As, Bs);
      __syncthreads();
      const int kr = 8 * (lane >> 4);
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&As[32 * wr + (lane & 15)][kr]);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&As[32 * wr + 16 + (lane & 15)][kr]);
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&Bs[32 * wc + (lane & 15)][kr]);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&Bs[32 * wc + 16 + (lane & 15)][kr]);
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // C/D map (16x16 MFMA, every dtype): col = lane & 15, row = 4*(lane >> 4) + reg
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int i = i0 + 32 * wr + 16 * mi + 4 * (lane >> 4) + rg;
        const int j = j0 + 32 * wc + 16 * ni + (lane & 15);
        store_c<MODE>(p, s, i, j, acc[mi][ni][rg]);
      }
}

}  // namespace

namespace rlmd {

int gemm_launch(int prec, int mode, const GemmBatch& b, int groups, hipStream_t stream) {
  RLMD_CHECK(groups >= 1 && groups <= RLMD_GEMM_MAX_GROUPS, "bad GEMM group count");
  const int n_out = b.shape.N + (mode == GEMM_BWD_W ? 1 : 0);
  if (b.shape.M <= 0 || n_out <= 0) return 0;
  dim3 grid((n_out + BN - 1) / BN, (b.shape.M + BM - 1) / BM, groups);
#define RLMD_GEMM_CASE(P, M)                                                          \
  if (prec == P && mode == M) {                                                       \
    hipLaunchKernelGGL((gemm_kernel<P, M>), grid, dim3(256), 0, stream, b);          \
    RLMD_LAUNCH_CHECK();                                                              \
    return 0;                                                                         \
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
  b.shape = {M, N, K, relu};
  b.prob[0] = {A, lda, B, ldb, bias, C, ldc, mask, ldm, bias_grad};
  return rlmd::gemm_launch(prec, mode, b, 1, (hipStream_t)stream);
}

}  // extern "C"
