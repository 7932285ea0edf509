// act.hip — fused policy acting for all lanes (gfx950, bf16 MFMA).
//
// Replaces, batched over every lane, select_next_action / eval_next_action
// (algos/algo_sac.py:192-236, algos/algo_td3.py:198-238) = the actor forward
// (algos/networks_sac.py:101-178, :268-285; algos/networks_td3.py:76-91) +
// tanh-Gaussian sampling / TD3 exploration noise.  One launch, nothing but the
// observations in and the actions out touches HBM:
//   obs [64 rows] --VALU--> h1 = relu(obs W1^T + b1)  (bf16, LDS)
//   h1 --v_mfma_f32_16x16x32_bf16, W2 fragments straight from L2--> h2 (f32 acc)
//   relu(h2 + b2) . {pi, log_scale} heads  (shuffle + LDS reductions per row)
//   mu, log-scale -> clamp -> sample -> tanh * max_action
// Block = 4 waves x 64 rows; wave w owns output columns [64w, 64w + 64).
// Shapes: H1 % 32 == 0, H2 == 256, A <= 2 (the SAC 256/256 headline net);
// other nets use the generic GEMM path (learn.hip: agent_act).
#include <math.h>

#include "learn_kernels.h"
#include "rlmd_common.h"
#include "rlmd_policy.h"

namespace rlmd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 64;
constexpr int kH2 = 256;
constexpr int kMaxA = 2;

__device__ __forceinline__ unsigned short f2bf_rne(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

// fc2.weight [H2][H1] f32 -> bf16 in the fragment-major order (frag_index) the
// MFMA loop reads: each wave's fragment load is one contiguous KB
__global__ void w_to_bf16_kernel(const float* __restrict__ w, unsigned short* __restrict__ out, int H1, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int row = i / H1, col = i - row * H1;
    out[frag_index(row, col, H1, 1)] = f2bf_rne(w[i]);
  }
}

struct FusedActArgs {
  const float* obs;             // [n, S]
  const float* params;          // actor params (f32 masters)
  const unsigned short* w2bf;   // fc2.weight as bf16 [H2, H1]
  NetOff off;
  float* actions;               // [n, A]
  int32_t n, S, A, algo, mode;
  uint64_t seed;
  uint32_t tag, ctr;
  const float* eps_in;          // injected noise [n, A] (nullable)
  float max_action, ls_min, ls_max, noise_std;
  int32_t dist;  // SAC sampler (rlmd_policy.h)
};

template <int H1>
__global__ void __launch_bounds__(256) fused_act_kernel(FusedActArgs a) {
  constexpr int HP = H1 + 8;  // bf16 row pitch: 16-B aligned fragment reads
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned short* h1s = reinterpret_cast<unsigned short*>(smem);                 // [64][HP]
  float* part = reinterpret_cast<float*>(smem + kRows * HP * 2);                 // [4][64][2A]
  float* w1s = part + 4 * kRows * 2 * kMaxA;                                      // [H1][S] + b1[H1]
  float* obs_s = w1s + H1 * a.S + H1;                                             // [64][S]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * kRows;
  const NetOff& o = a.off;
  const int S = a.S, A = a.A;
  // -- stage W1, b1 (contiguous in torch order) and this block's observations:
  //    8 loads per thread per operand in flight before any LDS store (one round
  //    trip at these sizes); rows past n read 0 through the range check
  {
    const int nW = H1 * S + H1, nO = kRows * S;
    const int rows = a.n - row0 < kRows ? a.n - row0 : kRows;
    const __amdgpu_buffer_rsrc_t rw = rlmd_rsrc(a.params + o.w1, (int64_t)nW * 4);
    const __amdgpu_buffer_rsrc_t ro = rlmd_rsrc(a.obs + (int64_t)row0 * S, (int64_t)rows * S * 4);
    const int nmax = nW > nO ? nW : nO;
    for (int base = 0; base < nmax; base += 8 * 256) {
      float vw[8], vo[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = base + j * 256 + tid;
        vw[j] = rlmd_ldf(rw, e, e < nW);
        vo[j] = rlmd_ldf(ro, e, e < nO);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = base + j * 256 + tid;
        if (e < nW) w1s[e] = vw[j];
        if (e < nO) obs_s[e] = vo[j];
      }
    }
  }
  __syncthreads();
  // -- layer 1 on the VALU (K = S is tiny), bf16 into LDS.  For S <= 16 each
  //    thread keeps its unit's fc1 row in registers and sweeps rows reading the
  //    observations as LDS broadcasts.
  if (S <= 16) {
    constexpr int NR = 256 / H1;  // threads per hidden unit
    const int c = tid % H1, rg = tid / H1;
    float w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = k < S ? w1s[c * S + k] : 0.f;
    const float b = w1s[H1 * S + c];
    for (int r = rg; r < kRows; r += NR) {
      float acc = b;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < S) acc = fmaf(obs_s[r * S + k], w[k], acc);
      h1s[r * HP + c] = f2bf_rne(fmaxf(acc, 0.f));
    }
  } else {
    for (int e = tid; e < kRows * H1; e += 256) {
      const int r = e / H1, c = e % H1;
      float acc = w1s[H1 * S + c];
      for (int k = 0; k < S; ++k) acc = fmaf(obs_s[r * S + k], w1s[c * S + k], acc);
      h1s[r * HP + c] = f2bf_rne(fmaxf(acc, 0.f));
    }
  }
  __syncthreads();
  // -- layer 2: 64 rows x 64 columns per wave, K = H1 in steps of 32
  f32x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) acc[m][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int col0 = 64 * wave;
  const int kq = 8 * (lane >> 4);
  // fragment (band 4 wave + nb, K-step s): 64 lanes x 16 B at ((band * H1/32 + s) * 64 + lane) * 8
  constexpr int nS = H1 / 32;
  const bf16x8* wf = reinterpret_cast<const bf16x8*>(a.w2bf) + (int64_t)(4 * wave) * nS * 64 + lane;
  bf16x8 bnext[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) bnext[nb] = wf[nb * nS * 64];
#pragma unroll 2
  for (int k0 = 0; k0 < H1; k0 += 32) {
    bf16x8 bcur[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) bcur[nb] = bnext[nb];
    if (k0 + 32 < H1) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) bnext[nb] = wf[(nb * nS + k0 / 32 + 1) * 64];
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(&h1s[(16 * m + (lane & 15)) * HP + k0 + kq]);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bcur[nb], acc[m][nb], 0, 0, 0);
    }
  }
  // -- epilogue: relu(h2 + b2) . heads, partial per row over this wave's 64 columns
  const int nh = a.algo == RLMD_SAC ? 2 * A : A;  // heads: pi (+ log_scale)
  float hw[4][2 * kMaxA];
  float b2v[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int c = col0 + 16 * nb + (lane & 15);
    b2v[nb] = a.params[o.b2 + c];
#pragma unroll
    for (int h = 0; h < 2 * kMaxA; ++h) {
      const int64_t base = h < A ? o.w3 + (int64_t)h * kH2 : o.w4 + (int64_t)(h - A) * kH2;
      hw[nb][h] = h < nh ? a.params[base + c] : 0.f;
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      float ph[2 * kMaxA];
#pragma unroll
      for (int h = 0; h < 2 * kMaxA; ++h) ph[h] = 0.f;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float v = fmaxf(acc[m][nb][rg] + b2v[nb], 0.f);
#pragma unroll
        for (int h = 0; h < 2 * kMaxA; ++h) ph[h] = fmaf(v, hw[nb][h], ph[h]);
      }
#pragma unroll
      for (int h = 0; h < 2 * kMaxA; ++h) {
        float c = ph[h];
        c += __shfl_xor(c, 1, 64);
        c += __shfl_xor(c, 2, 64);
        c += __shfl_xor(c, 4, 64);
        c += __shfl_xor(c, 8, 64);
        ph[h] = c;
      }
      if ((lane & 15) == 0) {
        const int r = 16 * m + 4 * (lane >> 4) + rg;
#pragma unroll
        for (int h = 0; h < 2 * kMaxA; ++h) part[(wave * kRows + r) * 2 * kMaxA + h] = ph[h];
      }
    }
  }
  __syncthreads();
  // -- per row: sum the 4 wave partials, sample, write the action
  if (tid < kRows && row0 + tid < a.n) {
    const int r = tid, b = row0 + tid;
    for (int j = 0; j < A; ++j) {
      float mu = a.params[o.b3 + j], ls_raw = 0.f;
      for (int w = 0; w < 4; ++w) mu += part[(w * kRows + r) * 2 * kMaxA + j];
      if (a.algo == RLMD_SAC) {
        ls_raw = a.params[o.b4 + j];
        for (int w = 0; w < 4; ++w) ls_raw += part[(w * kRows + r) * 2 * kMaxA + A + j];
      }
      float noise = 0.f;
      if (a.mode == 0)
        noise = a.eps_in ? a.eps_in[(int64_t)b * A + j]
                         : policy_draw(a.algo == RLMD_SAC ? a.dist : RLMD_DIST_N, a.seed, (uint32_t)b, a.ctr, a.tag, j);
      float act;
      if (a.algo == RLMD_SAC) {
        const PolicyComp pc = policy_comp(a.dist, mu, ls_raw, noise, a.ls_min, a.ls_max);
        act = tanhf(a.mode == 1 ? pc.mu : pc.u) * a.max_action;
      } else {
        act = tanhf(mu) * a.max_action;
        if (a.mode == 0) act = fminf(fmaxf(act + noise * a.noise_std, -a.max_action), a.max_action);
      }
      a.actions[(int64_t)b * A + j] = act;
    }
  }
}

}  // namespace

bool fused_act_supported(const rlmd_agent_cfg& c) {
  return c.precision == RLMD_BF16 && c.h2 == kH2 && (c.h1 == 256 || c.h1 == 128) &&
         c.action_dim <= kMaxA && c.state_dim <= 64;
}

int fused_act_launch(const rlmd_agent_cfg& c, const float* obs, int64_t n, float* actions,
                     const float* actor_params, const NetOff& off, unsigned short* w2bf, int mode,
                     uint64_t seed, uint32_t ctr, const float* eps, hipStream_t st) {
  const int nw2 = c.h2 * c.h1;
  hipLaunchKernelGGL(w_to_bf16_kernel, dim3((nw2 + 255) / 256), dim3(256), 0, st, actor_params + off.w2,
                     w2bf, c.h1, nw2);
  RLMD_LAUNCH_CHECK();
  FusedActArgs a{};
  a.obs = obs;
  a.params = actor_params;
  a.w2bf = w2bf;
  a.off = off;
  a.actions = actions;
  a.n = (int32_t)n;
  a.S = c.state_dim;
  a.A = c.action_dim;
  a.algo = c.algo;
  a.mode = mode;
  a.seed = seed;
  a.tag = RLMD_TAG_ACT_NOISE;
  a.ctr = ctr;
  a.eps_in = eps;
  a.max_action = c.max_action;
  a.ls_min = c.log_scale_min;
  a.ls_max = c.log_scale_max;
  a.noise_std = c.policy_noise;
  a.dist = c.policy_dist;
  const dim3 grid((unsigned)((n + kRows - 1) / kRows));
  const size_t lds_bytes = (size_t)kRows * (c.h1 + 8) * 2 + 4 * kRows * 2 * kMaxA * 4 +
                           ((size_t)c.h1 * c.state_dim + c.h1 + kRows * c.state_dim) * 4;
  if (c.h1 == 256)
    hipLaunchKernelGGL(fused_act_kernel<256>, grid, dim3(256), lds_bytes, st, a);
  else
    hipLaunchKernelGGL(fused_act_kernel<128>, grid, dim3(256), lds_bytes, st, a);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd
