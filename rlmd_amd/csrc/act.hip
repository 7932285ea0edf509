// act.hip — fused policy acting for all lanes (gfx950, bf16 MFMA).
//
// Replaces, batched over every lane, select_next_action / eval_next_action
// (algos/algo_sac.py:192-236, algos/algo_td3.py:198-238) = the actor forward
// (algos/networks_sac.py:101-178, :268-285; algos/networks_td3.py:76-91) +
// tanh-Gaussian sampling / TD3 exploration noise.  One launch, nothing but the
// observations in and the actions out touches HBM:
//   obs [64 rows] --VALU--> h1 = relu(obs W1^T + b1)  (bf16, LDS)
//   h1 --v_mfma_f32_16x16x32_bf16, W2 fragments straight from L2--> h2 (f32 acc)
//   relu(h2 + b2) . {pi, log_scale} / mu heads  (shuffle + LDS reductions per row)
//   mu, log-scale -> clamp -> sample -> tanh * max_action
// Block = 4 waves x 64 rows; wave w owns NB bands of 16 output columns.
// W2 is the actor's bf16 compute copy wc [H2p][H1p] (fragment-major, zero
// padded to 32, kept current by the optimiser; learn.hip refresh_copies), so
// the same kernel serves SAC 256/256 (H1p 256, NB 4) and TD3 400/300 (H1p 416,
// NB 5: 320 columns); other nets use the generic GEMM path (learn.hip: agent_act).
#include <math.h>

#include "learn_kernels.h"
#include "rlmd_common.h"
#include "rlmd_policy.h"

namespace rlmd {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 64;
constexpr int kMaxA = 2;

__device__ __forceinline__ unsigned short f2bf_rne(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

struct FusedActArgs {
  const float* obs;             // [n, S]
  const float* params;          // actor params (f32 masters)
  const unsigned short* w2bf;   // fc2.weight as the bf16 compute copy [H2p][H1p], fragment-major
  NetOff off;
  float* actions;               // [n, A]
  int32_t n, S, A, algo, mode, H1, H2;
  uint64_t seed;
  uint32_t tag, ctr;
  const float* eps_in;          // injected noise [n, A] (nullable)
  float max_action, ls_min, ls_max, noise_std;
  int32_t dist;  // SAC sampler (rlmd_policy.h)
};

template <int H1P, int NB>
__global__ void __launch_bounds__(256) fused_act_kernel(FusedActArgs a) {
  constexpr int HP = H1P + 8;  // bf16 row pitch: 16-B aligned fragment reads
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned short* h1s = reinterpret_cast<unsigned short*>(smem);                 // [64][HP]
  float* part = reinterpret_cast<float*>(smem + kRows * HP * 2);                 // [4][64][2A]
  float* w1s = part + 4 * kRows * 2 * kMaxA;                                      // [H1][S] + b1[H1]
  const int H1 = a.H1, H2 = a.H2;
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
  // layer-2 B fragments of the first K step: issued now, consumed after layer 1
  // fragment (band NB wave + nb, K-step s): 64 lanes x 16 B at ((band * H1P/32 + s) * 64 + lane) * 8
  constexpr int nS = H1P / 32;
  const bf16x8* wf = reinterpret_cast<const bf16x8*>(a.w2bf) + (int64_t)(NB * wave) * nS * 64 + lane;
  bf16x8 bnext[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) bnext[nb] = wf[nb * nS * 64];
  __syncthreads();
  // -- layer 1 on the VALU (K = S is tiny), bf16 into LDS; padded units are 0.
  //    For S <= 16 each thread keeps its unit's fc1 row in registers and sweeps
  //    rows reading the observations as LDS broadcasts.
  if (S <= 16) {
    constexpr int NR = H1P >= 256 ? 1 : 256 / H1P;  // threads per hidden unit
    constexpr int UPT = H1P >= 256 ? (H1P + 255) / 256 : 1;  // hidden units per thread
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int c = H1P >= 256 ? tid + 256 * u : tid % H1P, rg = H1P >= 256 ? 0 : tid / H1P;
      if (c < H1P) {
        const bool live = c < H1;
        float w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = live && k < S ? w1s[c * S + k] : 0.f;
        const float b = live ? w1s[H1 * S + c] : 0.f;
        for (int r = rg; r < kRows; r += NR) {
          float acc = b;
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (k < S) acc = fmaf(obs_s[r * S + k], w[k], acc);
          h1s[r * HP + c] = f2bf_rne(fmaxf(acc, 0.f));
        }
      }
    }
  } else {
    for (int e = tid; e < kRows * H1P; e += 256) {
      const int r = e / H1P, c = e % H1P;
      float acc = 0.f;
      if (c < H1) {
        acc = w1s[H1 * S + c];
        for (int k = 0; k < S; ++k) acc = fmaf(obs_s[r * S + k], w1s[c * S + k], acc);
      }
      h1s[r * HP + c] = f2bf_rne(fmaxf(acc, 0.f));
    }
  }
  __syncthreads();
  // -- layer 2: 64 rows x 16 NB columns per wave, K = H1P in steps of 32
  f32x4 acc[4][NB];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[m][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int col0 = 16 * NB * wave;
  const int kq = 8 * (lane >> 4);
#pragma unroll 2
  for (int k0 = 0; k0 < H1P; k0 += 32) {
    bf16x8 bcur[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) bcur[nb] = bnext[nb];
    if (k0 + 32 < H1P) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) bnext[nb] = wf[(nb * nS + k0 / 32 + 1) * 64];
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(&h1s[(16 * m + (lane & 15)) * HP + k0 + kq]);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bcur[nb], acc[m][nb], 0, 0, 0);
    }
  }
  // -- epilogue: relu(h2 + b2) . heads, partial per row over this wave's columns
  //    (columns past H2 have zero weights and biases)
  const int nh = a.algo == RLMD_SAC ? 2 * A : A;  // heads: pi (+ log_scale)
  float hw[NB][2 * kMaxA];
  float b2v[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int c = col0 + 16 * nb + (lane & 15);
    const bool live = c < H2;
    b2v[nb] = live ? a.params[o.b2 + c] : 0.f;
#pragma unroll
    for (int h = 0; h < 2 * kMaxA; ++h) {
      const int64_t base = h < A ? o.w3 + (int64_t)h * H2 : o.w4 + (int64_t)(h - A) * H2;
      hw[nb][h] = live && h < nh ? a.params[base + c] : 0.f;
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
      for (int nb = 0; nb < NB; ++nb) {
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

// (H1p, NB) instantiations: SAC 128|256 / 256, TD3 400 / 300
static bool fused_shape(const rlmd_agent_cfg& c, int& h1p, int& nb) {
  h1p = (c.h1 + 31) / 32 * 32;
  nb = (c.h2 + 63) / 64;
  return (h1p == 128 && nb == 4) || (h1p == 256 && nb == 4) || (h1p == 416 && nb == 5);
}

bool fused_act_supported(const rlmd_agent_cfg& c) {
  int h1p, nb;
  return c.precision == RLMD_BF16 && fused_shape(c, h1p, nb) && (c.h2 + 31) / 32 * 32 <= 16 * 4 * nb &&
         c.action_dim <= kMaxA && c.state_dim <= 64;
}

int fused_act_launch(const rlmd_agent_cfg& c, const float* obs, int64_t n, float* actions,
                     const float* actor_params, const NetOff& off, const unsigned short* w2bf, int mode,
                     uint64_t seed, uint32_t ctr, const float* eps, hipStream_t st) {
  int h1p, nb;
  RLMD_CHECK(fused_shape(c, h1p, nb), "fused acting: unsupported net shape");
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
  a.H1 = c.h1;
  a.H2 = c.h2;
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
  const size_t lds_bytes = (size_t)kRows * (h1p + 8) * 2 + 4 * kRows * 2 * kMaxA * 4 +
                           ((size_t)c.h1 * c.state_dim + c.h1 + kRows * c.state_dim) * 4;
  if (h1p == 256)
    hipLaunchKernelGGL((fused_act_kernel<256, 4>), grid, dim3(256), lds_bytes, st, a);
  else if (h1p == 128)
    hipLaunchKernelGGL((fused_act_kernel<128, 4>), grid, dim3(256), lds_bytes, st, a);
  else
    hipLaunchKernelGGL((fused_act_kernel<416, 5>), grid, dim3(256), lds_bytes, st, a);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd
