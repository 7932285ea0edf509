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

#ifdef RLMD_TIMING
// experiment builds only (tools/ts_probe.py act): per-workgroup checkpoints of
// thread 0 — [0] s_memrealtime at entry, [1..5] s_memtime after each phase,
// [6] s_memrealtime at exit; up to 4096 workgroups
__device__ unsigned long long g_ts_act[4096][8];
#define RLMD_TSA(i, v)                                                              \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_ts_act[blockIdx.x][i] = (v);       \
  } while (0)
#else
#define RLMD_TSA(i, v) \
  do {                 \
  } while (0)
#endif

// RNE f32 -> bf16, NaN kept quiet; branch-free (a select, not a divergent branch)
__device__ __forceinline__ unsigned short f2bf_rne(float f) {
  const unsigned u = __float_as_uint(f);
  const unsigned r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  return (unsigned short)((u & 0x7fffffffu) > 0x7f800000u ? ((u >> 16) | 0x40u) : r);
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

// Layer-1 LDS operands, zero padded so every MFMA operand read is unconditional:
//   w1g [SP][16][NTP]: W1[16 t + j][k] at (k * 16 + j) * NTP + t — a lane's 8
//                      tiles of one K row are 2 contiguous 16-B reads, and the
//                      pitch NTP (= 4 mod 8 dwords... 20 / 36) keeps the 16
//                      lanes of a K row on distinct bank quads;
//   b1  [H1P];
//   obs [64][SP].
template <int H1P>
struct L1Tiles {
  static constexpr int NT = H1P / 16;
  static constexpr int NTP = (NT + 7) / 8 * 8 + 4;
};

template <int H1P, int NB, int SP>
__global__ void __launch_bounds__(256) fused_act_kernel(FusedActArgs a) {
  constexpr int HP = H1P + 8;  // bf16 row pitch: 16-B aligned fragment reads
  constexpr int NT = L1Tiles<H1P>::NT, NTP = L1Tiles<H1P>::NTP;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned short* h1s = reinterpret_cast<unsigned short*>(smem);                 // [64][HP]
  float* part = reinterpret_cast<float*>(smem + kRows * HP * 2);                 // [4][64][2A]
  const int H1 = a.H1, H2 = a.H2;
  float* w1s = part + 4 * kRows * 2 * kMaxA;                                      // w1g [SP][16][NTP]
  float* b1s = w1s + SP * 16 * NTP;                                               // [H1P]
  float* obs_s = b1s + H1P;                                                       // [64][SP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * kRows;
  const NetOff& o = a.off;
  const int S = a.S, A = a.A;
  RLMD_TSA(0, __builtin_amdgcn_s_memrealtime());
  RLMD_TSA(1, __builtin_amdgcn_s_memtime());
  // epilogue operands (fc2 bias, head weights of this wave's columns; columns
  // past H2 read 0): issued first, so their latency hides under layers 1-2
  const int nh = a.algo == RLMD_SAC ? 2 * A : A;  // heads: pi (+ log_scale)
  const int col0 = 16 * NB * wave;
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
  // -- stage W1, b1 and this block's observations into the zero-padded LDS
  //    tiles (destination-indexed gathers, compile-time index math; padding
  //    reads 0 through the predicate), 8 loads per thread in flight per pass
  {
    constexpr int nW = SP * 16 * NTP + H1P, nO = kRows * SP;
    constexpr int nmax = nW > nO ? nW : nO;
    const int rows = a.n - row0 < kRows ? a.n - row0 : kRows;
    const __amdgpu_buffer_rsrc_t rw = rlmd_rsrc(a.params + o.w1, (int64_t)(H1 * S + H1) * 4);
    const __amdgpu_buffer_rsrc_t ro = rlmd_rsrc(a.obs + (int64_t)row0 * S, (int64_t)rows * S * 4);
    for (int base = 0; base < nmax; base += 8 * 256) {
      float vw[8], vo[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = base + j * 256 + tid;
        const bool isb = e >= SP * 16 * NTP;  // the b1 tail
        const int k = e / (16 * NTP), jt = e - k * (16 * NTP);
        const int jj = jt / NTP, t = jt - jj * NTP;
        const int c = isb ? e - SP * 16 * NTP : 16 * t + jj;
        const bool wl = e < nW && c < H1 && (isb || (t < NT && k < S));
        vw[j] = rlmd_ldf(rw, isb ? H1 * S + c : c * S + k, wl);
        const int r = e / SP, ko = e - r * SP;
        vo[j] = rlmd_ldf(ro, r * S + ko, e < nO && ko < S && r < rows);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = base + j * 256 + tid;
        if (e < nW) w1s[e] = vw[j];  // b1 follows w1g contiguously
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
  RLMD_TSA(2, __builtin_amdgcn_s_memtime());
  // -- layer 1 on the f32 MFMA (v_mfma_f32_16x16x4f32, K = SP in steps of 4),
  //    computed transposed (h1^T = W1 obs^T) so a lane ends with 4 consecutive
  //    units of one row: one 8-B LDS store per tile.  Wave w owns rows
  //    [16w, 16w + 16) and all H1P units in 16-wide tiles, in groups of 8 tiles
  //    whose operands arrive as 16-B LDS reads and whose MFMAs issue back to back.
  {
    typedef float f32x8 __attribute__((ext_vector_type(8)));
    const int j = lane & 15, kl = lane >> 4;
    const int ra = 16 * wave + j;
#pragma unroll
    for (int t0 = 0; t0 < NT; t0 += 8) {
      f32x4 h[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) h[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      float av[SP / 4];
      f32x8 bv[SP / 4];
#pragma unroll
      for (int ks = 0; ks < SP / 4; ++ks) {
        av[ks] = obs_s[ra * SP + 4 * ks + kl];
        bv[ks] = *reinterpret_cast<const f32x8*>(&w1s[((4 * ks + kl) * 16 + j) * NTP + t0]);
      }
      f32x4 bias[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (t0 + u < NT) bias[u] = *reinterpret_cast<const f32x4*>(&b1s[16 * (t0 + u) + 4 * kl]);
#pragma unroll
      for (int ks = 0; ks < SP / 4; ++ks)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (t0 + u < NT) h[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[ks][u], av[ks], h[u], 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (t0 + u < NT) {
          uint2 pk;
          pk.x = (uint32_t)f2bf_rne(fmaxf(h[u][0] + bias[u][0], 0.f)) |
                 ((uint32_t)f2bf_rne(fmaxf(h[u][1] + bias[u][1], 0.f)) << 16);
          pk.y = (uint32_t)f2bf_rne(fmaxf(h[u][2] + bias[u][2], 0.f)) |
                 ((uint32_t)f2bf_rne(fmaxf(h[u][3] + bias[u][3], 0.f)) << 16);
          *reinterpret_cast<uint2*>(&h1s[ra * HP + 16 * (t0 + u) + 4 * kl]) = pk;
        }
      }
    }
  }
  __syncthreads();
  RLMD_TSA(3, __builtin_amdgcn_s_memtime());
  // -- layer 2: 64 rows x 16 NB columns per wave, K = H1P in steps of 32
  f32x4 acc[4][NB];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[m][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
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
  RLMD_TSA(4, __builtin_amdgcn_s_memtime());
  // -- epilogue: relu(h2 + b2) . heads, partial per row over this wave's columns
  //    (columns past H2 have zero weights and biases)
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
      for (int h = 0; h < 2 * kMaxA; ++h)
        if (h < nh) ph[h] = rlmd_row16_sum(ph[h]);
      if ((lane & 15) == 0) {
        const int r = 16 * m + 4 * (lane >> 4) + rg;
#pragma unroll
        for (int h = 0; h < 2 * kMaxA; ++h)
          if (h < nh) part[(wave * kRows + r) * 2 * kMaxA + h] = ph[h];
      }
    }
  }
  __syncthreads();
  RLMD_TSA(5, __builtin_amdgcn_s_memtime());
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
  RLMD_TSA(6, __builtin_amdgcn_s_memrealtime());
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
         c.action_dim <= kMaxA && c.state_dim <= 16;
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
  const int sp = c.state_dim <= 8 ? 8 : 16;
  auto lds = [&](int ntp) {
    return (size_t)kRows * (h1p + 8) * 2 + 4 * kRows * 2 * kMaxA * 4 + ((size_t)sp * 16 * ntp + h1p + kRows * sp) * 4;
  };
#define ACT_LAUNCH(H1P_, NB_, SP_)                                                                  \
  hipLaunchKernelGGL((fused_act_kernel<H1P_, NB_, SP_>), grid, dim3(256), lds(L1Tiles<H1P_>::NTP), st, a)
  if (h1p == 256)
  {
    if (sp == 8) ACT_LAUNCH(256, 4, 8);
    else ACT_LAUNCH(256, 4, 16);
  }
  else if (h1p == 128)
  {
    if (sp == 8) ACT_LAUNCH(128, 4, 8);
    else ACT_LAUNCH(128, 4, 16);
  }
  else
  {
    if (sp == 8) ACT_LAUNCH(416, 5, 8);
    else ACT_LAUNCH(416, 5, 16);
  }
#undef ACT_LAUNCH
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd

#ifdef RLMD_TIMING
extern "C" int rlmd_debug_ts_act(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlmd::g_ts_act), sizeof(unsigned long long) * 8 * n) != hipSuccess;
}
#endif
