// rlmd_act_rows.h — the fused acting body (policy forward + sampling for a
// 64-row block), shared by act.hip's fused_act_kernel and env.hip's fused
// acting + env-step kernel.  See act.hip for the design.
//
// Replaces, batched over every lane, select_next_action / eval_next_action
// (algos/algo_sac.py:192-236, algos/algo_td3.py:198-238).
#pragma once
#include <math.h>

#include "learn_kernels.h"
#include "rlmd_common.h"
#include "rlmd_policy.h"

#ifndef RLMD_TSA
#define RLMD_TSA(i, v) \
  do {                 \
  } while (0)
#endif

namespace rlmd {
namespace actrows {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kRows = 64;

constexpr int kMaxA = 2;   // the headline shapes (one gamble / asset: investors A / B, Dice_SH A)
constexpr int kMaxA4 = 4;  // the wide-action instantiation (investors C, Dice_SH B / C)

// Workgroups per CU the 256-wide, two-action acting kernels are compiled for (the
// WPC template argument: launch bounds).  At 3 they hold 140 VGPRs without
// spills; at 4 (what their LDS allows, act_lds) they fit 128 VGPRs with 8-22
// dwords spilled.  4 pays only when 3 per CU would leave a second dispatch round:
// C2's 1,024 blocks (act_env 34.0 -> 32.4 us), not C4's 128 (19.6 -> 20.8 us).
inline int act_wpc(int h1p, int ma, int64_t blocks) {
  if (h1p != 256 || ma != kMaxA) return 3;
  static int ncu[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 3;
  if (ncu[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 3;
    ncu[dev] = n;
  }
  static const int forced = [] {
    const char* e = getenv("RLMD_ACT_WPC");  // 3 / 4: A/B runs
    return e ? atoi(e) : 0;
  }();
  if (forced == 3 || forced == 4) return forced;
  return blocks > 3LL * ncu[dev] ? 4 : 3;
}


// RNE f32 -> bf16, NaN kept quiet; branch-free (a select, not a divergent branch)
__device__ __forceinline__ unsigned short f2bf_rne(float f) {
  const unsigned u = __float_as_uint(f);
  const unsigned r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
  return (unsigned short)((u & 0x7fffffffu) > 0x7f800000u ? ((u >> 16) | 0x40u) : r);
}


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

// Dynamic LDS of the acting body (byte offsets).  h1 [64][HP] bf16 comes first.
// Up to H1P = 256 the layer-1 tiles w1g and the head partials live inside h1's
// bytes (alias): every wave takes its W1 operands into registers before any
// wave writes h1, and a barrier after layer 2 precedes the partials.  That puts
// a 256-wide block at 36 KB, four workgroups per CU (1,024 blocks of 65,536
// lanes in one round instead of 768 + 256); wider nets keep separate regions.
struct ActLds {
  int h1, part, w1, b1, obs, samp, total;
  bool alias;
};
// park: the parked instantiations (4 workgroups per CU, act_park) also hold the
// sampling rows' head biases and noise in LDS
__host__ __device__ constexpr ActLds act_lds(int h1p, int sp, int ma, bool park = false) {
  const int nt = h1p / 16, ntp = (nt + 7) / 8 * 8 + 4;
  const int h1b = kRows * (h1p + 8) * 2, partb = 4 * kRows * 2 * ma * 4, w1b = sp * 16 * ntp * 4;
  const bool al = h1p <= 256;
  ActLds l{};
  l.alias = al;
  l.h1 = 0;
  l.part = al ? 0 : h1b;
  l.w1 = al ? 0 : h1b + partb;
  l.b1 = al ? h1b : l.w1 + w1b;
  l.obs = l.b1 + h1p * 4;
  l.samp = l.obs + kRows * sp * 4;  // the sampling rows' head biases and noise [3][ma][64] (parked)
  l.total = l.samp + (park ? 3 * ma * kRows * 4 : 0);
  return l;
}

// The acting body for one 64-row block.  pro() runs once every thread has issued
// its epilogue loads (a fused caller issues its own per-row loads there); epi(r,
// b, act, obs_row) runs on thread r < 64 of each valid row b with the row's
// actions act[MA] (f32; MA = kMaxA, or kMaxA4 for 3-4 actions: twice the head
// registers and partials) and its observation in LDS (obs_row[0 .. S)).
struct NoPark {
  __device__ void operator()() const {}
};
// park() runs once this thread's staging loads have landed (after their LDS
// stores, before the barrier): a fused caller moves the per-row values its pro()
// loaded into LDS there (kParkBytes past act_lds().total), so that they are not
// held in registers across the body — at 4 workgroups per CU (128 VGPRs) they
// were spilled to scratch, each spill store waiting for its load on the spot
constexpr int kParkWords = 8;
constexpr int kParkBytes = kRows * kParkWords * 4;
// PARK: the 4-workgroups-per-CU instantiations (128 VGPRs), whose values held
// across the body were spilled; act_park(H1P, SP, MA, WPC)
__host__ __device__ constexpr bool act_park(int h1p, int sp, int ma, int wpc) {
  return h1p == 256 && sp == 8 && ma == kMaxA && wpc == 4;  // act_lds + kParkBytes fit 40 KB
}
template <int H1P, int NB, int SP, int MA, bool PARK, typename ProF, typename EpiF, typename ParkF = NoPark>
__device__ __forceinline__ void act_rows(const FusedActArgs& a, unsigned char* smem, ProF pro, EpiF epi,
                                         ParkF park = ParkF()) {
  constexpr int kMaxA = MA;
  constexpr int HP = H1P + 8;  // bf16 row pitch: 16-B aligned fragment reads
  constexpr int NT = L1Tiles<H1P>::NT, NTP = L1Tiles<H1P>::NTP;
  constexpr ActLds LY = act_lds(H1P, SP, MA, PARK);
  unsigned short* h1s = reinterpret_cast<unsigned short*>(smem + LY.h1);  // [64][HP]
  float* part = reinterpret_cast<float*>(smem + LY.part);                 // [4][64][2A]
  const int H1 = a.H1, H2 = a.H2;
  float* w1s = reinterpret_cast<float*>(smem + LY.w1);                    // w1g [SP][16][NTP]
  float* b1s = reinterpret_cast<float*>(smem + LY.b1);                    // [H1P]
  float* obs_s = reinterpret_cast<float*>(smem + LY.obs);                 // [64][SP]
  float* samp_s = reinterpret_cast<float*>(smem + LY.samp);               // [3][MA][64]
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
  // every load of this round through a range-checked buffer resource (an
  // excluded element reads 0): no load sits in a branch, whose merge would wait
  // for it (four such waits had serialised this prologue's load round)
  const __amdgpu_buffer_rsrc_t rp = rlmd_rsrc(a.params, 0x7fffffff);
  float hw[NB][2 * kMaxA];
  float b2v[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int c = col0 + 16 * nb + (lane & 15);
    const bool live = c < H2;
    b2v[nb] = rlmd_ldf(rp, o.b2 + c, live);
#pragma unroll
    for (int h = 0; h < 2 * kMaxA; ++h) {
      const int64_t base = h < A ? o.w3 + (int64_t)h * H2 : o.w4 + (int64_t)(h - A) * H2;
      hw[nb][h] = rlmd_ldf(rp, base + c, live && h < nh);
    }
  }
  // the sampling threads' head biases and policy noise (Philox -> f64 Box-Muller):
  // independent of the forward pass, so drawn here, under the load latency, not
  // in the epilogue's tail
  float mu_b[kMaxA], ls_b[kMaxA], nz[kMaxA];
  const __amdgpu_buffer_rsrc_t re = rlmd_rsrc(a.eps_in, a.eps_in ? (int64_t)a.n * A * 4 : 0);
#pragma unroll
  for (int j = 0; j < kMaxA; ++j) {
    const bool mine = tid < kRows && row0 + tid < a.n && j < A;
    mu_b[j] = rlmd_ldf(rp, o.b3 + j, mine);
    ls_b[j] = rlmd_ldf(rp, o.b4 + j, mine && a.algo == RLMD_SAC);
    const float ein = rlmd_ldf(re, (int64_t)(row0 + tid) * A + j, mine && a.mode == 0);
    // drawn by every thread and selected: a draw in a branch overwrote the
    // register the speculatively issued eps load targets, which waited on it
    const float drawn = policy_draw(a.algo == RLMD_SAC ? a.dist : RLMD_DIST_N, a.seed, (uint32_t)(row0 + tid), a.ctr,
                                    a.tag, j);
    nz[j] = mine && a.mode == 0 ? (a.eps_in ? ein : drawn) : 0.f;
  }
  pro();
  // -- stage W1, b1 and this block's observations into the zero-padded LDS
  //    tiles (destination-indexed gathers, compile-time index math; padding
  //    reads 0 through the predicate): every thread's loads in one round, all
  //    issued before its first LDS store
  {
    constexpr int nW = SP * 16 * NTP + H1P, nO = kRows * SP;
    constexpr int PW = (nW + 255) / 256, PO = (nO + 255) / 256;
    const int rows = a.n - row0 < kRows ? a.n - row0 : kRows;
    const __amdgpu_buffer_rsrc_t rw = rlmd_rsrc(a.params + o.w1, (int64_t)(H1 * S + H1) * 4);
    const __amdgpu_buffer_rsrc_t ro = rlmd_rsrc(a.obs + (int64_t)row0 * S, (int64_t)rows * S * 4);
    float vw[PW], vo[PO];
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int e = j * 256 + tid;
      const bool isb = e >= SP * 16 * NTP;  // the b1 tail
      const int k = e / (16 * NTP), jt = e - k * (16 * NTP);
      const int jj = jt / NTP, t = jt - jj * NTP;
      const int c = isb ? e - SP * 16 * NTP : 16 * t + jj;
      const bool wl = e < nW && c < H1 && (isb || (t < NT && k < S));
      vw[j] = rlmd_ldf(rw, isb ? H1 * S + c : c * S + k, wl);
    }
#pragma unroll
    for (int j = 0; j < PO; ++j) {
      const int e = j * 256 + tid;
      const int r = e / SP, ko = e - r * SP;
      vo[j] = rlmd_ldf(ro, r * S + ko, e < nO && ko < S && r < rows);
    }
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int e = j * 256 + tid;
      constexpr int nG = SP * 16 * NTP;
      if (e < nW) (e < nG ? w1s[e] : b1s[e - nG]) = vw[j];
    }
#pragma unroll
    for (int j = 0; j < PO; ++j) {
      const int e = j * 256 + tid;
      if (e < nO) obs_s[e] = vo[j];
    }
    // the sampling threads' head biases and noise to LDS, read back at sampling
    // time: held in registers across the body they were spilled (see park())
    if (PARK && tid < kRows) {
#pragma unroll
      for (int j = 0; j < kMaxA; ++j) {
        samp_s[(0 * kMaxA + j) * kRows + tid] = mu_b[j];
        samp_s[(1 * kMaxA + j) * kRows + tid] = ls_b[j];
        samp_s[(2 * kMaxA + j) * kRows + tid] = nz[j];
      }
    }
    park();
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
    // aliased layout: every group's W1 operands into registers, then a barrier,
    // before this wave's first h1 store can overwrite w1g
    constexpr int NG = LY.alias ? (NT + 7) / 8 : 1;
    f32x8 bvg[NG][SP / 4];
    if constexpr (LY.alias) {
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int ks = 0; ks < SP / 4; ++ks)
          bvg[g][ks] = *reinterpret_cast<const f32x8*>(&w1s[((4 * ks + kl) * 16 + j) * NTP + 8 * g]);
      __syncthreads();
    }
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
        if constexpr (LY.alias)
          bv[ks] = bvg[t0 / 8][ks];
        else
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
#if !defined(RLMD_ABL_ACT)
    if (k0 + 32 < H1P) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) bnext[nb] = wf[(nb * nS + k0 / 32 + 1) * 64];
    }
#endif  // timing ablation (experiment builds only; results wrong): layer 2 without its fragment stream
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(&h1s[(16 * m + (lane & 15)) * HP + k0 + kq]);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bcur[nb], acc[m][nb], 0, 0, 0);
    }
  }
  RLMD_TSA(4, __builtin_amdgcn_s_memtime());
  if constexpr (LY.alias) __syncthreads();  // the partials overwrite h1
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
  // -- per row: sum the 4 wave partials, sample, write the action.  The row
  //    index and the algorithm flag are formed here from opaque scalar copies:
  //    at 128 VGPRs the compiler had kept them in VGPRs from the prologue and
  //    spilled them (a scratch reload and its wait at sampling time)
  int row0_l = row0, algo_l = a.algo;
  if constexpr (PARK) {
    asm volatile("s_mov_b32 %0, %1" : "=s"(row0_l) : "s"(row0));
    asm volatile("s_mov_b32 %0, %1" : "=s"(algo_l) : "s"(a.algo));
  }
  if (tid < kRows && row0_l + tid < a.n) {
    const int r = tid, b = row0_l + tid;
    float acts[kMaxA];
#pragma unroll
    for (int j = 0; j < kMaxA; ++j) acts[j] = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxA; ++j) {
      if (j >= A) break;
      float mu = PARK ? samp_s[(0 * kMaxA + j) * kRows + r] : mu_b[j], ls_raw = 0.f;
      for (int w = 0; w < 4; ++w) mu += part[(w * kRows + r) * 2 * kMaxA + j];
      if (algo_l == RLMD_SAC) {
        ls_raw = PARK ? samp_s[(1 * kMaxA + j) * kRows + r] : ls_b[j];
        for (int w = 0; w < 4; ++w) ls_raw += part[(w * kRows + r) * 2 * kMaxA + A + j];
      }
      const float noise = PARK ? samp_s[(2 * kMaxA + j) * kRows + r] : nz[j];
      float act;
      if (algo_l == RLMD_SAC) {
        const PolicyComp pc = policy_comp(a.dist, mu, ls_raw, noise, a.ls_min, a.ls_max);
        act = tanhf(a.mode == 1 ? pc.mu : pc.u) * a.max_action;
      } else {
        act = tanhf(mu) * a.max_action;
        if (a.mode == 0) act = fminf(fmaxf(act + noise * a.noise_std, -a.max_action), a.max_action);
      }
      acts[j] = act;
    }
    epi(r, b, acts, obs_s + r * SP);
  }
  RLMD_TSA(6, __builtin_amdgcn_s_memrealtime());
}


// (H1p, NB) of a net: SAC 128|256 / 256, TD3 400 / 300
inline bool fused_shape(const rlmd_agent_cfg& c, int& h1p, int& nb) {
  h1p = (c.h1 + 31) / 32 * 32;
  nb = (c.h2 + 63) / 64;
  return (h1p == 128 && nb == 4) || (h1p == 256 && nb == 4) || (h1p == 416 && nb == 5);
}

// dynamic LDS of act_rows<h1p, *, sp, ma>
inline size_t act_lds_bytes(int h1p, int sp, int ma = kMaxA, bool park = false) {
  return (size_t)act_lds(h1p, sp, ma, park).total;
}

// the acting body's action bound for an action count
inline int act_ma(int action_dim) { return action_dim <= kMaxA ? kMaxA : kMaxA4; }

}  // namespace actrows
}  // namespace rlmd
