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
// FP contraction is off, as in env.hip, whose act_env_kernel runs the same
// acting body: the two-launch and the fused steady state are bit-equal
// (tests/test_fused_env_gpu.py).
#pragma clang fp contract(off)
#include <math.h>
#include <hip/hip_ext.h>

#ifdef RLMD_TIMING
namespace rlmd {
namespace actrows {
// experiment builds only (tools/ts_probe.py act): per-workgroup checkpoints of
// thread 0 — [0] s_memrealtime at entry, [1..5] s_memtime after each phase,
// [6] s_memrealtime at exit; up to 4096 workgroups
__device__ unsigned long long g_ts_act[4096][8];
}  // namespace actrows
}  // namespace rlmd
#define RLMD_TSA(i, v)                                                                          \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < 4096) ::rlmd::actrows::g_ts_act[blockIdx.x][i] = (v);  \
  } while (0)
#endif

#include "rlmd_act_rows.h"

namespace rlmd {
namespace {
using namespace actrows;

template <int H1P, int NB, int SP, int MA, int WPC>
__global__ void __launch_bounds__(256, H1P == 256 ? (MA == kMaxA ? WPC : 2) : 1) fused_act_kernel(FusedActArgs a) {
  RLMD_KERNARG_PREFETCH(a);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  act_rows<H1P, NB, SP, MA, act_park(H1P, SP, MA, WPC)>(
      a, smem, [] {},
      [&](int, int b, const float* acts, const float*) {
        for (int j = 0; j < a.A; ++j) a.actions[(int64_t)b * a.A + j] = acts[j];
      });
}

}  // namespace

bool fused_act_supported(const rlmd_agent_cfg& c) {
  int h1p, nb;
  return c.precision == RLMD_BF16 && fused_shape(c, h1p, nb) && (c.h2 + 31) / 32 * 32 <= 16 * 4 * nb &&
         c.action_dim <= kMaxA4 && c.state_dim <= 16;
}

FusedActArgs fused_act_args(const rlmd_agent_cfg& c, const float* obs, int64_t n, float* actions,
                            const float* actor_params, const NetOff& off, const unsigned short* w2bf, int mode,
                            uint64_t seed, uint32_t ctr, const float* eps) {
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
  return a;
}

int fused_act_launch(const rlmd_agent_cfg& c, const float* obs, int64_t n, float* actions,
                     const float* actor_params, const NetOff& off, const unsigned short* w2bf, int mode,
                     uint64_t seed, uint32_t ctr, const float* eps, hipStream_t st, hipEvent_t ev_start,
                     hipEvent_t ev_stop) {
  int h1p, nb;
  RLMD_CHECK(fused_shape(c, h1p, nb), "fused acting: unsupported net shape");
  const FusedActArgs a = fused_act_args(c, obs, n, actions, actor_params, off, w2bf, mode, seed, ctr, eps);
  const dim3 grid((unsigned)((n + kRows - 1) / kRows));
  const int sp = c.state_dim <= 8 ? 8 : 16;
  RLMD_CHECK(c.action_dim <= kMaxA4, "fused acting: at most 4 actions");
  const bool wpc4 = act_wpc(h1p, c.action_dim <= kMaxA ? kMaxA : kMaxA4, grid.x) == 4;
#define ACT_LAUNCH2(H1P_, NB_, SP_, MA_, W_)                                                                          \
  hipExtLaunchKernelGGL((fused_act_kernel<H1P_, NB_, SP_, MA_, W_>), grid, dim3(256),                           \
                        act_lds_bytes(H1P_, SP_, MA_, act_park(H1P_, SP_, MA_, W_)), st, ev_start, ev_stop, 0, a)
#define ACT_LAUNCH1(H1P_, NB_, SP_, MA_)                                                        \
  do {                                                                                          \
    if (wpc4) ACT_LAUNCH2(H1P_, NB_, SP_, MA_, ((H1P_) == 256 && (MA_) == kMaxA) ? 4 : 3);      \
    else ACT_LAUNCH2(H1P_, NB_, SP_, MA_, 3);                                                   \
  } while (0)
#define ACT_LAUNCH(H1P_, NB_, SP_)                                            \
  {                                                                           \
    if (c.action_dim <= kMaxA) ACT_LAUNCH1(H1P_, NB_, SP_, kMaxA);            \
    else ACT_LAUNCH1(H1P_, NB_, SP_, kMaxA4);                                 \
  }
  if (h1p == 256) {
    if (sp == 8) ACT_LAUNCH(256, 4, 8)
    else ACT_LAUNCH(256, 4, 16)
  } else if (h1p == 128) {
    if (sp == 8) ACT_LAUNCH(128, 4, 8)
    else ACT_LAUNCH(128, 4, 16)
  } else {
    if (sp == 8) ACT_LAUNCH(416, 5, 8)
    else ACT_LAUNCH(416, 5, 16)
  }
#undef ACT_LAUNCH
#undef ACT_LAUNCH1
#undef ACT_LAUNCH2
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd

#ifdef RLMD_TIMING
extern "C" int rlmd_debug_ts_act(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rlmd::actrows::g_ts_act), sizeof(unsigned long long) * 8 * n) != hipSuccess;
}
#endif
