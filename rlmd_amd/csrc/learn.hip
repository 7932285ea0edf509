// learn.hip — SAC / TD3 learn() for gfx950 as a chain of HIP kernels.
//
// Restated reference (majidsina/rlmd):
//   SAC  algos/algo_sac.py:300-367 (_multi_step_target), :369-595 (learn),
//        :597-615 (Polyak); networks algos/networks_sac.py:101-178, :337-362
//   TD3  algos/algo_td3.py:302-361, :363-531, :533-563; algos/networks_td3.py:76-91, :152-168
//   critic losses / tail index  tools/critic_loss.py:26-341 (loss_function :344-453)
//   Adam (torch defaults, betas .9/.999, eps 1e-8), Polyak tau
// The MLP contractions run on the MFMA GEMM of gemm.hip; everything else here
// is row-parallel (one wave per mini-batch row) or a single-workgroup
// reduction/sort over the mini-batch (B <= 1024: bitonic sorts in LDS).
// All per-update scalars (Cauchy scales, log alpha, learn counter) stay on the
// device in LearnState; nothing synchronises with the host inside learn().
#include <math.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "learn_kernels.h"
#include "rlmd_update.h"
#include "rlmd_act_rows.h"
#include "rlmd_block.h"
#include "rlmd_loss.h"
#include "rlmd_policy.h"
#include "rlmd_adam.h"
#include "rlmd_gemm.h"

namespace rlmd {
namespace {


// ---------------------------------------------------------------------------
// actor heads + policy sampling (networks_sac.py:101-178, :268-285;
// networks_td3.py:76-91; algo_td3.py:198-223, :327-344).  One wave per row.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) actor_head_kernel(HeadArgs h) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= h.n) return;
  const NetOff& o = h.off;
  const int H = o.h2, A = h.A;
  const float* x = h.h2 + (int64_t)b * H;
  const uint32_t c1 = h.ctr ? (uint32_t)*h.ctr : h.ctr_host;
  if (h.xsa)
    for (int k = lane; k < h.S; k += 64) h.xsa[(int64_t)b * (h.S + A) + k] = h.state[(int64_t)b * h.S + k];
  float lp_sum = 0.f, m2_sum = 0.f, hld_sum = 0.f, jac_sum = 0.f;
  for (int j = 0; j < A; ++j) {
    float dm = 0.f, dl = 0.f;
    const float* wm = h.params + o.w3 + (int64_t)j * H;
    const float* wl = h.params + o.w4 + (int64_t)j * H;
    for (int k = lane; k < H; k += 64) {
      const float xv = x[k];
      dm = fmaf(xv, wm[k], dm);
      if (h.algo == RLMD_SAC) dl = fmaf(xv, wl[k], dl);
    }
    dm = wave_sum(dm);
    if (h.algo == RLMD_SAC) dl = wave_sum(dl);
    if (lane != 0) continue;
    const float mu = dm + h.params[o.b3 + j];
    float a;
    float noise = 0.f;
    if (h.mode == 0 || h.algo == RLMD_TD3) {
      if (h.eps_in) noise = h.eps_in[(int64_t)b * A + j];
      else if (h.mode == 0)
        noise = policy_draw(h.algo == RLMD_SAC ? h.dist : RLMD_DIST_N, h.seed, (uint32_t)b, c1, h.tag, j);
    }
    if (h.algo == RLMD_SAC) {
      const float ls_raw = dl + h.params[o.b4 + j];
      const PolicyComp pc = policy_comp(h.dist, mu, ls_raw, noise, h.ls_min, h.ls_max);
      if (h.mode == 1) {
        a = tanhf(pc.mu) * h.max_action;
      } else {
        a = tanhf(pc.u) * h.max_action;
        const float an = a / h.max_action;
        lp_sum += pc.lp;
        m2_sum += pc.m2;
        hld_sum += pc.hld;
        jac_sum += logf(1.f - an * an + h.reparam_noise);
        if (h.save) {
          float* sv = h.save + (int64_t)b * 5 * A;
          sv[j] = pc.mu;
          sv[A + j] = pc.sigma;
          sv[2 * A + j] = pc.c;
          sv[3 * A + j] = pc.u;
          sv[4 * A + j] = ls_raw;
        }
      }
    } else {
      const float t = tanhf(mu);
      a = t * h.max_action;
      if (h.mode == 0) {
        float nz = noise * h.noise_std;
        if (h.clamp_noise) nz = fminf(fmaxf(nz, -h.noise_clip), h.noise_clip);
        a = fminf(fmaxf(a + nz, -h.max_action), h.max_action);
      }
      if (h.save) h.save[(int64_t)b * 5 * A + j] = mu;  // pre-tanh for backward
    }
    if (h.actions) h.actions[(int64_t)b * A + j] = a;
    if (h.xsa) h.xsa[(int64_t)b * (h.S + A) + h.S + j] = a;
  }
  if (lane == 0 && h.logp) h.logp[b] = policy_logp(h.dist, A, lp_sum, m2_sum, hld_sum, jac_sum);
}

// ---------------------------------------------------------------------------
// Critic loss, top-k, tail index, CIM kernel, Nagy scale as one workgroup
// (rlmd_loss.h).  Launched for B > 512 (dq + statistics) and, on updates
// without an actor step, for the statistics alone (cbwd_rows forms dq).
// ---------------------------------------------------------------------------
#ifdef RLMD_TIMING
// experiment builds only (tools/ts_probe.py): thread-0 s_memtime checkpoints
__device__ unsigned long long g_ts[64];
#define RLMD_TS(i)                                                   \
  do {                                                               \
    if (threadIdx.x == 0) g_ts[i] = __builtin_amdgcn_s_memtime();    \
  } while (0)
#else
#define RLMD_TS(i) \
  do {             \
  } while (0)
#endif

template <int NTH>
__global__ void __launch_bounds__(NTH) critic_loss_kernel(LossArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t runs[NTH];
  __shared__ int rank_of[3][NTH];
  __shared__ float red[16 * 9];
  critic_loss_block<NTH / 64>(a, runs, &rank_of[0][0], red);
}

// ---------------------------------------------------------------------------
// Actor loss (algo_sac.py:524-562 / algo_td3.py:507-523) and the temperature
// gradient (algo_sac.py:580-587).  One workgroup; writes dL/dq per critic and
// dL/dlogp per row.
// ---------------------------------------------------------------------------
struct ActorLossArgs {
  const float* qpart[2];  // q per row without the head bias [B]; qpart[1] null for TD3
  const float* qb[2];
  const float* logp;  // SAC
  float* dq[2];
  float* dlogp;
  LearnState* st;
  float* stats;
  int32_t B, k, algo, topk;
  float target_entropy;
  int32_t cnt;  // learn_step_cntr (LearnState slot of log alpha)
};

template <int NTH>
__global__ void __launch_bounds__(NTH) actor_loss_kernel(ActorLossArgs a) {
  __shared__ __attribute__((aligned(16))) uint64_t runs[NTH];
  __shared__ int rank_of[NTH];
  __shared__ float red[16 * 4];
  const int b = threadIdx.x, B = a.B;
  const bool in = b < B;
  LearnState* st = a.st;
  const float alpha = a.algo == RLMD_SAC ? expf(st->log_alpha[slot_rd(a.cnt)]) : 0.f;
  const int64_t nB = (int64_t)B * 4;
  float q1 = rlmd_ldf(rlmd_rsrc(a.qpart[0], nB), b, in) + a.qb[0][0];
  float q2 = a.qpart[1] ? rlmd_ldf(rlmd_rsrc(a.qpart[1], nB), b, in) + a.qb[1][0] : q1;
  if (!in) q1 = q2 = 0.f;
  const float lp = a.logp ? rlmd_ldf(rlmd_rsrc(a.logp, nB), b, in) : 0.f;
  const float v = a.algo == RLMD_SAC ? fminf(q1, q2) - alpha * lp : q1;
  const int k = a.topk ? (B < a.k ? B : a.k) : B;
  bool sel = in;
  if (a.topk) {
    // SAC sorts descending, TD3 ascending
    const uint64_t key = in ? ((uint64_t)(a.algo == RLMD_SAC ? ~f2key(v) : f2key(v)) << 32) | (uint32_t)b : ~0ull;
    block_rank<NTH / 64>(key, runs, rank_of);
    sel = in && rank_of[b] < k;
  }
  float sm[2] = {sel ? v : 0.f, in ? -(lp + a.target_entropy) : 0.f};
  float mx[1] = {-INFINITY};
  block_allreduce<2, 0>(sm, mx, red);
  const float loss = -sm[0] / k;
  const float dv = sel ? -1.f / (float)k : 0.f;
  if (in) {
    if (a.algo == RLMD_SAC) {
      // d min(q1, q2): ties split evenly (torch.minimum backward)
      const float g1 = q1 < q2 ? 1.f : (q1 > q2 ? 0.f : 0.5f);
      a.dq[0][b] = dv * g1;
      a.dq[1][b] = dv * (1.f - g1);
      a.dlogp[b] = -alpha * dv;
    } else {
      a.dq[0][b] = dv;
    }
  }
  if (b == 0) {
    // temperature: d/dlog_alpha mean(-alpha (logp + target_entropy)) (algo_sac.py:580-587)
    if (a.algo == RLMD_SAC) st->pad_temp_grad = sm[1] / B * alpha;
    a.stats[10] = loss;
  }
}

}  // namespace
}  // namespace rlmd

// ============================================================================
// host orchestration
// ============================================================================
namespace rlmd {
namespace {

NetOff make_net(int in, int h1, int h2, int out, bool two_heads) {
  NetOff o{};
  o.in = in;
  o.h1 = h1;
  o.h2 = h2;
  o.out = out;
  o.w1 = 0;
  o.b1 = o.w1 + (int64_t)h1 * in;
  o.w2 = o.b1 + h1;
  o.b2 = o.w2 + (int64_t)h2 * h1;
  o.w3 = o.b2 + h2;
  o.b3 = o.w3 + (int64_t)out * h2;
  if (two_heads) {
    o.w4 = o.b3 + out;
    o.b4 = o.w4 + (int64_t)out * h2;
    o.size = o.b4 + out;
  } else {
    o.w4 = o.b4 = -1;
    o.size = o.b3 + out;
  }
  return o;
}

struct Scratch {
  // mini-batch
  float *s, *a, *r, *s2, *xsa;
  uint8_t* done;
  // target path: target q per row (no head bias), logp of the next actions
  float *logp_next, *tpart[2], *y;
  float* tpartn[2];  // TD3 target pairing: the next update's target q (fwd_rows npair)
  float* qbias;  // [4] q_value.bias of the online, then target critics at loss time
  // critic path
  float *c1[2], *c2[2], *qpart[2], *dq[2], *dc2[2], *dc1[2];
  // actor path
  float *h1, *h2, *logp, *xsan, *save;
  float *e1[2], *e2[2], *qnpart[2], *dqn[2], *dlogp;
  float *gh, *dh2, *dh1;
  // ReLU masks (bytes, rows.hip m1_index / m2_index layouts) of c1/c2, e1/e2, h1/h2
  uint8_t *cm1[2], *cm2[2], *em1[2], *em2[2], *am1, *am2;
  float* stats;  // [16] when the caller passes none
  // fused critic update (update.hip): row-packed h1 / h2 (compute type), the
  // backward basis U1 (f32) and the q_value.weight snapshot per critic
  unsigned char *hp1[2], *hp2[2];
  float *u1[2], *w3s[2];
  // fused actor update: the policy's row-packed h1 / h2, its per-head backward
  // bases, the head weights' snapshot, the critics' dq/da per row
  unsigned char *hp1a, *hp2a;
  float *ua, *wheads, *dqda[2];
  int32_t* rank1;  // the rows' top-k selection ranks of this update (critic update -> statistics)
};

// In-library event profiler of one agent handle (bench.py: live per-phase kernel
// durations of its train steps and acting calls).
struct PhaseProfiler {
  ~PhaseProfiler() {
    for (auto& ph : ev)
      for (auto& v : ph)
        for (hipEvent_t e : v) (void)hipEventDestroy(e);
  }
  bool enabled = false;
  int mask = 7;  // phases recorded: bit p = phase p (rlmd_profile_enable: 1 all, 2 the env kernel's only)
  // rlmd_profile_enable(3): kernel-attached pairs only — the env kernel's dispatch
  // (phase 1) and, in unfused train steps, the acting kernel's own dispatch (phase
  // 0) instead of markers around acting: the in-step acting-only reference of the
  // fused kernel's marginal (same cache state as act_env_kernel, after K updates)
  bool kernel_pairs = false;
  std::vector<hipEvent_t> ev[3][2];  // phase x {start, stop}: 0 act, 1 env, 2 learn
  size_t used[3] = {0, 0, 0};
  // sampling (rlmd_profile_stride): only every stride-th occurrence of a phase is
  // timed — each attached event pair costs the stream a few us, so the headline's
  // live kernel timing samples the timed region instead of stamping every step
  int stride = 1;
  uint64_t seen[3] = {0, 0, 0};
  bool skip[3] = {false, false, false};
  bool sample(int phase) { return (seen[phase]++ % (uint64_t)stride) == 0; }
  int record(int phase, int which, hipStream_t s) {
    if (!enabled || !(mask >> phase & 1)) return 0;
    if (which == 0) skip[phase] = !sample(phase);
    if (skip[phase]) return 0;
    auto& v = ev[phase][which];
    const size_t i = which == 0 ? used[phase] : used[phase] - 1;
    if (i >= v.size()) {
      hipEvent_t e;
      RLMD_HIP(hipEventCreate(&e));
      v.push_back(e);
    }
    RLMD_HIP(hipEventRecord(v[i], s));
    if (which == 0) used[phase]++;
    return 0;
  }
  // a {start, stop} pair for one kernel launch (hipExtLaunchKernelGGL stamps
  // them at the dispatch's own begin / end, like rocprofv3's kernel trace);
  // {null, null} when disabled
  int pair(int phase, hipEvent_t* start, hipEvent_t* stop) {
    *start = *stop = nullptr;
    if (!enabled || !(mask >> phase & 1)) return 0;
    if (!sample(phase)) return 0;
    const size_t i = used[phase];
    for (int w = 0; w < 2; ++w)
      if (i >= ev[phase][w].size()) {
        hipEvent_t e;
        RLMD_HIP(hipEventCreate(&e));
        ev[phase][w].push_back(e);
      }
    *start = ev[phase][0][i];
    *stop = ev[phase][1][i];
    used[phase]++;
    return 0;
  }
};
}  // namespace
}  // namespace rlmd

struct rlmd_agent_s {
  rlmd_agent_cfg cfg;
  float *params, *target, *grads, *m, *v;
  int64_t n_params, off_actor, off_c[2];
  rlmd::NetOff actor, critic;
  rlmd::LearnState* st;
  float* zipf_x;
  float zipf_x2;
  rlmd::Scratch sc;
  std::vector<void*> allocs;
  // fc2.weight compute copies (rows.hip RowNet), slot x {wc, wt}:
  // 0 actor, 1 target actor, 2/3 critics, 4/5 target critics
  unsigned char* wcopy = nullptr;
  // K mini-batches sampled by one launch (agent_learn_k)
  int kcap = 0;
  float *kb_s = nullptr, *kb_a = nullptr, *kb_r = nullptr, *kb_s2 = nullptr, *kb_xsa = nullptr;
  uint8_t* kb_done = nullptr;
  int64_t* kb_idx = nullptr;
  int32_t* kb_eff = nullptr;
  size_t wcopy_bytes = 0;  // per copy
  float *act_h1 = nullptr, *act_h2 = nullptr;
  int64_t act_cap = 0;
  int64_t host_cntr = 0;
  // fused optimiser epilogue of the weight-gradient GEMM (rlmd_gemm.h)
  __attribute__((ext_vector_type(4))) float* slabs = nullptr;
  unsigned* tile_ctr = nullptr;
  int32_t max_tiles = 0;
  bool fuse_adam = false;
  int fuse_splits = RLMD_GRAD_SPLITS;
  // the compute copies may differ from the f32 masters: set at creation and by
  // rlmd_agent_params_written (host writes through the parameter tensors);
  // the optimiser keeps them current otherwise
  bool copies_dirty = true;
  // critic step as one launch (update.hip) for B <= 512; RLMD_NO_FUSED_UPDATE=1:
  // row backward + weight-gradient GEMM + Adam launches
  bool fused_update = false;
  bool target_pair = true;  // TD3: next update's target path in this update's forward (RLMD_TARGET_PAIR=0: off)
  bool fused_actor = false;  // the actor step too (actions <= 2)
  int n_cu = 256;            // compute units this agent may count on (column-split decisions;
                             // the device's, or rlmd_agent_set_cu_budget)
  int qsplit_max = 2;        // qeval_rows column split allowed (RLMD_QSPLIT=1: off)
  int fsplit_max = 2;        // fwd_rows critic column split allowed (RLMD_FSPLIT=1: off)
  rlmd::PhaseProfiler prof;  // rlmd_profile_enable / _read
};

namespace rlmd {
namespace {

int agent_alloc(rlmd_agent_s* ag, void** p, size_t bytes) {
  RLMD_HIP(hipMalloc(p, bytes < 16 ? 16 : bytes));
  ag->allocs.push_back(*p);
  return 0;
}
#define RLMD_ALLOC(ptr, count)                                                             \
  do {                                                                                     \
    int _r = rlmd::agent_alloc(ag, (void**)&(ptr), sizeof(*(ptr)) * (size_t)(count));             \
    if (_r) return _r;                                                                     \
  } while (0)

// y = relu?(x W^T + b) for up to two nets of identical shape
int fwd(rlmd_agent_s* ag, int groups, int M, int N, int K, bool relu, const float* const* X,
        int ldx, const float* const* W, const float* const* bias, float* const* Y,
        hipStream_t s, const float* const* head_w = nullptr, float* const* head_part = nullptr) {
  GemmBatch b{};
  for (int g = 0; g < groups; ++g)
    gemm_add(b, {M, N, K, relu ? 1 : 0},
             {X[g], ldx, W[g], K, bias[g], Y[g], N, nullptr, 0, nullptr, head_w ? head_w[g] : nullptr,
              head_part ? head_part[g] : nullptr});
  b.splits = 1;
  return gemm_launch(ag->cfg.precision, GEMM_FWD, b, s);
}

// dW [M=out, N=in] = G^T X over K = batch rows; db = colsum(G).  Appends to a
// multi-problem batch launched once per phase (gemm_launch, RLMD_GRAD_SPLITS slabs).
void add_bwd_w(GemmBatch& b, int M, int N, int K, const float* G, int ldg, const float* X, int ldx,
               float* DW, float* DB) {
  gemm_add(b, {M, N, K, 0}, {G, ldg, X, ldx, nullptr, DW, N, nullptr, 0, DB, nullptr, nullptr});
}


#define RLMD_TRY(x)         \
  do {                      \
    int _r = (x);           \
    if (_r) return _r;      \
  } while (0)

HeadArgs head_args(rlmd_agent_s* ag, const float* params, const float* h2, const float* state, int n) {
  const rlmd_agent_cfg& c = ag->cfg;
  HeadArgs h{};
  h.h2 = h2;
  h.params = params;
  h.off = ag->actor;
  h.state = state;
  h.n = n;
  h.S = c.state_dim;
  h.A = c.action_dim;
  h.algo = c.algo;
  h.seed = c.seed;
  h.max_action = c.max_action;
  h.ls_min = c.log_scale_min;
  h.ls_max = c.log_scale_max;
  h.reparam_noise = c.reparam_noise;
  h.dist = c.policy_dist;
  return h;
}

int launch_head(const HeadArgs& h, hipStream_t s) {
  hipLaunchKernelGGL(actor_head_kernel, dim3((h.n + 3) / 4), dim3(256), 0, s, h);
  RLMD_LAUNCH_CHECK();
  return 0;
}

// torch.optim.Adam's bias corrections for step t, evaluated in double on the
// host as torch evaluates them in Python floats, handed over as f32 scalars.
void adam_scalars(double lr, int t, float& step_size, float& bc2_sqrt) {
  const double bc1 = 1.0 - pow(0.9, (double)t), bc2 = 1.0 - pow(0.999, (double)t);
  step_size = (float)(lr / bc1);
  bc2_sqrt = (float)sqrt(bc2);
}

// Adam over the nets of one phase: sums the RLMD_GRAD_SPLITS weight-gradient
// slabs in slab order, then steps, Polyak-averages and refreshes the compute
// copies (rlmd_adam.h).  Block 0 also steps the temperature.
__global__ void __launch_bounds__(256) adam_kernel(AdamArgs a, int64_t split_stride) {
  const bool polyak = adam_polyak(a);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)a.n; i += gridDim.x * blockDim.x) {
    const AdamIn in = adam_load(a, i, polyak);
    float g = a.g[i];
#pragma unroll
    for (int sp = 1; sp < RLMD_GRAD_SPLITS; ++sp) g += a.g[i + sp * split_stride];
    adam_apply(a, i, g, in, polyak);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) adam_scalar_step(a);
}

// Weight gradients of one phase, then the optimiser step.  Two launches: the
// split-K GEMM writes RLMD_GRAD_SPLITS slabs over 4x the workgroups, and
// adam_kernel reduces them.  GemmBatch::fuse_adam instead lets each tile's last
// arriving split sum the slabs and step its parameters inside the GEMM
// (write-through slabs + arrival tickets); it is exact (same slab order) but
// measured slower at C2: 18.4 + 13.1 us against 8.0 + 6.3 and 6.5 + 5.2 us
// separate, the publish / ticket / cross-XCD read tail costing more than the
// launch it saves.  Kept selectable (RLMD_FUSE_ADAM=1 at agent creation) for
// larger nets and covered by tests/test_learn_gpu.py; RLMD_FUSE_SPLITS=1 / 2
// (one tile owns the whole K-sum and steps from its accumulators) is slower
// still at C2 (bench 77.2M / 82.5M against 84.1M fused split-4 and 90.7M
// separate): the critic phase has ~150 tiles, too few to fill 256 CUs.

int launch_bwd_w_adam(rlmd_agent_s* ag, GemmBatch& b, const AdamArgs& ad_in, hipStream_t s) {
  b.splits = ag->fuse_adam ? ag->fuse_splits : RLMD_GRAD_SPLITS;
  b.split_stride = ag->n_params;
  AdamArgs a = ad_in;
  adam_scalars(a.lr, a.cnt / a.interval, a.step_size, a.bc2_sqrt);
  if (a.temp && a.cnt % a.temp_interval == 0)
    adam_scalars(a.lr_temp, a.cnt / a.temp_interval, a.temp_step_size, a.temp_bc2_sqrt);
  if (ag->fuse_adam) {
    b.fuse_adam = 1;
    b.adam = a;
    b.slabs = ag->slabs;
    b.tile_ctr = ag->tile_ctr;
    b.max_tiles = ag->max_tiles;
    return gemm_launch(ag->cfg.precision, GEMM_BWD_W, b, s);
  }
  RLMD_TRY(gemm_launch(ag->cfg.precision, GEMM_BWD_W, b, s));
  const int64_t blocks = std::min<int64_t>((a.n + 255) / 256, 1024);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s, a,
                     (int64_t)ag->n_params);
  RLMD_LAUNCH_CHECK();
  return 0;
}

enum { SLOT_ACTOR = 0, SLOT_TACTOR = 1, SLOT_C0 = 2, SLOT_TC0 = 4 };

RowDims row_dims(const rlmd_agent_s* ag) {
  const rlmd_agent_cfg& c = ag->cfg;
  RowDims d{};
  d.S = c.state_dim;
  d.A = c.action_dim;
  d.X = c.state_dim + c.action_dim;
  d.H1 = c.h1;
  d.H2 = c.h2;
  d.H1p = pad32(c.h1);
  d.H2p = pad32(c.h2);
  d.B = c.batch;
  d.algo = c.algo;
  d.prec = c.precision;
  return d;
}

void* copy_wc(rlmd_agent_s* ag, int slot) { return ag->wcopy + (size_t)(2 * slot) * ag->wcopy_bytes; }
void* copy_wt(rlmd_agent_s* ag, int slot) { return ag->wcopy + (size_t)(2 * slot + 1) * ag->wcopy_bytes; }

RowNet row_net(rlmd_agent_s* ag, int slot) {
  const float* base = (slot == SLOT_TACTOR || slot >= SLOT_TC0) ? ag->target : ag->params;
  const int64_t off = slot <= SLOT_TACTOR ? ag->off_actor : ag->off_c[(slot - SLOT_C0) & 1];
  return RowNet{base + off, copy_wc(ag, slot), copy_wt(ag, slot)};
}

// Re-derive every compute copy from the f32 masters when the host has written
// parameters since the last refresh (rlmd_agent_params_written); Adam keeps
// them current between host writes, so a clean agent skips the six copies.
int refresh_copies(rlmd_agent_s* ag, hipStream_t st) {
  if (!ag->copies_dirty) return 0;
  ag->copies_dirty = false;
  CopyJob jobs[6];
  for (int slot = 0; slot < 6; ++slot) {
    const RowNet n = row_net(ag, slot);
    const NetOff& o = slot <= SLOT_TACTOR ? ag->actor : ag->critic;
    jobs[slot] = CopyJob{n.p + o.w2, copy_wc(ag, slot), copy_wt(ag, slot)};
  }
  return w2_copies_launch(jobs, 6, row_dims(ag), st);
}

void adam_copies(rlmd_agent_s* ag, AdamArgs& ad, const NetOff& o, int slot0, int n, bool targets) {
  const rlmd_agent_cfg& c = ag->cfg;
  ad.ncopy = n;
  ad.bf16 = c.precision == RLMD_BF16;
  ad.net_size = o.size;
  ad.w2_off = o.w2;
  ad.H1 = c.h1;
  ad.H2 = c.h2;
  ad.H1p = pad32(c.h1);
  ad.H2p = pad32(c.h2);
  const int tslot0 = slot0 == SLOT_ACTOR ? SLOT_TACTOR : SLOT_TC0;
  for (int i = 0; i < n; ++i) {
    ad.wc[i] = copy_wc(ag, slot0 + i);
    ad.wt[i] = copy_wt(ag, slot0 + i);
    ad.twc[i] = targets ? copy_wc(ag, tslot0 + i) : nullptr;
    ad.twt[i] = targets ? copy_wt(ag, tslot0 + i) : nullptr;
  }
}

// One learn() on the mini-batch already in ag->sc (s, r, s2, done, xsa).
// eps_a / eps_b: injected noise (nullable).  stats: [16] device.
// Launches (SAC, actor step): fwd rows | critic loss | critic bwd rows | critic
// dW | Adam critics | q rows on (s, a_new) | actor loss | actor bwd rows |
// actor dW | Adam actor (+ temperature).
// One mini-batch (device): s, s' [B, S], r [B], done [B], critic input
// xsa = [s | a] [B, S+A], eff [B] (nullable = 1).
struct Batch {
  const float *s, *r, *s2, *xsa;
  const uint8_t* done;
  const int32_t* eff;
};

// TD3 target pairing between consecutive updates of one call (algo_td3.py:
// learn() forms the target from the target networks, which change only at
// learn_step_cntr % td3_target_{critic,actor}_update == 0): when update n changes
// no target network, update n + 1's target path — target actor on its s', the
// clipped noise of its counter, both target critics — runs as two more jobs of
// update n's forward (same kernel code, same parameters: bit-identical), and
// update n + 1's forward skips jobs 0 / 1.  s2n: the next mini-batch's s'
// (nullable: last update of the call); ready: this update's targets are in
// tpartn; paired (out): the next update's targets were computed here.
struct PairCtl {
  const float* s2n;
  bool ready, paired;
  int split;  // the pairing update's fwd column split: its target halves are this update's
};

int learn_body(rlmd_agent_s* ag, const Batch& mb, const float* eps_a, const float* eps_b, float* stats,
               hipStream_t st, PairCtl* pc = nullptr) {
  const rlmd_agent_cfg& c = ag->cfg;
  Scratch& S_ = ag->sc;
  const int B = c.batch, S = c.state_dim, A = c.action_dim, X = S + A, H1 = c.h1, H2 = c.h2;
  const bool sac = c.algo == RLMD_SAC;
  float* P = ag->params;
  float* T = ag->target;
  float* G = ag->grads;
  const NetOff& ao = ag->actor;
  const NetOff& co = ag->critic;
  const int64_t cntr = ++ag->host_cntr;  // learn_step_cntr after this update's increment
  const bool actor_step = cntr % c.actor_update_interval == 0;
  const int nq = sac ? 2 : 1;
  const RowDims d = row_dims(ag);
  const SampleCfg smp{c.seed, (uint32_t)cntr, c.max_action, c.log_scale_min, c.log_scale_max,
                      c.reparam_noise, c.algo == RLMD_SAC ? c.policy_dist : RLMD_DIST_N};
  float* Pc[2] = {P + ag->off_c[0], P + ag->off_c[1]};
  float* Tc[2] = {T + ag->off_c[0], T + ag->off_c[1]};
  float* Gc[2] = {G + ag->off_c[0], G + ag->off_c[1]};
  float* Ga = G + ag->off_actor;
  const RowNet crit[2] = {row_net(ag, SLOT_C0), row_net(ag, SLOT_C0 + 1)};
  const bool ready = pc && pc->ready;
  const bool target_change = cntr % c.target_critic_update == 0 || (actor_step && cntr % c.target_actor_update == 0);
  const bool pair = pc && pc->s2n && !ready && !sac && ag->target_pair && ag->fused_update && eps_a == nullptr &&
                    !target_change;
  if (pc) pc->paired = pair;
  // column split of the forward's critic streams (target critics, online critics
  // + their U1 bases): two workgroups per (rows, job) when the grid still fits
  // the chip in one round; the halves' partial sums meet in the critic step
  int fsplit = 1;
  {
    const int ny = (actor_step ? 5 : 4) - (ready ? 2 : 0) + (pair ? 2 : 0);
    if (ag->fused_update && ag->fsplit_max > 1 && d.H2p % 64 == 0 && 2 * ((B + 15) / 16) * ny <= ag->n_cu)
      fsplit = 2;
    // targets computed by the previous update's forward carry its split (the
    // partial layout of tpartn); this update's fewer jobs fit whenever its did
    if (ready) fsplit = pc->split;
    if (pc) pc->split = fsplit;
  }

  // ---- forward rows: target path (algo_sac.py:300-367 / algo_td3.py:302-361),
  //      critics on (s, a) (algo_sac.py:413-417), policy on s for the actor step
  {
    FwdRowsArgs f{};
    f.d = d;
    f.ao = ao;
    f.co = co;
    f.smp = smp;
    f.tactor = row_net(ag, sac ? SLOT_ACTOR : SLOT_TACTOR);  // SAC samples next actions from the online actor
    f.tcrit[0] = row_net(ag, SLOT_TC0);
    f.tcrit[1] = row_net(ag, SLOT_TC0 + 1);
    f.s2 = mb.s2;
    f.eps_next = eps_a;
    f.t_tag = sac ? RLMD_TAG_EPS_NEXT : RLMD_TAG_TD3_TARGET;
    f.t_clamp = sac ? 0 : 1;
    f.t_noise_std = c.target_policy_noise;
    f.t_noise_clip = c.target_policy_clip;
    f.logp_next = S_.logp_next;
    for (int g = 0; g < 2; ++g) {
      f.qt[g] = S_.tpart[g];
      f.crit[g] = crit[g];
      f.c1[g] = S_.c1[g];
      f.c2[g] = S_.c2[g];
      f.cm1[g] = S_.cm1[g];
      f.cm2[g] = S_.cm2[g];
      f.q[g] = S_.qpart[g];
    }
    f.xsa = mb.xsa;
    f.with_actor = actor_step ? 1 : 0;
    f.a_mode = sac ? 0 : 1;  // TD3 actor.forward: tanh(mu) * max_action, no noise
    f.a_tag = RLMD_TAG_EPS_CUR;
    f.actor = row_net(ag, SLOT_ACTOR);
    f.s = mb.s;
    f.eps_cur = eps_b;
    f.h1a = S_.h1;
    f.h2a = S_.h2;
    f.am1 = S_.am1;
    f.am2 = S_.am2;
    f.xsan = S_.xsan;
    f.logp = S_.logp;
    f.save = S_.save;
    if (ag->fused_update) {
      for (int g = 0; g < 2; ++g) {
        f.u1[g] = S_.u1[g];
        f.hp1[g] = S_.hp1[g];
        f.hp2[g] = S_.hp2[g];
        f.w3s[g] = S_.w3s[g];
      }
      f.bsnap = S_.qbias;
    }
    if (ag->fused_actor && actor_step) {
      f.hp1a = S_.hp1a;
      f.hp2a = S_.hp2a;
    }
    f.y0 = ready ? 2 : 0;
    if (pair) {
      f.npair = 1;
      f.s2n = pc->s2n;
      f.qtn[0] = S_.tpartn[0];
      f.qtn[1] = S_.tpartn[1];
      f.ctrn = (uint32_t)(cntr + 1);
    }
    RLMD_TRY(fwd_rows_launch(f, st, fsplit));
  }
  // ---- critic loss (algo_sac.py:413-465)
  LossArgs loss_fused{}, loss_stats{};  // B == 0: not used
  {
    LossArgs la{};
    for (int g = 0; g < 2; ++g) {
      la.qpart[g] = S_.qpart[g];
      la.qb[g] = Pc[g] + co.b3;
      la.tpart[g] = ready ? S_.tpartn[g] : S_.tpart[g];
      la.tb[g] = Tc[g] + co.b3;
    }
    la.r = mb.r;
    la.done = mb.done;
    la.eff = mb.eff;
    la.logp_next = S_.logp_next;
    la.gamma = c.gamma;
    la.reward_scale = c.reward_scale;
    la.y_out = S_.y;
    la.dq[0] = S_.dq[0];
    la.dq[1] = S_.dq[1];
    la.zipf_x = ag->zipf_x;
    la.zipf_x2 = ag->zipf_x2;
    la.st = ag->st;
    la.stats = stats;
    la.B = B;
    la.k = c.topk;
    la.loss_type = c.loss_type;
    la.algo = c.algo;
    la.log_noise = c.log_noise;
    la.grad_scale = sac ? 0.5f : 1.0f;  // SAC: 0.5 (q1_loss + q2_loss)
    la.cnt = (int32_t)cntr;
    la.qsplit = fsplit;
    if (B > 512) {
      hipLaunchKernelGGL(critic_loss_kernel<1024>, dim3(1), dim3(1024), 0, st, la);
      RLMD_LAUNCH_CHECK();
    } else {
      // B <= 512: cbwd_rows forms dq per row workgroup; the statistics come
      // from a workgroup of abwd_rows (actor step) or a kernel after cbwd
      // the statistics run after the critic Adam step has moved the heads'
      // biases: they read the loss-time biases cbwd_rows saved
      loss_fused = la;
      loss_stats = la;
      loss_stats.dq[0] = loss_stats.dq[1] = nullptr;
      for (int g = 0; g < 2; ++g) {
        loss_stats.qb[g] = S_.qbias + g;
        loss_stats.tb[g] = S_.qbias + 2 + g;
      }
    }
  }
  // ---- critic step in one launch: loss gradient of every row, weight-gradient
  //      tiles, Adam + Polyak + compute copies of the owned parameters (update.hip)
  if (ag->fused_update) {
    CritUpdArgs cu{};
    cu.d = d;
    cu.co = co;
    cu.loss = loss_fused;
    for (int g = 0; g < 2; ++g) {
      cu.loss.qb[g] = S_.qbias + g;  // loss-time biases: the forward's snapshot
      cu.loss.tb[g] = S_.qbias + 2 + g;
      cu.m2[g] = S_.cm2[g];
      cu.hp1[g] = S_.hp1[g];
      cu.hp2[g] = S_.hp2[g];
      cu.u1[g] = S_.u1[g];
      cu.w3s[g] = S_.w3s[g];
    }
    cu.x = mb.xsa;
    AdamArgs ad{};
    ad.p = Pc[0];
    ad.g = Gc[0];
    ad.m = ag->m + ag->off_c[0];
    ad.v = ag->v + ag->off_c[0];
    ad.target = Tc[0];
    ad.n = 2 * co.size;
    ad.lr = c.lr_critic;
    ad.tau = c.tau;
    ad.cnt = (int32_t)cntr;
    ad.interval = 1;
    ad.polyak_interval = c.target_critic_update;
    ad.st = ag->st;
    adam_copies(ag, ad, co, SLOT_C0, 2, true);
    adam_scalars(ad.lr, ad.cnt / ad.interval, ad.step_size, ad.bc2_sqrt);
    cu.adam = ad;
    cu.tj = critic_update_tj(d);
    cu.ti = d.H2p / 32;
    cu.n_w2 = cu.ti * cu.tj;
    cu.n_w1 = d.H1p / 32;
    // the statistics workgroups of the fused actor step reuse the selection ranks
    if (ag->fused_actor && actor_step && loss_stats.B > 0) cu.rank_out = S_.rank1;
    // no actor step: the statistics run as two workgroups of the critic step's launch
    if (loss_stats.B > 0 && !actor_step) cu.cstats = loss_stats;
    RLMD_TRY(critic_update_launch(cu, st));
  } else {
    CBwdArgs cb{};
    cb.d = d;
    cb.co = co;
    for (int g = 0; g < 2; ++g) {
      cb.crit[g] = crit[g];
      cb.dq[g] = S_.dq[g];
      cb.cm1[g] = S_.cm1[g];
      cb.cm2[g] = S_.cm2[g];
      cb.dc2[g] = S_.dc2[g];
      cb.dc1[g] = S_.dc1[g];
    }
    cb.loss = loss_fused;
    cb.bias_out = S_.qbias;
    RLMD_TRY(cbwd_rows_launch(cb, st));
    if (loss_stats.B > 0 && !actor_step) {
      hipLaunchKernelGGL(critic_loss_kernel<512>, dim3(1), dim3(512), 0, st, loss_stats);
      RLMD_LAUNCH_CHECK();
    }
    GemmBatch gb{};
    for (int g = 0; g < 2; ++g) {
      add_bwd_w(gb, 1, H2, B, S_.dq[g], 1, S_.c2[g], H2, Gc[g] + co.w3, Gc[g] + co.b3);
      add_bwd_w(gb, H2, H1, B, S_.dc2[g], H2, S_.c1[g], H1, Gc[g] + co.w2, Gc[g] + co.b2);
      add_bwd_w(gb, H1, X, B, S_.dc1[g], H1, mb.xsa, X, Gc[g] + co.w1, Gc[g] + co.b1);
    }
    AdamArgs ad{};
    ad.p = Pc[0];
    ad.g = Gc[0];
    ad.m = ag->m + ag->off_c[0];
    ad.v = ag->v + ag->off_c[0];
    ad.target = Tc[0];
    ad.n = 2 * co.size;
    ad.lr = c.lr_critic;
    ad.tau = c.tau;
    ad.cnt = (int32_t)cntr;
    ad.interval = 1;
    ad.polyak_interval = c.target_critic_update;
    ad.st = ag->st;
    adam_copies(ag, ad, co, SLOT_C0, 2, true);
    RLMD_TRY(launch_bwd_w_adam(ag, gb, ad, st));
  }
  // ---- actor (+ temperature) update every actor_update_interval
  if (!actor_step) return 0;
  {
    QEvalArgs qe{};
    qe.d = d;
    qe.co = co;
    qe.x = S_.xsan;
    for (int g = 0; g < 2; ++g) {
      qe.crit[g] = crit[g];
      qe.e1[g] = nullptr;  // only the masks are consumed (abwd)
      qe.e2[g] = nullptr;
      qe.em1[g] = S_.em1[g];
      qe.em2[g] = S_.em2[g];
      qe.qn[g] = S_.qnpart[g];
      if (ag->fused_actor) qe.dqda[g] = S_.dqda[g];
    }
    qe.nq = nq;
    if (ag->fused_actor) {  // + the policy's per-head backward bases
      qe.nab = sac ? 2 * A : A;
      qe.ao = ao;
      qe.actor = row_net(ag, SLOT_ACTOR);
      qe.am1 = S_.am1;
      qe.am2 = S_.am2;
      qe.ua = S_.ua;
      qe.wheads = S_.wheads;
    }
    // column split of the critic / basis jobs: two workgroups per (rows, job), each
    // streaming half of an fc2 copy, when the halves are whole K-steps and the
    // grid still fits the chip in one round
    int qsplit = 1;
    if (ag->fused_actor && ag->qsplit_max > 1 && d.H2p % 64 == 0 &&
        ((B + 15) / 16) * (2 * nq + qe.nab) <= ag->n_cu)
      qsplit = 2;
    qe.split = qsplit;
    RLMD_TRY(qeval_rows_launch(qe, nq, st, qsplit));
    if (ag->fused_actor) {
      // the actor (+ temperature) step in one launch (update.hip)
      ActUpdArgs au{};
      au.d = d;
      au.ao = ao;
      au.smp = smp;
      au.nq = nq;
      for (int g = 0; g < 2; ++g) {
        au.qn[g] = S_.qnpart[g];
        au.qb[g] = Pc[g] + co.b3;
        au.dqda[g] = S_.dqda[g];
      }
      au.logp = S_.logp;
      au.save = S_.save;
      au.am2 = S_.am2;
      au.hp1a = S_.hp1a;
      au.hp2a = S_.hp2a;
      au.ua = S_.ua;
      au.wheads = S_.wheads;
      au.s = mb.s;
      au.st = ag->st;
      au.stats = stats;
      au.k = c.topk;
      au.topk = c.actor_topk;
      au.target_entropy = -(float)A;
      AdamArgs ad{};
      ad.p = P + ag->off_actor;
      ad.g = Ga;
      ad.m = ag->m + ag->off_actor;
      ad.v = ag->v + ag->off_actor;
      ad.target = sac ? nullptr : T + ag->off_actor;
      ad.n = ao.size;
      ad.lr = c.lr_actor;
      ad.tau = c.tau;
      ad.cnt = (int32_t)cntr;
      ad.interval = c.actor_update_interval;
      ad.polyak_interval = sac ? 0 : c.target_actor_update;
      ad.st = ag->st;
      ad.temp = sac ? 1 : 0;
      ad.lr_temp = c.lr_temp;
      ad.temp_interval = c.temp_update_interval;
      ad.stats = stats;
      adam_copies(ag, ad, ao, SLOT_ACTOR, 1, !sac);
      adam_scalars(ad.lr, ad.cnt / ad.interval, ad.step_size, ad.bc2_sqrt);
      if (ad.temp && ad.cnt % ad.temp_interval == 0)
        adam_scalars(ad.lr_temp, ad.cnt / ad.temp_interval, ad.temp_step_size, ad.temp_bc2_sqrt);
      au.adam = ad;
      au.cstats = loss_stats;
      au.cstats.rank_in = S_.rank1;  // critic_update_kernel wrote them (cu.rank_out)
      au.cstats.keep_actor_slot = 1;   // stats[10]: the actor loss
      au.cstats.keep_logtemp_slot = 1; // stats[11]: the temperature step
      au.tj = d.H1p / 32;
      au.ti = d.H2p / 32;
      au.n_w2 = au.ti * au.tj;
      au.n_w1 = actor_update_n_w1(d);
      au.qsplit = qsplit;
      RLMD_TRY(actor_update_launch(au, st));
      return 0;
    }
    // B <= 512: the actor loss is fused into abwd_rows (row ranks + a loss
    // workgroup); larger mini-batches use the one-workgroup loss kernel
    const bool fused_loss = B <= 512;
    if (!fused_loss) {
      ActorLossArgs al{};
      al.qpart[0] = S_.qnpart[0];
      al.qpart[1] = sac ? S_.qnpart[1] : nullptr;
      al.qb[0] = Pc[0] + co.b3;
      al.qb[1] = Pc[1] + co.b3;
      al.logp = sac ? S_.logp : nullptr;
      al.dq[0] = S_.dqn[0];
      al.dq[1] = S_.dqn[1];
      al.dlogp = S_.dlogp;
      al.st = ag->st;
      al.stats = stats;
      al.B = B;
      al.k = c.topk;
      al.algo = c.algo;
      al.topk = c.actor_topk;
      al.target_entropy = -(float)A;
      al.cnt = (int32_t)cntr;
      hipLaunchKernelGGL(actor_loss_kernel<1024>, dim3(1), dim3(1024), 0, st, al);
      RLMD_LAUNCH_CHECK();
    }
    ABwdArgs ab{};
    ab.d = d;
    ab.ao = ao;
    ab.co = co;
    ab.smp = smp;
    ab.nq = nq;
    for (int g = 0; g < 2; ++g) {
      ab.crit[g] = crit[g];
      ab.qn[g] = S_.qnpart[g];
      ab.em1[g] = S_.em1[g];
      ab.em2[g] = S_.em2[g];
      ab.dqn_ext[g] = fused_loss ? nullptr : S_.dqn[g];
    }
    ab.dlogp_ext = fused_loss ? nullptr : S_.dlogp;
    ab.actor = row_net(ag, SLOT_ACTOR);
    ab.logp = S_.logp;
    ab.save = S_.save;
    ab.am1 = S_.am1;
    ab.am2 = S_.am2;
    ab.st = ag->st;
    ab.stats = stats;
    ab.k = c.topk;
    ab.topk = c.actor_topk;
    ab.target_entropy = -(float)A;
    ab.gh = S_.gh;
    ab.dh2 = S_.dh2;
    ab.dh1 = S_.dh1;
    ab.cstats = loss_stats;
    ab.cstats.keep_actor_slot = 1;  // stats[10] belongs to the actor-loss workgroup
    RLMD_TRY(abwd_rows_launch(ab, st));
    GemmBatch gb{};
    add_bwd_w(gb, A, H2, B, S_.gh, 2 * A, S_.h2, H2, Ga + ao.w3, Ga + ao.b3);
    if (sac) add_bwd_w(gb, A, H2, B, S_.gh + A, 2 * A, S_.h2, H2, Ga + ao.w4, Ga + ao.b4);
    add_bwd_w(gb, H2, H1, B, S_.dh2, H2, S_.h1, H1, Ga + ao.w2, Ga + ao.b2);
    add_bwd_w(gb, H1, S, B, S_.dh1, H1, mb.s, S, Ga + ao.w1, Ga + ao.b1);
    AdamArgs ad{};
    ad.p = P + ag->off_actor;
    ad.g = Ga;
    ad.m = ag->m + ag->off_actor;
    ad.v = ag->v + ag->off_actor;
    ad.target = sac ? nullptr : T + ag->off_actor;
    ad.n = ao.size;
    ad.lr = c.lr_actor;
    ad.tau = c.tau;
    ad.cnt = (int32_t)cntr;
    ad.interval = c.actor_update_interval;
    ad.polyak_interval = sac ? 0 : c.target_actor_update;
    ad.st = ag->st;
    ad.temp = sac ? 1 : 0;
    ad.lr_temp = c.lr_temp;
    ad.temp_interval = c.temp_update_interval;
    ad.stats = stats;
    adam_copies(ag, ad, ao, SLOT_ACTOR, 1, !sac);
    RLMD_TRY(launch_bwd_w_adam(ag, gb, ad, st));
  }
  return 0;
}

float* stats_slot(rlmd_agent_s* ag, float* stats, int i) {
  return stats ? stats + 16 * (int64_t)i : ag->sc.stats;
}

int agent_learn_k(rlmd_agent_s* ag, rlmd_replay_t rb, int k, float* stats, hipStream_t st,
                  bool copies_current = false) {
  const rlmd_agent_cfg& c = ag->cfg;
  const ReplayView v = replay_view(rb);
  const int64_t mem = replay_mem_idx(rb);
  const int64_t M = mem < v.capacity ? mem : v.capacity;
  RLMD_CHECK(v.S == c.state_dim && v.A == c.action_dim, "replay / agent dims differ");
  if (k <= 0) return 0;
  const int B = c.batch, S = c.state_dim, A = c.action_dim;
  if (k > ag->kcap) {  // K mini-batches of scratch, grown on demand
    for (void* p : {(void*)ag->kb_s, (void*)ag->kb_a, (void*)ag->kb_r, (void*)ag->kb_s2, (void*)ag->kb_xsa,
                    (void*)ag->kb_done, (void*)ag->kb_idx, (void*)ag->kb_eff})
      if (p) RLMD_HIP(hipFree(p));
    const size_t KB = (size_t)k * B;
    RLMD_HIP(hipMalloc(&ag->kb_s, sizeof(float) * KB * S));
    RLMD_HIP(hipMalloc(&ag->kb_a, sizeof(float) * KB * A));
    RLMD_HIP(hipMalloc(&ag->kb_r, sizeof(float) * KB));
    RLMD_HIP(hipMalloc(&ag->kb_s2, sizeof(float) * KB * S));
    RLMD_HIP(hipMalloc(&ag->kb_xsa, sizeof(float) * KB * (S + A)));
    RLMD_HIP(hipMalloc(&ag->kb_done, KB));
    RLMD_HIP(hipMalloc(&ag->kb_idx, sizeof(int64_t) * KB));
    RLMD_HIP(hipMalloc(&ag->kb_eff, sizeof(int32_t) * KB));
    ag->kcap = k;
  }
  if (!copies_current) RLMD_TRY(refresh_copies(ag, st));
  // all K mini-batches at once: the ring does not change during the K updates;
  // batch i draws with counter learn_step_cntr + i (as K single draws would)
  const bool ms = v.n_steps > 1;
  RLMD_TRY(replay_sample_launch(v, M, B, k, c.seed ^ 0x5eed5eed5eedull, (uint64_t)ag->host_cntr, ag->kb_idx,
                                ag->kb_s, ag->kb_a, ag->kb_r, ag->kb_s2, ag->kb_done, ag->kb_xsa,
                                ms ? ag->kb_eff : nullptr, st));
  PairCtl pc{nullptr, false, false, 1};
  for (int i = 0; i < k; ++i) {
    const size_t o = (size_t)i * B;
    const Batch mb{ag->kb_s + o * S, ag->kb_r + o, ag->kb_s2 + o * S, ag->kb_xsa + o * (S + A), ag->kb_done + o,
                   ms ? ag->kb_eff + o : nullptr};
    pc.s2n = i + 1 < k ? ag->kb_s2 + (o + B) * S : nullptr;
    RLMD_TRY(learn_body(ag, mb, nullptr, nullptr, stats_slot(ag, stats, i), st, &pc));
    pc.ready = pc.paired;
  }
  return 0;
}

// copies_current: the compute copies already match the f32 masters (the fused
// training step refreshes them once at its start); otherwise the actor's copy is
// re-derived first, as the host may have written parameters since the last update.
int agent_act(rlmd_agent_s* ag, const float* obs, int64_t n, float* actions, int mode,
              uint64_t noise_ctr, const float* eps, hipStream_t st, bool copies_current = false,
              hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr) {
  const rlmd_agent_cfg& c = ag->cfg;
  if (n <= 0) return 0;
  RLMD_CHECK(n <= INT32_MAX, "too many rows");
  static const bool fused_ok = getenv("RLMD_NO_FUSED_ACT") == nullptr;
  if (fused_ok && fused_act_supported(c)) {
    if (!copies_current && ag->copies_dirty) {
      const RowNet an = row_net(ag, SLOT_ACTOR);
      const CopyJob job{an.p + ag->actor.w2, copy_wc(ag, SLOT_ACTOR), copy_wt(ag, SLOT_ACTOR)};
      RLMD_TRY(w2_copies_launch(&job, 1, row_dims(ag), st));
    }
    return fused_act_launch(c, obs, n, actions, ag->params + ag->off_actor, ag->actor,
                            static_cast<const unsigned short*>(copy_wc(ag, SLOT_ACTOR)), mode,
                            c.seed ^ 0xac7ac7ac7ull, (uint32_t)noise_ctr, eps, st, ev_start, ev_stop);
  }
  if (n > ag->act_cap) {
    if (ag->act_h1) {
      RLMD_HIP(hipFree(ag->act_h1));
      RLMD_HIP(hipFree(ag->act_h2));
    }
    RLMD_HIP(hipMalloc(&ag->act_h1, sizeof(float) * n * c.h1));
    RLMD_HIP(hipMalloc(&ag->act_h2, sizeof(float) * n * c.h2));
    ag->act_cap = n;
  }
  RLMD_CHECK(n <= INT32_MAX, "too many rows");
  if (ev_start) RLMD_HIP(hipEventRecord(ev_start, st));  // the generic path: several launches
  const float* Pa = ag->params + ag->off_actor;
  const NetOff& ao = ag->actor;
  const float* x[1] = {obs};
  const float* w1[1] = {Pa + ao.w1};
  const float* b1[1] = {Pa + ao.b1};
  float* y1[1] = {ag->act_h1};
  RLMD_TRY(fwd(ag, 1, (int)n, c.h1, c.state_dim, true, x, c.state_dim, w1, b1, y1, st));
  const float* x2[1] = {ag->act_h1};
  const float* w2[1] = {Pa + ao.w2};
  const float* b2[1] = {Pa + ao.b2};
  float* y2[1] = {ag->act_h2};
  RLMD_TRY(fwd(ag, 1, (int)n, c.h2, c.h1, true, x2, c.h1, w2, b2, y2, st));
  HeadArgs h = head_args(ag, Pa, ag->act_h2, obs, (int)n);
  h.actions = actions;
  h.mode = mode;
  h.eps_in = eps;
  h.tag = RLMD_TAG_ACT_NOISE;
  h.ctr_host = (uint32_t)noise_ctr;
  h.seed = c.seed ^ 0xac7ac7ac7ull;
  if (c.algo == RLMD_TD3) {
    h.noise_std = c.policy_noise;
    h.clamp_noise = 0;
  }
  RLMD_TRY(launch_head(h, st));
  if (ev_stop) RLMD_HIP(hipEventRecord(ev_stop, st));
  return 0;
}

}  // namespace
}  // namespace rlmd

extern "C" {

int rlmd_agent_layout(const rlmd_agent_cfg* c, int64_t* n, int64_t* oa, int64_t* o1, int64_t* o2) {
  RLMD_CHECK(c, "null cfg");
  const rlmd::NetOff a = rlmd::make_net(c->state_dim, c->h1, c->h2, c->action_dim, c->algo == RLMD_SAC);
  const rlmd::NetOff q = rlmd::make_net(c->state_dim + c->action_dim, c->h1, c->h2, 1, false);
  if (oa) *oa = 0;
  if (o1) *o1 = a.size;
  if (o2) *o2 = a.size + q.size;
  if (n) *n = a.size + 2 * q.size;
  return 0;
}

int rlmd_agent_create(const rlmd_agent_cfg* cfg, float* params, float* target, float* grads,
                      float* m, float* v, rlmd_agent_t* out) {
  RLMD_CHECK(cfg && params && target && grads && m && v && out, "null argument");
  const rlmd_agent_cfg& c = *cfg;
  RLMD_CHECK(c.algo == RLMD_SAC || c.algo == RLMD_TD3, "bad algo");
  RLMD_CHECK(c.batch >= 2 && c.batch <= RLMD_MAX_BATCH, "mini-batch must be in [2, 1024]");
  RLMD_CHECK(c.topk >= 1, "topk must be >= 1");
  RLMD_CHECK(c.action_dim >= 1 && c.action_dim <= RLMD_MAX_ACTION, "action dim out of range");
  RLMD_CHECK(c.precision == RLMD_FP32 || c.precision == RLMD_BF16, "bad precision");
  RLMD_CHECK(c.loss_type >= RLMD_LOSS_MSE && c.loss_type <= RLMD_LOSS_MSE6, "bad loss type");
  RLMD_CHECK(c.actor_update_interval >= 1 && c.target_critic_update >= 1 && c.temp_update_interval >= 1 &&
                 c.target_actor_update >= 1,
             "update intervals must be >= 1");
  auto* ag = new rlmd_agent_s();
  ag->cfg = c;
  ag->params = params;
  ag->target = target;
  ag->grads = grads;
  ag->m = m;
  ag->v = v;
  ag->actor = rlmd::make_net(c.state_dim, c.h1, c.h2, c.action_dim, c.algo == RLMD_SAC);
  ag->critic = rlmd::make_net(c.state_dim + c.action_dim, c.h1, c.h2, 1, false);
  rlmd_agent_layout(cfg, &ag->n_params, &ag->off_actor, &ag->off_c[0], &ag->off_c[1]);
  const int B = c.batch, S = c.state_dim, A = c.action_dim, X = S + A, H1 = c.h1, H2 = c.h2;
  rlmd::Scratch& s = ag->sc;
  RLMD_ALLOC(s.s, B * S);
  RLMD_ALLOC(s.a, B * A);
  RLMD_ALLOC(s.r, B);
  RLMD_ALLOC(s.s2, B * S);
  RLMD_ALLOC(s.xsa, B * X);
  RLMD_ALLOC(s.done, B);
  RLMD_ALLOC(s.logp_next, B);
  RLMD_ALLOC(s.y, B);
  RLMD_ALLOC(s.h1, B * H1);
  RLMD_ALLOC(s.h2, B * H2);
  {
    const size_t nrb = (size_t)(B + 15) / 16, m1b = nrb * rlmd::pad32(H1) * 16, m2b = nrb * rlmd::pad32(H2) * 16;
    RLMD_ALLOC(s.am1, m1b);
    RLMD_ALLOC(s.am2, m2b);
    for (int g = 0; g < 2; ++g) {
      RLMD_ALLOC(s.cm1[g], m1b);
      RLMD_ALLOC(s.cm2[g], m2b);
      RLMD_ALLOC(s.em1[g], m1b);
      RLMD_ALLOC(s.em2[g], m2b);
    }
  }
  RLMD_ALLOC(s.logp, B);
  RLMD_ALLOC(s.xsan, B * X);
  RLMD_ALLOC(s.save, B * 5 * A);
  RLMD_ALLOC(s.dlogp, B);
  RLMD_ALLOC(s.gh, B * 2 * A);
  RLMD_ALLOC(s.dh2, B * H2);
  RLMD_ALLOC(s.dh1, B * H1);
  RLMD_ALLOC(s.stats, 16);
  RLMD_ALLOC(s.qbias, 4);
  {
    const size_t nrb = (size_t)(B + 15) / 16, ts = c.precision == RLMD_BF16 ? 2 : 4;
    const size_t e1 = nrb * rlmd::pad32(H1) * 16, e2 = nrb * rlmd::pad32(H2) * 16;
    for (int g = 0; g < 2; ++g) {
      RLMD_ALLOC(s.hp1[g], e1 * ts);
      RLMD_ALLOC(s.hp2[g], e2 * ts);
      RLMD_ALLOC(s.u1[g], 2 * e1);  // two partial halves (fwd_rows column split)
      RLMD_ALLOC(s.w3s[g], H2);
    }
    const char* tp = getenv("RLMD_TARGET_PAIR");  // default on; RLMD_TARGET_PAIR=0 turns it off
    ag->target_pair = !(tp && atoi(tp) == 0);
    const char* nf = getenv("RLMD_NO_FUSED_UPDATE");
    ag->fused_update = B <= 512 && X <= 8 && !(nf && atoi(nf) != 0);
    const char* na = getenv("RLMD_NO_FUSED_ACTOR");
    ag->fused_actor = ag->fused_update && A <= 2 && !(na && atoi(na) != 0);
    const int nh = c.algo == RLMD_SAC ? 2 * A : A;
    RLMD_ALLOC(s.hp1a, e1 * ts);
    RLMD_ALLOC(s.hp2a, e2 * ts);
    // two halves of the partial bases, dq/da and q (qeval_rows column split)
    RLMD_ALLOC(s.ua, 2 * e1 * nh);
    RLMD_ALLOC(s.wheads, nh * H2);
    for (int g = 0; g < 2; ++g) RLMD_ALLOC(s.dqda[g], 2 * B * A);
    {
      int dev = 0, ncu = 0;
      if (hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0)
        ag->n_cu = ncu;
      const char* qs = getenv("RLMD_QSPLIT");
      ag->qsplit_max = qs ? std::max(1, std::min(2, atoi(qs))) : 2;
      const char* fs = getenv("RLMD_FSPLIT");
      ag->fsplit_max = fs ? std::max(1, std::min(2, atoi(fs))) : 2;
    }
    RLMD_ALLOC(s.rank1, B);
  }
  {  // weight-gradient tiles of the larger phase (critics: both nets; actor)
    using rlmd::bwd_w_tiles;
    const int tc = 2 * (bwd_w_tiles(1, H2) + bwd_w_tiles(H2, H1) + bwd_w_tiles(H1, X));
    const int ta = 2 * bwd_w_tiles(A, H2) + bwd_w_tiles(H2, H1) + bwd_w_tiles(H1, S);
    ag->max_tiles = tc > ta ? tc : ta;
    RLMD_ALLOC(ag->slabs, (size_t)ag->max_tiles * RLMD_GRAD_SPLITS * 256);
    RLMD_ALLOC(ag->tile_ctr, ag->max_tiles);
    RLMD_HIP(hipMemset(ag->tile_ctr, 0, sizeof(unsigned) * ag->max_tiles));
    const char* fz = getenv("RLMD_FUSE_ADAM");
    ag->fuse_adam = fz && atoi(fz) != 0;
    const char* fs = getenv("RLMD_FUSE_SPLITS");  // splits of the fused GEMM (1..RLMD_GRAD_SPLITS)
    ag->fuse_splits = fs ? std::max(1, std::min(RLMD_GRAD_SPLITS, atoi(fs))) : RLMD_GRAD_SPLITS;
  }
  for (int g = 0; g < 2; ++g) {
    RLMD_ALLOC(s.tpart[g], 2 * B);
    RLMD_ALLOC(s.tpartn[g], 2 * B);
    RLMD_ALLOC(s.c1[g], B * H1);
    RLMD_ALLOC(s.c2[g], B * H2);
    RLMD_ALLOC(s.qpart[g], 2 * B);
    RLMD_ALLOC(s.dq[g], B);
    RLMD_ALLOC(s.dc2[g], B * H2);
    RLMD_ALLOC(s.dc1[g], B * H1);
    RLMD_ALLOC(s.e1[g], B * H1);
    RLMD_ALLOC(s.e2[g], B * H2);
    RLMD_ALLOC(s.qnpart[g], 2 * B);
    RLMD_ALLOC(s.dqn[g], B);
  }
  ag->wcopy_bytes = (size_t)rlmd::pad32(H1) * rlmd::pad32(H2) * (c.precision == RLMD_BF16 ? 2 : 4);
  RLMD_ALLOC(ag->wcopy, 12 * ag->wcopy_bytes);
  RLMD_HIP(hipMemset(ag->wcopy, 0, 12 * ag->wcopy_bytes));
  // Zipf-plot x axis (algo_sac.py:157-162): x_j = log((1 + k) / j), centred
  const int k = c.topk;
  std::vector<float> zx(k);
  for (int j = 0; j < k; ++j) zx[j] = logf((1.0f + (float)k) / (float)(j + 1));
  double mean = 0.0;
  for (int j = 0; j < k; ++j) mean += zx[j];
  const float meanf = (float)(mean / k);
  double x2 = 0.0;
  for (int j = 0; j < k; ++j) {
    zx[j] -= meanf;
    x2 += (double)zx[j] * zx[j];
  }
  ag->zipf_x2 = (float)x2;
  RLMD_ALLOC(ag->zipf_x, k);
  RLMD_HIP(hipMemcpy(ag->zipf_x, zx.data(), sizeof(float) * k, hipMemcpyHostToDevice));
  RLMD_ALLOC(ag->st, 1);
  rlmd::LearnState st{};
  st.cauchy[0][0] = st.cauchy[0][1] = st.cauchy[1][0] = st.cauchy[1][1] = c.cauchy_scale;
  st.log_alpha[0] = st.log_alpha[1] = c.initial_logtemp;
  RLMD_HIP(hipMemcpy(ag->st, &st, sizeof(st), hipMemcpyHostToDevice));
  RLMD_HIP(hipMemset(m, 0, sizeof(float) * ag->n_params));
  RLMD_HIP(hipMemset(v, 0, sizeof(float) * ag->n_params));
  RLMD_HIP(hipMemset(grads, 0, sizeof(float) * ag->n_params * RLMD_GRAD_SPLITS));
  RLMD_HIP(hipDeviceSynchronize());
  *out = ag;
  return 0;
}

int rlmd_agent_destroy(rlmd_agent_t ag) {
  if (!ag) return 0;
  for (void* p : ag->allocs) (void)hipFree(p);
  if (ag->act_h1) (void)hipFree(ag->act_h1);
  if (ag->act_h2) (void)hipFree(ag->act_h2);
  for (void* p : {(void*)ag->kb_s, (void*)ag->kb_a, (void*)ag->kb_r, (void*)ag->kb_s2, (void*)ag->kb_xsa,
                  (void*)ag->kb_done, (void*)ag->kb_idx, (void*)ag->kb_eff})
    if (p) (void)hipFree(p);
  delete ag;
  return 0;
}

int rlmd_eval_market(rlmd_env_t env, rlmd_agent_t ag, const int32_t* start_dev, int64_t cum_step,
                     int32_t warmup_steps, int32_t smoothing_window, float* obs_dev, float* actions_dev,
                     uint8_t* live_dev, double* reward_dev, int32_t* steps_dev, double* risk_dev, void* stream) {
  RLMD_CHECK(env && ag && start_dev && obs_dev && actions_dev && live_dev && reward_dev && steps_dev,
             "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int N = rlmd::env_lanes(env);
  RLMD_CHECK(ag->cfg.state_dim == rlmd::env_state_dim(env) && ag->cfg.action_dim == rlmd::env_action_dim(env),
             "agent / env dims differ");
  // eval_episodes.py:499-507: action_window while cum_steps <= smoothing_window,
  // which clips only past the warm-up (utils.py:366-371)
  const bool window = cum_step <= smoothing_window && cum_step > warmup_steps;
  double lo = -INFINITY, hi = INFINITY;
  if (window) {
    const double width = (sin(M_PI * ((double)cum_step / (double)smoothing_window - 0.5)) + 1.0) / 2.0;
    lo = width * -0.99;
    hi = width * 0.99;
  }
  RLMD_TRY(rlmd::env_market_eval_reset(env, start_dev, obs_dev, reward_dev, steps_dev, live_dev, st));
  const int T = rlmd::env_episode_steps(env);
  RLMD_TRY(rlmd::refresh_copies(ag, st));
  if (rlmd::fused_act_supported(ag->cfg)) {  // the whole test slice in one launch
    int h1p = 0, nb = 0;
    rlmd::actrows::fused_shape(ag->cfg, h1p, nb);
    const rlmd::FusedActArgs fa =
        rlmd::fused_act_args(ag->cfg, obs_dev, N, actions_dev, ag->params + ag->off_actor, ag->actor,
                             (const unsigned short*)rlmd::copy_wc(ag, rlmd::SLOT_ACTOR), 1, 0, 0, nullptr);
    bool launched = false;
    RLMD_TRY(rlmd::env_act_market_eval(env, fa, h1p, nb, T, window ? 1 : 0, lo, hi, obs_dev, reward_dev, steps_dev,
                                       risk_dev, live_dev, st, &launched));
    if (launched) return 0;
  }
  for (int t = 0; t < T; ++t) {
    RLMD_TRY(rlmd::agent_act(ag, obs_dev, N, actions_dev, 1, 0, nullptr, st, true));  // eval_next_action
    RLMD_TRY(rlmd::env_market_eval_step(env, actions_dev, window ? 1 : 0, lo, hi, obs_dev, reward_dev, steps_dev,
                                        risk_dev, live_dev, st));
  }
  return 0;
}

int rlmd_agent_act(rlmd_agent_t ag, const float* obs, int64_t n, float* actions, int32_t mode,
                   uint64_t noise_ctr, const float* eps, void* stream) {
  RLMD_CHECK(ag && obs && actions, "null argument");
  RLMD_CHECK(mode == 0 || mode == 1, "mode must be 0 (stochastic) or 1 (deterministic)");
  // with rlmd_profile_enable, the fused acting kernel's own begin / end land in phase 0
  hipEvent_t e0, e1;
  RLMD_TRY(ag->prof.pair(0, &e0, &e1));
  return rlmd::agent_act(ag, obs, n, actions, mode, noise_ctr, eps, (hipStream_t)stream, false, e0, e1);
}

int rlmd_agent_learn(rlmd_agent_t ag, rlmd_replay_t rb, int32_t k, float* stats, void* stream) {
  RLMD_CHECK(ag && rb, "null argument");
  return rlmd::agent_learn_k(ag, rb, k, stats, (hipStream_t)stream);
}

int rlmd_agent_learn_batch(rlmd_agent_t ag, const float* s, const float* a, const float* r,
                           const float* s2, const uint8_t* done, const int32_t* eff,
                           const float* eps_a, const float* eps_b, float* stats, void* stream) {
  RLMD_CHECK(ag && s && a && r && s2 && done, "null argument");
  const rlmd_agent_cfg& c = ag->cfg;
  hipStream_t st = (hipStream_t)stream;
  rlmd::Scratch& S_ = ag->sc;
  const int B = c.batch, S = c.state_dim, A = c.action_dim;
  RLMD_HIP(hipMemcpyAsync(S_.s, s, sizeof(float) * B * S, hipMemcpyDeviceToDevice, st));
  RLMD_HIP(hipMemcpyAsync(S_.s2, s2, sizeof(float) * B * S, hipMemcpyDeviceToDevice, st));
  RLMD_HIP(hipMemcpyAsync(S_.r, r, sizeof(float) * B, hipMemcpyDeviceToDevice, st));
  RLMD_HIP(hipMemcpyAsync(S_.done, done, B, hipMemcpyDeviceToDevice, st));
  RLMD_HIP(hipMemcpy2DAsync(S_.xsa, sizeof(float) * (S + A), s, sizeof(float) * S, sizeof(float) * S,
                            B, hipMemcpyDeviceToDevice, st));
  RLMD_HIP(hipMemcpy2DAsync(S_.xsa + S, sizeof(float) * (S + A), a, sizeof(float) * A,
                            sizeof(float) * A, B, hipMemcpyDeviceToDevice, st));
  RLMD_TRY(rlmd::refresh_copies(ag, st));
  const rlmd::Batch mb{S_.s, S_.r, S_.s2, S_.xsa, S_.done, eff};
  return rlmd::learn_body(ag, mb, eps_a, eps_b, rlmd::stats_slot(ag, stats, 0), st);
}

#ifdef RLMD_TIMING
int rlmd_debug_ts(unsigned long long* out) {
  RLMD_HIP(hipDeviceSynchronize());
  RLMD_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(rlmd::g_ts), sizeof(unsigned long long) * 64));
  return 0;
}
#endif

int rlmd_agent_params_written(rlmd_agent_t ag) {
  RLMD_CHECK(ag, "null agent");
  ag->copies_dirty = true;
  return 0;
}

int rlmd_agent_scalars(rlmd_agent_t ag, double* out) {
  RLMD_CHECK(ag && out, "null argument");
  rlmd::LearnState st;
  RLMD_HIP(hipDeviceSynchronize());
  RLMD_HIP(hipMemcpy(&st, ag->st, sizeof(st), hipMemcpyDeviceToHost));
  const int s = rlmd::slot_wr(st.learn_cntr);  // the last update's values (both slots start equal)
  out[0] = st.cauchy[s][0];
  out[1] = st.cauchy[s][1];
  out[2] = st.log_alpha[s];
  out[3] = st.learn_cntr;
  out[4] = st.nan_flag;
  return 0;
}

int rlmd_status_poll(rlmd_agent_t ag, int32_t* flags_host, int32_t* nan_update_host, void* stream) {
  RLMD_CHECK(ag && flags_host, "null argument");
  hipStream_t s = (hipStream_t)stream;
  int32_t v[2];
  static_assert(offsetof(rlmd::LearnState, nan_update) == offsetof(rlmd::LearnState, nan_flag) + 8,
                "LearnState layout");
  RLMD_HIP(hipMemcpyAsync(&v[0], &ag->st->nan_flag, 4, hipMemcpyDeviceToHost, s));
  RLMD_HIP(hipMemcpyAsync(&v[1], &ag->st->nan_update, 4, hipMemcpyDeviceToHost, s));
  RLMD_HIP(hipStreamSynchronize(s));
  *flags_host = v[0];
  if (nan_update_host) *nan_update_host = v[0] ? v[1] : -1;
  return 0;
}


int rlmd_profile_enable(rlmd_agent_t ag, int32_t on) {
  RLMD_CHECK(ag, "null agent");
  RLMD_HIP(hipDeviceSynchronize());
  rlmd::PhaseProfiler& pr = ag->prof;
  pr.enabled = on != 0;
  // 2: only the events attached to the env kernel's own dispatch (phase 1): the
  // phase markers around acting / learning cost the stream ~25 us per C2 step.
  // 3: kernel-attached pairs on the env kernel and the unfused acting kernel
  pr.mask = on == 2 ? 2 : on == 3 ? 3 : 7;
  pr.kernel_pairs = on == 3;
  for (int p = 0; p < 3; ++p) {
    pr.used[p] = 0;
    pr.seen[p] = 0;
    pr.skip[p] = false;
  }
  return 0;
}

int rlmd_profile_stride(rlmd_agent_t ag, int32_t stride) {
  RLMD_CHECK(ag && stride >= 1, "bad profile stride");
  ag->prof.stride = stride;
  return 0;
}

int rlmd_profile_samples(rlmd_agent_t ag, int32_t phase, double* ms_out, int64_t cap, int64_t* count_out) {
  RLMD_CHECK(ag && count_out && phase >= 0 && phase < 3 && (cap == 0 || ms_out), "bad argument");
  RLMD_HIP(hipDeviceSynchronize());
  const rlmd::PhaseProfiler& pr = ag->prof;
  const int64_t n = (int64_t)pr.used[phase];
  for (int64_t i = 0; i < n && i < cap; ++i) {
    float ms = 0.f;
    RLMD_HIP(hipEventElapsedTime(&ms, pr.ev[phase][0][i], pr.ev[phase][1][i]));
    ms_out[i] = ms;
  }
  *count_out = n;
  return 0;
}

int rlmd_agent_set_cu_budget(rlmd_agent_t ag, int32_t n_cu) {
  RLMD_CHECK(ag && n_cu >= 1, "bad CU budget");
  ag->n_cu = n_cu;
  return 0;
}

int rlmd_profile_read(rlmd_agent_t ag, double* ms_out3, int64_t* count_out3) {
  RLMD_CHECK(ag && ms_out3 && count_out3, "null argument");
  RLMD_HIP(hipDeviceSynchronize());
  const rlmd::PhaseProfiler& pr = ag->prof;
  for (int p = 0; p < 3; ++p) {
    double tot = 0.0;
    for (size_t i = 0; i < pr.used[p]; ++i) {
      float ms = 0.f;
      RLMD_HIP(hipEventElapsedTime(&ms, pr.ev[p][0][i], pr.ev[p][1][i]));
      tot += ms;
    }
    ms_out3[p] = tot;
    count_out3[p] = (int64_t)pr.used[p];
  }
  return 0;
}

int rlmd_train_step(rlmd_env_t env, rlmd_replay_t rb, rlmd_agent_t ag, const rlmd_train_cfg* cfg,
                    float* obs, float* actions, double* ep_stats, float* stats, void* stream) {
  RLMD_CHECK(env && rb && cfg && obs && actions, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int N = rlmd::env_lanes(env);
  const rlmd::ReplayView v = rlmd::replay_view(rb);
  RLMD_CHECK(v.n_steps <= 1 || (v.lanes == N && rlmd::replay_mem_idx(rb) % N == 0),
             "multi-step replay: its lane count must equal the env's lanes");
  RLMD_CHECK(v.S == rlmd::env_state_dim(env) && v.A == rlmd::env_action_dim(env),
             "replay / env dims differ");
  const int64_t cs = cfg->cum_step;
  const bool random = cs < cfg->warmup_steps;
  // action_window (tools/utils.py:345-373): only warmup < cum_step <= smoothing_window
  const bool window = cs <= cfg->smoothing_window && cs > cfg->warmup_steps;
  // post-window policy steps (the steady state): acting + env step in one launch
  // (env.hip act_env_kernel) when the env / net shapes have an instantiation
  int h1p = 0, nb = 0, sp = 0;
  rlmd::FusedActArgs fa{};
  bool fused = false;
  if (!random && !window && ag && rlmd::fused_act_supported(ag->cfg) && rlmd::env_act_fusable(env)) {
    rlmd::actrows::fused_shape(ag->cfg, h1p, nb);
    sp = ag->cfg.state_dim <= 8 ? 8 : 16;
    fused = (sp == 8 || sp == 16) && ((h1p == 256 && nb == 4) || (h1p == 416 && nb == 5));
    if (fused)
      fa = rlmd::fused_act_args(ag->cfg, obs, N, actions, ag->params + ag->off_actor, ag->actor,
                                (const unsigned short*)rlmd::copy_wc(ag, rlmd::SLOT_ACTOR), 0,
                                ag->cfg.seed ^ 0xac7ac7ac7ull, (uint32_t)cs, nullptr);
  }
  if (!random) {
    RLMD_CHECK(ag, "policy acting needs an agent");
    const bool kp = ag->prof.kernel_pairs;
    if (!kp) RLMD_TRY(ag->prof.record(0, 0, st));
    // one refresh of every compute copy serves the acting and the K updates below
    RLMD_TRY(rlmd::refresh_copies(ag, st));
    if (!fused) {
      hipEvent_t a0 = nullptr, a1 = nullptr;
      if (kp) RLMD_TRY(ag->prof.pair(0, &a0, &a1));
      RLMD_TRY(rlmd::agent_act(ag, obs, N, actions, 0, (uint64_t)cs, nullptr, st, true, a0, a1));
    }
    if (!kp) RLMD_TRY(ag->prof.record(0, 1, st));
  }
  double lo = -INFINITY, hi = INFINITY;
  if (window) {
    const double ratio = (double)cs / (double)cfg->smoothing_window;
    const double width = (sin(M_PI * (ratio - 0.5)) + 1.0) / 2.0;
    lo = width * -0.99;
    hi = width * 0.99;
  }
  const int64_t base = rlmd::replay_mem_idx(rb);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (ag) RLMD_TRY(ag->prof.pair(1, &e0, &e1));
  rlmd::env_set_last_fused(env, fused);
  if (!fused) {
    RLMD_TRY(rlmd::env_train(env, v, base, (uint32_t)cs, actions, random ? 1 : 0, cfg->abs_warmup, window ? 1 : 0,
                             lo, hi, obs, ep_stats, st, e0, e1));
  } else {
    bool launched = false;
    RLMD_TRY(rlmd::env_act_train(env, v, base, (uint32_t)cs, fa, h1p, nb, sp, obs, ep_stats, st, e0, e1,
                                 &launched));
    RLMD_CHECK(launched, "fused acting + env step: no instantiation");
  }
  rlmd::replay_advance(rb, N);
  if (ag && cfg->k_updates > 0 && rlmd::replay_mem_idx(rb) > ag->cfg.batch) {
    RLMD_TRY(ag->prof.record(2, 0, st));
    RLMD_TRY(rlmd::agent_learn_k(ag, rb, cfg->k_updates, stats, st, !random));
    RLMD_TRY(ag->prof.record(2, 1, st));
  }
  return 0;
}

}  // extern "C"
