// learn_kernels.h — device kernels of the SAC/TD3 update (see learn.hip for the
// orchestration and the reference file:line each kernel restates).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rlmd_common.h"
#include "rlmd_internal.h"

namespace rlmd {

// Device-resident learner scalars (graph-replay safe: every per-update value a
// kernel needs is read from here, never baked into kernel arguments).
//
// The two scalars an update both reads and rewrites — the Cauchy scales (its
// loss scale, then the Nagy update) and log alpha (the target / actor loss,
// then the temperature step) — are kept in two slots by update parity: update n
// (learn_step_cntr n >= 1) reads slot (n - 1) & 1 and writes slot n & 1
// (slot_rd / slot_wr below).  Workgroups of one launch may then read the value
// the update started from while another workgroup of the same launch writes the
// new one, with no ordering between them (the fused update kernels, update.hip).
// The value after update n is in slot n & 1; both slots start at the initial value.
struct LearnState {
  float cauchy[2][2];  // [slot][critic] Cauchy scales (algo_sac.py:468-473, Nagy update)
  float kernel[2];  // CIM kernel sizes of the last update (algo_sac.py:419-420)
  float log_alpha[2];  // [slot] SAC log temperature (algo_sac.py:166-169)
  float temp_m, temp_v;
  int32_t learn_cntr;  // learn_step_cntr (algo_sac.py:475)
  int32_t nan_flag;    // tests/test_live_learning.py guards -> flag, no exit()
  float pad_temp_grad;  // temperature gradient handed from actor_loss to adam
  int32_t nan_update;   // learn_cntr when nan_flag was first set
};

__host__ __device__ inline int slot_rd(int cnt) { return (cnt - 1) & 1; }  // the value update cnt starts from
__host__ __device__ inline int slot_wr(int cnt) { return cnt & 1; }        // the value update cnt leaves

// Per-net parameter offsets (floats) inside a flat buffer, torch nn.Linear
// order: fc1.weight, fc1.bias, fc2.weight, fc2.bias, head(s).
struct NetOff {
  int64_t w1, b1, w2, b2, w3, b3, w4, b4;  // w4/b4: SAC log_scale head (else unused)
  int32_t in, h1, h2, out;                 // out: heads' rows (A for actor, 1 for critic)
  int64_t size;
};

// Arguments of the fused acting body (rlmd_act_rows.h, act.hip, env.hip).
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

struct HeadArgs {
  const float* h2;      // [n, H2] actor layer-2 activations
  const float* params;  // actor params base
  NetOff off;
  const float* state;   // [n, S] (copied into xsa)
  float* xsa;           // [n, S+A] critic input (nullable)
  float* actions;       // [n, A] (nullable)
  float* logp;          // [n] (nullable)
  float* save;          // [n, 5A]: mu, sigma, noise multiplier c, u, ls_raw for backward (nullable)
  const float* eps_in;  // injected eps [n, A] (nullable -> Philox)
  uint64_t seed;
  uint32_t tag;         // Philox tag for the eps draws
  const int32_t* ctr;   // device counter for Philox c1 (nullable -> ctr_host)
  uint32_t ctr_host;
  int32_t n, S, A, algo, mode;  // mode 0 stochastic, 1 deterministic (eval)
  float max_action, ls_min, ls_max, reparam_noise;
  float noise_std, noise_clip;  // TD3: policy / target smoothing noise (already x max_action)
  int32_t clamp_noise;          // TD3 target: clip noise to +-noise_clip
  int32_t dist;                 // SAC sampler, RLMD_DIST_*
};

// ---------------------------------------------------------------------------
// rows.hip: row-block kernels of the update.  Every per-row chain of learn()
// (forward of a 2-hidden-layer MLP -> heads -> policy sample -> next MLP, and the
// data-gradient backward) runs inside one 16-row workgroup: layer 1 on the VALU
// (K = state/action width is tiny), hidden layers on MFMA with the fc2 weight
// fragments read straight from a compute copy in HBM/L2, heads as LDS dot
// products.  Batch-wide reductions (losses, top-k, weight gradients) stay in
// their own kernels.
// ---------------------------------------------------------------------------
constexpr int kRowBlock = 16;

__host__ __device__ inline int pad32(int n) { return (n + 31) & ~31; }

// Compute copies of fc2.weight (wc [H2p][H1p], wt [H1p][H2p]) are stored
// fragment-major: element (row, col) of the logical [rows][ld] matrix sits in
// the 1-KB block of its MFMA B fragment (16 rows x KS columns; KS = 32 bf16 /
// 16 f32), lane-ordered (lane = row % 16 + 16 * (col % KS / EPF), EPF elements
// of 16 B per lane), blocks of one 16-row band in K order.  A wave's fragment
// load is then one contiguous KB and a band's K sweep one contiguous run, where
// the row-major copy spread each load over 16 half-used 128-B lines.
__host__ __device__ inline int64_t frag_index(int row, int col, int ld, int bf16) {
  const int KS = bf16 ? 32 : 16, EPF = KS / 4;
  const int s = col / KS, kin = col - s * KS;
  const int lane = (row & 15) + 16 * (kin / EPF);
  return ((int64_t)((row >> 4) * (ld / KS) + s) * 64 + lane) * EPF + kin % EPF;
}

// A net as the row kernels see it: f32 master parameters plus compute copies of
// fc2.weight in the MFMA operand type (bf16 or f32), zero-padded to 32:
//   wc [H2p][H1p] (= fc2.weight, forward), wt [H1p][H2p] (transposed, backward).
struct RowNet {
  const float* p;
  const void* wc;
  const void* wt;
};

struct RowDims {
  int32_t S, A, X, H1, H2, H1p, H2p, B, algo, prec;
};

struct SampleCfg {
  uint64_t seed;
  uint32_t ctr;  // Philox c1 = learn_step_cntr of this update
  float max_action, ls_min, ls_max, reparam_noise;
  int32_t dist;  // RLMD_DIST_* (rlmd_policy.h)
};

// Phase 1 of an update: y = 0 target path (policy on s2 -> sample -> both target
// critics), y = 1 + g online critic g on (s, a), y = 3 (with_actor) the policy on
// s for the actor update (its parameters do not change before the actor step).
struct FwdRowsArgs {
  RowDims d;
  NetOff ao, co;
  SampleCfg smp;
  RowNet tactor, tcrit[2];
  const float* s2;
  const float* eps_next;  // injected (nullable -> Philox)
  int32_t t_tag, t_clamp;
  float t_noise_std, t_noise_clip;
  float* qt[2];  // [B] target q without the head bias
  float* logp_next;
  RowNet crit[2];
  const float* xsa;
  float* c1[2];
  float* c2[2];
  uint8_t* cm1[2];  // ReLU masks of c1 / c2 in the backward layouts (rows.hip m1_index / m2_index)
  uint8_t* cm2[2];
  float* q[2];
  int32_t with_actor, a_mode, a_tag;
  RowNet actor;
  const float* s;
  const float* eps_cur;
  float* h1a;
  float* h2a;
  uint8_t* am1;
  uint8_t* am2;
  float* xsan;
  float* logp;
  float* save;  // [B, 5A]
  // fused critic update (update.hip) when u1[0] is set: per critic g the
  // row-packed operands of its weight-gradient tiles — h1 / h2 in the compute
  // type (hp1 / hp2), the backward basis U1 = [h1 > 0] * (([h2 > 0] * w3) W2)
  // in f32 (dh1 = dq * U1) — and snapshots of the head weights / biases the
  // update reads while other workgroups step them
  float* u1[2];
  void* hp1[2];
  void* hp2[2];
  float* w3s[2];  // [H2]
  float* bsnap;   // [4] online q bias 0 / 1, target q bias 0 / 1
  // fused actor update when hp1a is set: the policy's h1 / h2 row-packed in the
  // compute type (its masks go to am1 / am2; the bases are qeval_rows' head jobs)
  void* hp1a;
  void* hp2a;
  // TD3 target pairing (learn.hip): with npair = 1 the launch also runs the NEXT
  // update's target jobs (s2n, its noise counter ctrn, into qtn) — valid when no
  // target network changes in between; y0 = 2 when the previous launch already
  // computed this update's targets (jobs 0 / 1 skipped)
  const float* s2n;
  float* qtn[2];
  uint32_t ctrn;
  int32_t y0, npair;
};

// Critics evaluated on (s, a_new) after their update: y = g.
struct QEvalArgs {
  RowDims d;
  NetOff co;
  RowNet crit[2];
  const float* x;
  float* e1[2];  // nullable: the activations are needed only as masks
  float* e2[2];
  uint8_t* em1[2];
  uint8_t* em2[2];
  float* qn[2];
  // fused actor update: dq/da per row of each critic, [B][A] (nullable), and
  // y = nq + h (h < nab): the policy's backward basis of head h (mu rows, then
  // log-scale rows for SAC) U_h = [h1 > 0] * (([h2 > 0] W_head[h]) W2) from the
  // forward's masks am1 / am2, f32 row-packed [nh][nrb][H1p][16], and the head
  // weights' snapshot [nh][H2] the actor update reads while stepping them
  float* dqda[2];
  int32_t nq, nab;
  NetOff ao;
  RowNet actor;
  const uint8_t* am1;
  const uint8_t* am2;
  float* ua;
  float* wheads;
  int32_t split;  // column split of the critic jobs (1 or 2): grid y = nq * split + nab
};

// Critic data-gradients: y = g.  dh2 = dq w3 * [h2 > 0], dh1 = (dh2 W2) * [h1 > 0].
// Critic loss inputs (tools/critic_loss.py:26-453, algo_sac.py:413-473).  Used
// by critic_loss_kernel (learn.hip), by cbwd_rows (every row workgroup forms the
// per-row loss gradients of its rows) and by the critic-statistics workgroup of
// abwd_rows (rows.hip).
struct LossArgs {
  const float* qpart[2];  // online critics' q per row without the head bias [B]
  const float* qb[2];     // q_value.bias (online)
  const float* tpart[2];  // target critics' q per row without the head bias [B]
  const float* tb[2];     // q_value.bias (target)
  const float* r;
  const uint8_t* done;
  const int32_t* eff;
  const float* logp_next;  // SAC
  float gamma, reward_scale;
  float* dq[2];
  float* y_out;  // nullable
  const int32_t* rank_in;  // nullable: the rows' top-k selection ranks, already computed (critic update)
  const float* zipf_x;
  float zipf_x2;
  LearnState* st;
  float* stats;  // [16]
  int32_t B, k, loss_type, algo;
  float log_noise, grad_scale;
  int32_t keep_actor_slot;  // 1: leave stats[10] (actor loss) alone
  int32_t keep_logtemp_slot;  // 1: leave stats[11] (log temperature) to the temperature step
  int32_t cnt;  // learn_step_cntr of this update: LearnState slots slot_rd(cnt) / slot_wr(cnt)
  // fwd_rows' column split (1 or 2): qpart / tpart hold P partial sums at offsets
  // p * B, added in half order (and the critic step's U1 slabs likewise)
  int32_t qsplit;
};

struct CBwdArgs {
  RowDims d;
  NetOff co;
  RowNet crit[2];
  const float* dq[2];
  const uint8_t* cm1[2];
  const uint8_t* cm2[2];
  float* dc2[2];
  float* dc1[2];
  // B <= 512: the row workgroups form dq from the loss inputs themselves
  // (dq then written, not read); loss.B == 0: dq comes from critic_loss_kernel
  LossArgs loss;
  float* bias_out;  // [4] loss-time head biases (online 0/1, target 0/1) for the statistics
};

// Actor loss + data-gradients.  Row workgroups rank their own rows' objective
// v = min(q1, q2) - alpha logp (SAC, descending) / q1 (TD3, ascending) against
// all B (algo_sac.py:546-562 / algo_td3.py:507-523), form dL/dq and dL/dlogp,
// and back-propagate through nq critics, the sampling, the heads and fc2 of the
// policy.  One extra workgroup computes the loss value and the temperature
// gradient (algo_sac.py:580-587).  Outputs gh [B, 2A], dh2 [B, H2], dh1 [B, H1].
struct ABwdArgs {
  RowDims d;
  NetOff ao, co;
  SampleCfg smp;
  int32_t nq;
  RowNet crit[2];
  RowNet actor;
  const float* qn[2];  // updated critics on (s, a_new), no head bias [B]
  const float* logp;   // SAC
  const uint8_t* em1[2];
  const uint8_t* em2[2];
  const float* save;
  const uint8_t* am1;
  const uint8_t* am2;
  LearnState* st;
  float* stats;
  int32_t k, topk;
  float target_entropy;
  // B > 512: the loss comes from actor_loss_kernel (learn.hip) instead
  const float* dqn_ext[2];
  const float* dlogp_ext;
  float* gh;
  float* dh2;
  float* dh1;
  // critic statistics workgroup (stats, Cauchy scales, CIM kernel, NaN flag of
  // this update's critic loss) when cstats.B > 0
  LossArgs cstats;
};

size_t rows_lds_bytes(const RowDims& d);
int fwd_rows_launch(const FwdRowsArgs& a, hipStream_t st, int split = 1);  // split: critic column halves (gridDim.z)
int qeval_rows_launch(const QEvalArgs& a, int nq, hipStream_t st, int split = 1);  // split: gridDim.z column halves
int cbwd_rows_launch(const CBwdArgs& a, hipStream_t st);
int abwd_rows_launch(const ABwdArgs& a, hipStream_t st);
// Compute copies (wc, wt) of fc2.weight for n nets; refresh from the masters.
struct CopyJob {
  const float* w2;  // master fc2.weight [H2][H1]
  void* wc;
  void* wt;
};
int w2_copies_launch(const CopyJob* jobs, int n, const RowDims& d, hipStream_t st);

// act.hip: fused bf16 acting (obs -> actions in one launch) for the headline nets;
// w2bf = the actor's bf16 compute copy wc (fragment-major [H2p][H1p]).
bool fused_act_supported(const rlmd_agent_cfg& c);
FusedActArgs fused_act_args(const rlmd_agent_cfg& c, const float* obs, int64_t n, float* actions,
                            const float* actor_params, const NetOff& off, const unsigned short* w2bf, int mode,
                            uint64_t seed, uint32_t ctr, const float* eps);
// env.hip: acting + env step + replay insert + auto-reset in ONE launch for the
// post-window policy steps of rlmd_train_step (FusedActArgs of fused_act_args;
// h1p / nb / sp: the acting shape).  Returns 1 (nothing launched) when this env /
// net combination has no fused instantiation.
bool env_act_fusable(rlmd_env_t env);
// env.hip: rlmd_eval_market's day loop in one launch (eval_market_loop_kernel);
// *launched = false when the env / net shapes have no instantiation.
int env_act_market_eval(rlmd_env_t env, const FusedActArgs& a, int h1p, int nb, int T, int window, double lo,
                        double hi, float* obs, double* reward, int32_t* steps, double* risk, uint8_t* live,
                        hipStream_t stream, bool* launched);
int env_act_train(rlmd_env_t env, const ReplayView& rb, int64_t ring_base, uint32_t step, const FusedActArgs& a,
                  int h1p, int nb, int sp, float* obs, double* ep_stats, hipStream_t stream, hipEvent_t ev_start,
                  hipEvent_t ev_stop, bool* launched);
int fused_act_launch(const rlmd_agent_cfg& c, const float* obs, int64_t n, float* actions,
                     const float* actor_params, const NetOff& off, const unsigned short* w2bf, int mode,
                     uint64_t seed, uint32_t ctr, const float* eps, hipStream_t st, hipEvent_t ev_start = nullptr,
                     hipEvent_t ev_stop = nullptr);

}  // namespace rlmd
