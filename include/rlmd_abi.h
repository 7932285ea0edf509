/* rlmd_abi.h — C ABI of librlmd_amd.so, the MI355X (gfx950) hot path of
 * majidsina/rlmd re-designed as batched HIP kernels.
 *
 * The reference has no FFI: its boundary is a duck-typed Python interface
 * (SURVEY.md §8b).  Each entry point below replaces one reference method,
 * batched over lanes; the Python facade in rlmd_amd/ binds them with ctypes
 * (INTEGRATION.md shows the binding a maintainer would add).
 *
 * Conventions
 *   - every function returns 0 on success, non-zero on error; the message is
 *     in rlmd_last_error() (thread-local);
 *   - every pointer argument named *_dev is DEVICE memory (e.g. a torch CUDA
 *     tensor's data_ptr()); *_host is host memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); all
 *     device work is enqueued asynchronously on it;
 *   - the library owns the memory it allocates (env lane state, replay ring,
 *     learner scratch) and never frees caller memory (torch-owned params).
 */
#ifndef RLMD_ABI_H
#define RLMD_ABI_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ errors */
const char* rlmd_last_error(void);
int rlmd_device_sync(void);
/* A non-blocking HIP stream of this library's runtime (for several trainers in
 * one process, each on its own stream: rlmd_amd.trainer.SeedGroup) and its
 * release; *out receives the hipStream_t. */
int rlmd_stream_create(void** out);
int rlmd_stream_destroy(void* stream);
/* A non-blocking stream restricted to the CUs whose bits are set in
 * cu_mask[0 .. n_words) (bit i of word w: CU 32 w + i; hipExtStreamCreateWithCUMask).
 * The HIP runtime gives each CU-masked stream a hardware queue of its own instead
 * of a slot among the process's GPU_MAX_HW_QUEUES shared queues. */
int rlmd_stream_create_cu(const uint32_t* cu_mask, int32_t n_words, void** out);

/* --------------------------------------------------------------------- env */
/* families (envs/<family>_envs.py) and investors */
enum { RLMD_COIN = 0, RLMD_DICE = 1, RLMD_GBM = 2, RLMD_DICE_SH = 3, RLMD_MARKET = 4 };
enum { RLMD_INV_A = 0, RLMD_INV_B = 1, RLMD_INV_C = 2, RLMD_INV_INSURED = 3 };

typedef struct rlmd_env_s* rlmd_env_t;

typedef struct {
  int32_t family;      /* RLMD_COIN .. RLMD_MARKET */
  int32_t investor;    /* RLMD_INV_* (INSURED only with RLMD_DICE_SH) */
  int32_t n_lanes;     /* independent trajectories stepped per launch */
  int32_t n_gambles;   /* coin/dice/gbm: simultaneous gambles; market: n_assets */
  int32_t obs_days;    /* market: observed days (1 = D1 envs, >1 = Dx envs) */
  int32_t time_length; /* market: env time_length argument (train_days+obs_days-1) */
  int32_t action_days; /* market: days between actions (reference default 1) */
  int32_t shuffle_days;/* market: in-block shuffle interval (train 5, eval 3) */
  int32_t sample_days; /* market: days excluded from the start draw (rl_market.py:59) */
  int32_t slice_groups;/* market: lanes l, l' with l % G == l' % G draw the same episode
                          slices and shuffles (0 = every lane its own; a probe switch) */
  uint64_t seed;       /* Philox key for env draws */
} rlmd_env_cfg;

/* Replaces `Cls(n_gambles)` / `Cls()` / `Cls(n_assets, time_length, obs_days)`
 * (envs/<family>_envs.py __init__).  prices_host: market close prices [n_days, n_assets]
 * f64 row-major (tools/market_data/stooq_*.npy), NULL for other families. */
int rlmd_env_create(const rlmd_env_cfg* cfg, const double* prices_host, int64_t n_days,
                    rlmd_env_t* out);
int rlmd_env_destroy(rlmd_env_t env);
/* observation_space.shape[0], action_space.shape[0], risk width, draws per step */
int rlmd_env_dims(rlmd_env_t env, int32_t* state_dim, int32_t* action_dim, int32_t* risk_dim,
                  int32_t* draw_dim);

/* Replaces env.reset() (e.g. envs/gbm_envs.py:214-229; market: reset(obs) with
 * the episode slicing of scripts/rl_market.py:202-214).  Resets the lanes whose
 * lane_mask_dev byte is non-zero (NULL = all) and writes their state (f64, [N, S]). */
int rlmd_env_reset(rlmd_env_t env, const uint8_t* lane_mask_dev, double* state_dev, void* stream);

/* Replaces env.step(action) (e.g. envs/gbm_envs.py:147-212 + the *_dones of
 * tools/env_resources.py).  actions_dev f32 [N, A]; draws_dev f64 [N, D] injected
 * draws (uniforms for coin/dice/dice_sh, standard normals for gbm) or NULL for
 * Philox draws at the env's internal step counter; outputs f64 next_state [N, S],
 * reward [N], done/learn_done u8 [N, 2], risk [N, R] (nullable).  No auto-reset:
 * the caller resets finished lanes, as the reference driver does. */
int rlmd_env_step(rlmd_env_t env, const float* actions_dev, const double* draws_dev,
                  double* next_state_dev, double* reward_dev, uint8_t* done_dev, double* risk_dev,
                  void* stream);

/* The same step with FLOAT64 actions [N, A]: what the reference's env.step
 * receives inside the smoothing window (utils.action_window's np.clip with
 * np.float64 bounds promotes under NumPy 2, tools/utils.py:345-373), where every
 * action-derived quantity is float64. */
int rlmd_env_step_f64(rlmd_env_t env, const double* actions_dev, const double* draws_dev,
                      double* next_state_dev, double* reward_dev, uint8_t* done_dev, double* risk_dev,
                      void* stream);

/* Replaces the episode loop of eval_multiplicative (tools/eval_episodes.py:
 * 231-274): every lane of `env` (reset by the caller) is one evaluation episode
 * run with the constant action actions_dev f32 [N, A] (eval_next_action of the
 * reset state), after the action window when warmup_steps < cum_step <=
 * smoothing_window (float64 actions then), until done or max_steps.  Outputs the
 * last reward f64 [N], the step count i32 [N] and the last risk vector f64 [N, R]
 * (nullable).  draws_dev: injected draws f64 [N, max_steps, D] or NULL (Philox). */
int rlmd_eval_rollout(rlmd_env_t env, const float* actions_dev, int32_t max_steps, int64_t cum_step,
                      int32_t warmup_steps, int32_t smoothing_window, const double* draws_dev,
                      double* reward_dev, int32_t* steps_dev, double* risk_dev, void* stream);
/* The summary of eval_episodes.py:289-330 with NumPy's arithmetic (pairwise means,
 * std ddof 0, median_unbiased percentiles) over n <= 1024 episodes: stats_dev f64
 * [17] = l%, g% mean/med/5%/mad/std, V$ mean/med/5%/mad, steps mean/med/5%/mad/std,
 * mean stop-loss and mean retention (NaN unless InvB / InvC). */
int rlmd_eval_stats(const double* reward_dev, const int32_t* steps_dev, const double* risk_dev, int32_t n,
                    int32_t risk_dim, int32_t investor, double* stats_dev, void* stream);

/* Replaces agent_shadow_mean / shadow_means (tools/utils.py:374-400, :441-471):
 * for each of `rows` learn() statistic rows (stats_dev f32, leading dimension ld,
 * loss[11] first: mean 0-1, min 2-3, max 4-5, tail index 8-9) the power-law
 * shadow mean of critic 1 and 2 in float32, as the reference computes it on its
 * float32 loss entries (the empirical mean when the tail index is >= 1); written
 * to shadow_dev [rows, 2] with leading dimension ldo (stats_dev + 6 with ldo = ld
 * fills loss[6:8] in place, as the reference's loss[6:8] = ... does). */
int rlmd_shadow_means(const float* stats_dev, int32_t rows, int32_t ld, float low_mul, float high_mul,
                      float* shadow_dev, int32_t ldo, void* stream);

/* Replaces shadow_equiv (tools/utils.py:406-438) as tools/aggregate_data.py:
 * 441-447 applies it over arrays: out[i] = the max multiplier at which the
 * float64 shadow mean of (alpha[i], min[i], max[i], min_mul) equals mean[i],
 * solved from 1 (1 itself when alpha[i] >= 1).  All arrays f64 [n], device. */
int rlmd_shadow_equiv(const double* mean_dev, const double* alpha_dev, const double* min_dev, const double* max_dev,
                      double min_mul, int64_t n, double* out_dev, void* stream);

/* --------------------------------------------------- leverage sweeps (§8f-4) */
/* Workspace for rlmd_lev_coin_sweep: u16 up-count prefixes per 64-step chunk
 * and the up-count histogram u32 [horizon][horizon + 1]; -1 on bad sizes. */
int64_t rlmd_lev_workspace_bytes(int64_t investors, int32_t horizon);
/* Replaces coin_smart_lev (lev/lev_exp.py:128-237; lev/coin_flip.py:178-191):
 * outcomes_dev u8 [investors][ld] (1 = up; ld % 16 == 0, ld >= horizon rounded
 * up to 64; 16-byte aligned), levs_host the param_range leverages (negated
 * inside when -down_r > up_r, as the reference).  Writes data_dev f32
 * [n_lev][13][horizon - 1] (mean, mean_top, mean_adj, mad x3, std x3,
 * median x3, lev after each step t + 2) and, when non-null, data_T_dev f32
 * [n_lev][investors] (final values, the reference's sequential f32 products).
 * n_lev <= 32, horizon <= 5459.  workspace_bytes must be at least
 * rlmd_lev_workspace_bytes(investors, horizon) (checked).
 * Supported leverage domain: 1 + lev * up_r >= 0 and 1 + lev * down_r >= 0 for
 * every (sign-adjusted) leverage, i.e. both gamble factors non-negative, so a
 * value is monotone in the up-count (e.g. lev <= 2.5 at down_r = -0.4).  The
 * reference also runs leverages past that bound by sorting signed values; here
 * they are rejected (RLMD error), not approximated. */
int rlmd_lev_coin_sweep(const uint8_t* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld, int64_t top,
                        float value_0, float up_r, float down_r, const float* levs_host, int32_t n_lev,
                        void* workspace_dev, int64_t workspace_bytes, float* data_dev, float* data_T_dev,
                        void* stream);

/* Replaces dice_smart_lev (lev/lev_exp.py:586-705), dice_sh_smart_lev
 * (:1209-1332) and gbm_smart_lev (:1008-1119): per leverage, every investor's
 * f32 value times its gamble factor each step, then the step's values sorted
 * descending (top / adjusted groups) into data_dev f32 [n_lev][13][horizon - 1]
 * (mean x3, mad x3, std x3, lower median x3 of all / top / adjusted, lev) and the
 * final values into data_T_dev f32 [n_lev][investors] (nullable).
 * kind 0 (dice, dice_sh): outcomes_dev u8 [investors][ld] in {0 up, 1 down, 2 mid},
 *   table_host f32 [n_lev][3] the factors per outcome (the reference's
 *   1 + lev*r (+ (1 - lev)*r_sh) in its f32 arithmetic);
 * kind 1 (gbm): outcomes_dev f32 [investors][ld], factor expf(lev * outcome).
 * levs_host f32 [n_lev] (as the reference's lev_range, negation included);
 * workspace of rlmd_lev_sorted_workspace_bytes(investors, n_lev) bytes. */
int64_t rlmd_lev_sorted_workspace_bytes(int64_t investors, int32_t n_lev);
int rlmd_lev_sweep_sorted(int32_t kind, const void* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                          int64_t top, float value_0, const float* table_host, const float* levs_host, int32_t n_lev,
                          void* workspace, int64_t workspace_bytes, float* data_dev, float* data_T_dev,
                          void* stream);
/* Replaces coin_big_brain_lev (lev/lev_exp.py:270-452) and dice_big_brain_lev
 * (:741-932): per configuration c = (roll, stop) every investor re-levers each
 * step from its own value (coin_optimal_lev :240-267 / dice_optimal_lev
 * :704-738, f32).  outcomes_dev u8 codes [investors][ld] with rets_host3 the
 * return of each code; cfg_host f32 [n_cfg][5] = {stop * value_0, roll, the
 * initial leverage, roll > 0, stop}; data_dev f32 [n_cfg][26][horizon - 1]: value
 * statistics (rows 0-11), leverage statistics (12-23), stop, roll; the caller
 * orders configurations roll-major, as the reference's [n_roll][n_stop].
 * f64 = 0: coin (every quantity f32); 1: dice (the reference casts the outcomes
 * to float64, so values — and with roll 0 the leverages — are f64). */
int64_t rlmd_lev_brain_workspace_bytes(int64_t investors, int32_t n_cfg);
int rlmd_lev_brain(int32_t f64, const uint8_t* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                   int64_t top, float value_0, const double* rets_host3, float lev_factor, const float* cfg_host,
                   int32_t n_cfg, void* workspace, int64_t workspace_bytes, float* data_dev, void* stream);
/* Replaces the *_fixed_final_lev family (coin :56-127, dice :508-585, gbm
 * :935-1007, dice_sh :1121-1208), which reports the statistics of the values at
 * maturity only: the same inputs (coin: kind 0 with outcome 0 = down, 1 = up),
 * stats_dev f32 [n_lev][13] (the column of rlmd_lev_sweep_sorted at maturity)
 * and the final values values_dev f32 [n_lev][investors] (nullable).  The
 * values are sequential f32 products; the reference's gambles.prod(dim=1) rounds
 * in torch's reduction order. */
int rlmd_lev_final_sorted(int32_t kind, const void* outcomes_dev, int64_t investors, int32_t horizon, int64_t ld,
                          int64_t top, float value_0, const float* table_host, const float* levs_host, int32_t n_lev,
                          void* workspace, int64_t workspace_bytes, float* stats_dev, float* values_dev,
                          void* stream);

/* Lane wealth (f64 [N]) and time (i32 [N]) read back for tests/logging. */
int rlmd_env_lane_state(rlmd_env_t env, double* wealth_host, int32_t* time_host);
/* Market lanes' episode start rows (i32 [N]) read back (eval_market's
 * eval_start_idx = start_idx + step, rl_market.py:283-284). */
int rlmd_env_lane_start(rlmd_env_t env, int32_t* start_host);
/* Market envs: overwrite rows [row0, row0 + n_rows) of the env's device price
 * table (f64 [n_rows, n_assets], host memory), ordered on `stream`.  The
 * reference-API single env (Market_Inv?_D1/Dx(n_assets, time_length, obs_days):
 * reset(assets) / step(action, next_assets), envs/market_envs.py:133-223,
 * :611-703) hands each step's observation to the device this way: the step
 * kernel then reads the rows it gathers for that observation. */
int rlmd_env_write_prices(rlmd_env_t env, const double* rows_host, int64_t row0, int64_t n_rows, void* stream);

/* ------------------------------------------------------------------ replay */
typedef struct rlmd_replay_s* rlmd_replay_t;

/* Replaces tools/replay_torch.py ReplayBufferTorch.__init__ (:57-115): an
 * on-device ring of `capacity` transitions stored f32 SoA. */
int rlmd_replay_create(int64_t capacity, int32_t state_dim, int32_t action_dim,
                       rlmd_replay_t* out);
int rlmd_replay_destroy(rlmd_replay_t rb);
/* Replaces store_exp (tools/replay_torch.py:167-197): appends n transitions at
 * mem_idx % capacity; reward stored as max(r, r_abs_zero = -inf). */
int rlmd_replay_insert(rlmd_replay_t rb, int64_t n, const float* s_dev, const float* a_dev,
                       const float* r_dev, const float* s2_dev, const uint8_t* done_dev,
                       void* stream);
int rlmd_replay_mem_idx(rlmd_replay_t rb, int64_t* mem_idx);
/* Replaces the multi_steps > 1 path of tools/replay.py (ReplayBuffer
 * _episode_history :93-141 and the history sampling :176-332): `lanes`
 * independent transition streams (transition p of lane l at row
 * (p * lanes + l) % capacity), n-step returns summed (additive != 0, dynamics
 * "A") or multiplied (dynamics "M") with discount gamma.  Call before the first
 * insert; capacity must be a multiple of lanes.  n_steps <= 1 = single-step. */
int rlmd_replay_set_multistep(rlmd_replay_t rb, int32_t lanes, int32_t n_steps, int32_t additive,
                              double gamma);
/* Replaces sample_exp (tools/replay_torch.py:360-412 / tools/replay.py:334-376): B
 * DISTINCT uniform indices in [0, min(mem_idx, capacity)) drawn with
 * Philox(seed, (slot, draw_ctr, TAG, round)) and gathered; idx_dev i64 [B];
 * s/s2 f32 [B,S], a [B,A], r [B], done u8 [B], eff i32 [B] (nullable).  In
 * multi-step mode s/a/r are the history's initial state/action and n-step
 * return and eff the effective length (the target bootstraps with gamma^eff). */
int rlmd_replay_sample(rlmd_replay_t rb, int32_t batch, uint64_t seed, uint64_t draw_ctr,
                       int64_t* idx_dev, float* s_dev, float* a_dev, float* r_dev, float* s2_dev,
                       uint8_t* done_dev, int32_t* eff_dev, void* stream);
/* The gather half of sample_exp for caller-chosen rows (rows_dev i64 [n]). */
int rlmd_replay_gather(rlmd_replay_t rb, int32_t n, const int64_t* rows_dev, float* s_dev, float* a_dev,
                       float* r_dev, float* s2_dev, uint8_t* done_dev, int32_t* eff_dev, void* stream);

/* ------------------------------------------------------------------- agent */
enum { RLMD_SAC = 0, RLMD_TD3 = 1 };
/* critic losses, tools/critic_loss.py:344-453 */
enum {
  RLMD_LOSS_MSE = 0, RLMD_LOSS_HUB = 1, RLMD_LOSS_MAE = 2, RLMD_LOSS_HSC = 3, RLMD_LOSS_CAU = 4,
  RLMD_LOSS_TCAU = 5, RLMD_LOSS_CIM = 6, RLMD_LOSS_MSE2 = 7, RLMD_LOSS_MSE4 = 8, RLMD_LOSS_MSE6 = 9
};
enum { RLMD_FP32 = 0, RLMD_BF16 = 1 }; /* MLP GEMM operand precision (fp32 accumulate) */
/* SAC policy sampler, inputs["s_dist"] (algo_sac.py:207-218): "N", "L", "MVN" */
enum { RLMD_DIST_N = 0, RLMD_DIST_L = 1, RLMD_DIST_MVN = 2 };

typedef struct rlmd_agent_s* rlmd_agent_t;

typedef struct {
  int32_t algo, state_dim, action_dim, h1, h2;
  int32_t batch;       /* mini_batch_size (rl_multiplicative.py:108-113) */
  int32_t topk;        /* optimise_count = batch_size[algo] */
  int32_t loss_type;   /* RLMD_LOSS_* */
  int32_t precision;   /* RLMD_FP32 | RLMD_BF16 */
  int32_t actor_update_interval, target_critic_update, target_actor_update, temp_update_interval;
  int32_t actor_topk;  /* 1: actor percentile != 100 (sort + top-k), 0: plain mean */
  int32_t policy_dist; /* RLMD_DIST_* (SAC; ignored by TD3) */
  float gamma, tau, lr_actor, lr_critic, lr_temp, reward_scale, max_action;
  float log_scale_min, log_scale_max, reparam_noise, log_noise, cauchy_scale, initial_logtemp;
  float policy_noise, target_policy_noise, target_policy_clip; /* already x max_action */
  uint64_t seed;
} rlmd_agent_cfg;

/* Number of f32 parameters in the trainable set [actor | critic_1 | critic_2]
 * (torch nn.Linear layout, weight [out,in] then bias, per layer) and the
 * offsets of the three nets within it. */
int rlmd_agent_layout(const rlmd_agent_cfg* cfg, int64_t* n_params, int64_t* off_actor,
                      int64_t* off_critic1, int64_t* off_critic2);

/* Weight gradients are reduced over the mini-batch in RLMD_GRAD_SPLITS slabs
 * (split-K); the optimiser sums them in slab order (deterministic). */
#define RLMD_GRAD_SPLITS 4

/* Replaces Agent_sac.__init__ / Agent_td3.__init__ (algos/algo_sac.py:82-170,
 * algos/algo_td3.py:84-176).  Caller-owned device f32 buffers: params
 * (trainable) [n_params], target params [n_params] (same layout; SAC's
 * target_actor slot is unused as in the reference), grads
 * [RLMD_GRAD_SPLITS, n_params], Adam m and v [n_params]. */
int rlmd_agent_create(const rlmd_agent_cfg* cfg, float* params_dev, float* target_dev,
                      float* grads_dev, float* adam_m_dev, float* adam_v_dev, rlmd_agent_t* out);
int rlmd_agent_destroy(rlmd_agent_t ag);

/* Replaces select_next_action (mode 0, algo_sac.py:192-218 / algo_td3.py:198-223)
 * and eval_next_action (mode 1, :220-236 / :225-238), batched over n rows of
 * obs_dev f32 [n, S]; actions_dev f32 [n, A].  noise_ctr selects the Philox
 * counter of the acting noise; eps_dev (nullable) injects it instead. */
int rlmd_agent_act(rlmd_agent_t ag, const float* obs_dev, int64_t n, float* actions_dev,
                   int32_t mode, uint64_t noise_ctr, const float* eps_dev, void* stream);

/* Replaces eval_market (tools/eval_episodes.py:402-611) for n_eval = N lanes of
 * a market env built with the test slice's time_length and test_shuffle_days:
 * lane i starts at price row start_dev[i] (gap + eval_start_idx, :470-476),
 * the extract re-shuffled per lane; each step the deterministic policy acts on
 * the observation (eval_next_action), action_window applied when
 * warmup_steps < cum_step <= smoothing_window (then float64 actions, :499-507),
 * until done.  Out: last reward f64 [N], step count i32 [N], last risk f64
 * [N, R] (nullable).  Scratch: obs_dev f32 [N, S], actions_dev f32 [N, A],
 * live_dev u8 [N]. */
int rlmd_eval_market(rlmd_env_t env, rlmd_agent_t ag, const int32_t* start_dev, int64_t cum_step,
                     int32_t warmup_steps, int32_t smoothing_window, float* obs_dev, float* actions_dev,
                     uint8_t* live_dev, double* reward_dev, int32_t* steps_dev, double* risk_dev, void* stream);

/* Replaces learn() (algo_sac.py:369-595 / algo_td3.py:363-531): k_updates
 * updates, each sampling a fresh mini-batch from rb.  stats_dev (nullable) f32
 * [k_updates, 16] = loss[11] | logtemp | loss_params[4] per update. */
int rlmd_agent_learn(rlmd_agent_t ag, rlmd_replay_t rb, int32_t k_updates, float* stats_dev,
                     void* stream);

/* Parity hook: one learn() on a caller-supplied mini-batch with injected noise.
 * s/s2 f32 [B,S], a [B,A], r [B], done u8 [B], eff i32 [B] (multi-step length,
 * NULL = 1); eps_a / eps_b f32 [B,A]: SAC next / current eps, TD3 target noise
 * (eps_b unused). */
int rlmd_agent_learn_batch(rlmd_agent_t ag, const float* s_dev, const float* a_dev,
                           const float* r_dev, const float* s2_dev, const uint8_t* done_dev,
                           const int32_t* eff_dev, const float* eps_a_dev, const float* eps_b_dev,
                           float* stats_dev, void* stream);

/* Learner status word (sticky bits; the reference's NaN guards of
 * tests/test_live_learning.py become flags, never a process exit):
 *   RLMD_STATUS_NAN_BATCH  NaN in a mini-batch's q1 / q2 / critic target
 *                          (sac_critic_stability / td3_critic_stability :29-116)
 *   RLMD_STATUS_NAN_STATS  NaN in the critic statistics loss[0:6] + loss[8:10]
 *                          (critic_learning :119-255, the condition that exit()s)
 * Replaces the guard calls at scripts/rl_multiplicative.py:229-244.  Reads two
 * words on `stream` and synchronises it; nan_update_host (nullable) gets the
 * learn counter at which a flag was first set, -1 when none is. */
enum { RLMD_STATUS_NAN_BATCH = 1, RLMD_STATUS_NAN_STATS = 2 };
int rlmd_status_poll(rlmd_agent_t ag, int32_t* flags_host, int32_t* nan_update_host, void* stream);

/* Device scalars: [cauchy_1, cauchy_2, log_alpha, learn_step_cntr, nan_flag]. */
int rlmd_agent_scalars(rlmd_agent_t ag, double* out_host5);
/* The host wrote parameters (or targets) through the tensors it handed to
 * rlmd_agent_create (load_models, a state_dict copy): the next act / learn call
 * re-derives the bf16 / f32 MFMA compute copies from them.  The optimiser keeps
 * the copies current otherwise, so they are not rebuilt every step. */
int rlmd_agent_params_written(rlmd_agent_t ag);

/* ---------------------------------------------------------------- training */
/* One fused vector step of rl_multiplicative.py:190-227 over all lanes:
 * actions (random warm-up | policy), action_window clipping, env step,
 * replay insert of (s, a, max(r,-inf), s', learn_done), auto-reset of finished
 * lanes, then k_updates learn() calls.  obs_dev f32 [N, S] is the lanes'
 * current state (read and advanced in place); actions_dev f32 [N, A] scratch.
 * cum_step is the per-lane step counter of the warm-up / smoothing schedule
 * (rl_multiplicative.py:192-211).  episode_stats_dev (nullable) f64 [4]
 * accumulates {finished episodes, sum of final rewards, sum of lengths, -}
 * with one step of delay: each step's episodes are folded in by the next
 * rlmd_train_step on the same env, or by rlmd_train_flush_stats (call it before
 * reading the accumulator). */
typedef struct {
  int64_t cum_step;
  int32_t warmup_steps;    /* inputs["random"] */
  int32_t smoothing_window;/* inputs["smoothing_window"] */
  int32_t abs_warmup;      /* np.abs on warm-up samples (all but GBM, rl_multiplicative.py:196-201) */
  int32_t k_updates;
} rlmd_train_cfg;

int rlmd_train_step(rlmd_env_t env, rlmd_replay_t rb, rlmd_agent_t ag, const rlmd_train_cfg* cfg,
                    float* obs_dev, float* actions_dev, double* episode_stats_dev,
                    float* stats_dev, void* stream);

/* Fold the last rlmd_train_step's pending episode statistics into the
 * accumulator it was given (stream-ordered; no-op when nothing is pending). */
int rlmd_train_flush_stats(rlmd_env_t env, void* stream);

/* Per-episode log of rlmd_train_step (the reference's per-episode trial rows,
 * rl_multiplicative.py:275-283, :400-414): with cap_per_wave > 0 every lane that
 * finishes an episode appends one f32 row [env step counter, lane, final reward,
 * episode length, risk[R]] (4 + R floats; R from rlmd_env_dims) to its wave's
 * region of cap_per_wave rows; rows past the cap are counted, not kept.
 * cap_per_wave = 0 disables it (the default).  Synchronises the device. */
int rlmd_train_episode_log(rlmd_env_t env, int32_t cap_per_wave);
/* Move the logged rows into out_dev f32 [out_cap, 4 + R] (packed, wave order;
 * within a wave in append order, lanes ascending per step), reset the log, and
 * return the rows written (*n_out_host) and the rows appended since the last
 * drain including dropped ones (*appended_host, nullable).  Synchronises stream. */
int rlmd_train_episode_drain(rlmd_env_t env, float* out_dev, int64_t out_cap, int64_t* n_out_host,
                             int64_t* appended_host, void* stream);

/* Post-window policy steps of rlmd_train_step run acting + env step + replay
 * insert + reset as ONE kernel when the env / net shapes allow (one gamble,
 * S <= 8, A <= 2, the headline nets; RLMD_NO_FUSED_ENV=1 at env creation or
 * on = 0 here selects the separate launches).  Per env handle (one trainer per
 * handle; several trainers may share a process, each on its own stream).
 * rlmd_train_last_fused: 1 if this env's last step fused. */
int rlmd_train_set_fused(rlmd_env_t env, int32_t on);
int rlmd_train_last_fused(rlmd_env_t env);

/* What the replay row's `s` holds in rlmd_train_step (default
 * RLMD_STORE_REFERENCE).  The reference's coin / dice / GBM / market envs return
 * one self.next_state array that step() mutates in place (gbm_envs.py:125,
 * 184-186, 212; market_envs.py:111, 172-174, 202), and its loop stores `state`
 * after `state = next_state` (rl_multiplicative.py:213-245, rl_market.py:240-273),
 * so from an episode's second step on the stored state IS the post-step state
 * (s == s'); reset() returns a fresh array, so the first row holds the reset
 * state.  Dice_SH returns a fresh array per step: rows hold the pre-step state.
 * RLMD_STORE_REFERENCE reproduces this; RLMD_STORE_PRESTEP stores the true
 * pre-step state for every family (a diagnostic, not the reference).
 * rlmd_train_stored_state returns the mode in effect. */
enum { RLMD_STORE_REFERENCE = 0, RLMD_STORE_PRESTEP = 1 };
int rlmd_train_set_stored_state(rlmd_env_t env, int32_t mode);
int rlmd_train_stored_state(rlmd_env_t env);

/* Initialise obs_dev f32 [N, S] with every lane reset (episode start). */
int rlmd_train_reset(rlmd_env_t env, float* obs_dev, void* stream);

/* Live phase timing of rlmd_train_step with HIP events recorded on the step's
 * stream around its three phases (0 acting, 1 fused env kernel, 2 learn), per
 * agent handle (its train steps and rlmd_agent_act calls).
 * Phase 1 is the env kernel's own begin / end (the fused acting + env kernel
 * when the step fused); rlmd_agent_act's fused acting kernel adds its own
 * begin / end to phase 0.
 * enable(1) resets the counters and records every phase; enable(2) records
 * only phase 1 (events attached to the env kernel's dispatch, no markers on the
 * stream); enable(3) records kernel-attached pairs only: phase 1 as in (2)
 * and, in unfused train steps, phase 0 as the acting kernel's own dispatch (no
 * markers); enable(0) stops.  read() synchronises and returns the summed
 * milliseconds and the number of timed launches per phase. */
int rlmd_profile_enable(rlmd_agent_t ag, int32_t on);
int rlmd_profile_read(rlmd_agent_t ag, double* ms_out3, int64_t* count_out3);
/* The individual timed launches of one phase since rlmd_profile_enable (up to
 * cap of them, milliseconds each); *count_out = how many were timed. */
int rlmd_profile_samples(rlmd_agent_t ag, int32_t phase, double* ms_out, int64_t cap, int64_t* count_out);
/* Sample every stride-th occurrence of each phase (default 1 = every one): each
 * timed launch's event pair costs the stream a few microseconds, so a timed
 * region is sampled rather than stamped on every step.  Counting restarts at
 * rlmd_profile_enable. */
int rlmd_profile_stride(rlmd_agent_t ag, int32_t stride);
/* The compute units this agent's launches may count on (default: the device's).
 * The learner splits a critic's layer-2 columns over two workgroups only while
 * the doubled grid still fits that many CUs (one 512-thread workgroup per CU);
 * several trainers sharing a GPU (SeedGroup) each get a share, so the split is
 * not taken where the trainers' grids would queue behind each other.  It changes
 * f32 summation order, so runs compared bit for bit must use the same budget. */
int rlmd_agent_set_cu_budget(rlmd_agent_t ag, int32_t n_cu);

/* ------------------------------------------------------------- test hooks */
/* Copy ring rows (start + i) % capacity, i < n, into caller buffers (nullable). */
int rlmd_replay_read(rlmd_replay_t rb, int64_t start, int64_t n, float* s_dev, float* a_dev,
                     float* r_dev, float* s2_dev, uint8_t* done_dev, void* stream);
/* One MLP-layer GEMM (mode 0 forward y = relu?(A W^T + b), 1 input-gradient
 * C = mask(A W), 2 weight-gradient C = A^T W (+ bias_grad = colsum A)) on
 * caller buffers; the kernel the learner uses for every nn.Linear. */
int rlmd_gemm(int32_t precision, int32_t mode, int32_t M, int32_t N, int32_t K, int32_t relu,
              const float* A_dev, int32_t lda, const float* B_dev, int32_t ldb,
              const float* bias_dev, float* C_dev, int32_t ldc, const float* mask_dev,
              int32_t ldm, float* bias_grad_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RLMD_ABI_H */
