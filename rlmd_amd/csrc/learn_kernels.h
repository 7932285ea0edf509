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
struct LearnState {
  float cauchy[2];  // Cauchy scales (algo_sac.py:468-473, Nagy update)
  float kernel[2];  // CIM kernel sizes of the last update (algo_sac.py:419-420)
  float log_alpha;  // SAC log temperature (algo_sac.py:166-169)
  float temp_m, temp_v;
  int32_t learn_cntr;  // learn_step_cntr (algo_sac.py:475)
  int32_t nan_flag;    // tests/test_live_learning.py guards -> flag, no exit()
  float pad_temp_grad;  // temperature gradient handed from actor_loss to adam
};

// Per-net parameter offsets (floats) inside a flat buffer, torch nn.Linear
// order: fc1.weight, fc1.bias, fc2.weight, fc2.bias, head(s).
struct NetOff {
  int64_t w1, b1, w2, b2, w3, b3, w4, b4;  // w4/b4: SAC log_scale head (else unused)
  int32_t in, h1, h2, out;                 // out: heads' rows (A for actor, 1 for critic)
  int64_t size;
};

struct HeadArgs {
  const float* h2;      // [n, H2] actor layer-2 activations
  const float* params;  // actor params base
  NetOff off;
  const float* state;   // [n, S] (copied into xsa)
  float* xsa;           // [n, S+A] critic input (nullable)
  float* actions;       // [n, A] (nullable)
  float* logp;          // [n] (nullable)
  float* save;          // [n, 5A]: mu, sigma, eps, u, ls_raw for backward (nullable)
  const float* eps_in;  // injected eps [n, A] (nullable -> Philox)
  uint64_t seed;
  uint32_t tag;         // Philox tag for the eps draws
  const int32_t* ctr;   // device counter for Philox c1 (nullable -> ctr_host)
  uint32_t ctr_host;
  int32_t n, S, A, algo, mode;  // mode 0 stochastic, 1 deterministic (eval)
  float max_action, ls_min, ls_max, reparam_noise;
  float noise_std, noise_clip;  // TD3: policy / target smoothing noise (already x max_action)
  int32_t clamp_noise;          // TD3 target: clip noise to +-noise_clip
};

}  // namespace rlmd
