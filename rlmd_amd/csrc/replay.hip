// replay.hip — on-device replay ring + fused sample/gather for gfx950.
//
// Replaces tools/replay_torch.py (ReplayBufferTorch) / tools/replay.py:
//   store_exp   :167-197 (torch) / :143-174 (numpy): ring slot mem_idx % mem_size,
//               reward stored as max(r, r_abs_zero = -inf) == r;
//   sample_exp  :360-412 (torch randperm(max_mem)[:B]) / :334-376 (numpy
//               choice(max_mem, B, replace=False)): B DISTINCT uniform indices
//               over the filled part of the ring, then row gathers.
// Distinct indices on the GPU, two regimes (both restated in oracle/replay.py,
// so a sample is reproducible on the CPU index for index):
//   M <= 8192: a uniformly random B-subset as the B smallest of M random keys
//              (one LDS bitonic sort of (philox32 << 32 | index));
//   M >  8192: draw B candidates with Philox, redraw every slot whose index
//              already appeared at a smaller slot (found through an LDS hash
//              table whose entries keep the minimum owning slot), repeat
//              (collision rate <= B/M <= 1/8 per round).
// Multi-step mode (tools/replay.py:93-332): rows carry (position, episode,
// episode start) tags and every lane its episode bookkeeping, so the reference's
// history slicing — including its one-step-ahead slices of finished episodes and
// the episode-0 fallback of in-progress ones — is O(1) per
// sampled row; the n-step return, initial (next) state and action, and eff are
// gathered in the same kernel (restated in oracle/replay.py MultiStepRing).
#include <string.h>

#include <string>
#include <vector>

#include <stddef.h>
#include "rlmd_common.h"
#include "rlmd_internal.h"

struct rlmd_replay_s {
  rlmd::ReplayView v;
  int64_t mem_idx = 0;
};

namespace {

constexpr int kSampleThreads = RLMD_MAX_BATCH;

__device__ __forceinline__ int64_t ms_row(const rlmd::ReplayView& rb, int lane, int64_t pos) {
  return (pos * rb.lanes + lane) % rb.capacity;
}

// Gather row `row` into output slot i: single-step copies the row; multi-step
// follows MultiStepRing.gather (oracle/replay.py).
__device__ void gather_row(const rlmd::ReplayView& rb, int64_t row, int i, float* s, float* a, float* r,
                           float* s2, uint8_t* done, float* xsa, int32_t* eff) {
  const int S = rb.S, A = rb.A;
  int64_t src = row;  // row supplying the (initial) state and action
  float rew = rb.reward[row];
  int e = 1;
  if (rb.n_steps > 1) {
    const int lane = (int)(row % rb.lanes);
    const int32_t* t = rb.tag + 3 * row;
    const int32_t* ls = rb.lane + 4 * (int64_t)lane;
    const int64_t sp = t[0], j = t[1], aj = t[2], m = ls[1], d0 = ls[3];
    int64_t lo, b;
    if (j == 0) {
      lo = 0;
      b = sp;
    } else if (j < m) {
      lo = aj;
      b = rb.done[row] ? sp : sp + 1;
    } else {
      lo = 0;
      b = sp - aj + 1 < d0 ? sp - aj + 1 : d0;
    }
    e = (int)(b - lo + 1 < rb.n_steps ? b - lo + 1 : rb.n_steps);
    const int64_t f = b - e + 1;
    double acc = rb.additive ? 0.0 : 1.0;
    for (int k = 0; k < e - 1; ++k) {
      const double term = pow(rb.gamma, (double)k) * (double)rb.reward[ms_row(rb, lane, f + k)];
      acc = rb.additive ? acc + term : acc * term;
    }
    rew = (float)acc;
    src = ms_row(rb, lane, f);
    for (int k = 0; k < S; ++k) {
      const float v = rb.next_state[src * S + k];  // histories hold next states
      if (s) s[(int64_t)i * S + k] = v;
      if (xsa) xsa[(int64_t)i * (S + A) + k] = v;
    }
  } else {
    for (int k = 0; k < S; ++k) {
      const float v = rb.state[row * S + k];
      if (s) s[(int64_t)i * S + k] = v;
      if (xsa) xsa[(int64_t)i * (S + A) + k] = v;
    }
  }
  for (int k = 0; k < S; ++k)
    if (s2) s2[(int64_t)i * S + k] = rb.next_state[row * S + k];
  for (int k = 0; k < A; ++k) {
    const float v = rb.action[src * A + k];
    if (a) a[(int64_t)i * A + k] = v;
    if (xsa) xsa[(int64_t)i * (S + A) + S + k] = v;
  }
  if (r) r[i] = rew;
  if (done) done[i] = rb.done[row];
  if (eff) eff[i] = e;
}
// Single-step rows (the training loop's case): every load of the row issued
// before its first store. In gather_row's element loops each store is counted
// in vmcnt and the outputs may alias the ring as far as the compiler knows, so
// every element waited on its own scattered-row round trip (S + S + A + 2 of
// them per row). Clamped indices keep the loads branch-free; the stores are
// write-through (the next kernel reads them).
__device__ __forceinline__ void gather_row1(const rlmd::ReplayView& rb, int64_t row, int i, float* s, float* a,
                                            float* r, float* s2, uint8_t* done, float* xsa, int32_t* eff) {
  constexpr int C = 8;
  const int S = rb.S, A = rb.A, X = S + A;
  const float* st = rb.state + row * S;
  const float* ns = rb.next_state + row * S;
  const float* ac = rb.action + row * A;
  float sv[C], nv[C], av[C];
#pragma unroll
  for (int q = 0; q < C; ++q) {
    sv[q] = st[q < S ? q : S - 1];
    nv[q] = ns[q < S ? q : S - 1];
    av[q] = ac[q < A ? q : A - 1];
  }
  const float rew = rb.reward[row];
  const uint8_t dn = rb.done[row];
#pragma unroll
  for (int q = 0; q < C; ++q) {
    if (q < S) {
      if (s) rlmd_st_wt(s + (int64_t)i * S + q, sv[q]);
      if (xsa) rlmd_st_wt(xsa + (int64_t)i * X + q, sv[q]);
      if (s2) rlmd_st_wt(s2 + (int64_t)i * S + q, nv[q]);
    }
    if (q < A) {
      if (a) rlmd_st_wt(a + (int64_t)i * A + q, av[q]);
      if (xsa) rlmd_st_wt(xsa + (int64_t)i * X + S + q, av[q]);
    }
  }
  if (r) rlmd_st_wt(r + i, rew);
  if (done) rlmd_st_wt(done + i, dn);
  if (eff) rlmd_st_wt(eff + i, (int32_t)1);
  // wider rows (market Dx observations, many-action investors): the rest per chunk
  for (int k0 = C; k0 < S || k0 < A; k0 += C) {
#pragma unroll
    for (int q = 0; q < C; ++q) {
      const int k = k0 + q;
      sv[q] = st[k < S ? k : S - 1];
      nv[q] = ns[k < S ? k : S - 1];
      av[q] = ac[k < A ? k : A - 1];
    }
#pragma unroll
    for (int q = 0; q < C; ++q) {
      const int k = k0 + q;
      if (k < S) {
        if (s) rlmd_st_wt(s + (int64_t)i * S + k, sv[q]);
        if (xsa) rlmd_st_wt(xsa + (int64_t)i * X + k, sv[q]);
        if (s2) rlmd_st_wt(s2 + (int64_t)i * S + k, nv[q]);
      }
      if (k < A) {
        if (a) rlmd_st_wt(a + (int64_t)i * A + k, av[q]);
        if (xsa) rlmd_st_wt(xsa + (int64_t)i * X + S + k, av[q]);
      }
    }
  }
}

constexpr int kMaxRounds = 64;
constexpr int kSortPopulation = 8192;  // M at or below: sort-based subset

// replay_sample_kernel's explicit arguments as laid out in the kernarg segment
// (each at its natural alignment, in order): their exact byte count bounds the
// argument prefetch
struct SampleKargs {
  rlmd::ReplayView rb;
  int64_t M;
  int B, G;
  uint64_t seed;
  uint32_t ctr_lo, ctr_hi;
  int64_t* idx_out;
  float *s, *a, *r, *s2;
  uint8_t* done;
  float* xsa;
  int32_t* eff;
};

__global__ void __launch_bounds__(kSampleThreads)
    replay_sample_kernel(rlmd::ReplayView rb, int64_t M, int B, int G, uint64_t seed, uint32_t ctr_lo,
                         uint32_t ctr_hi, int64_t* idx_out, float* s, float* a,
                         float* r, float* s2, uint8_t* done, float* xsa, int32_t* eff) {
  rlmd_kernarg_prefetch<(int)(offsetof(SampleKargs, eff) + sizeof(int32_t*))>();
  __shared__ uint64_t keys[kSortPopulation];
  __shared__ int64_t cand[kSampleThreads];
  __shared__ int any_dup;
  const int i = threadIdx.x;
  // workgroups [G k, G k + G) of a K-batch launch all draw mini-batch k with
  // counter ctr + k (the same distinct set: the draw is a function of the
  // counter) and each gathers 1 / G of its rows — the gather's scattered
  // row reads spread over G CUs — into offset k
  const int part = blockIdx.x % G;
  {
    const int k = blockIdx.x / G;
    const uint64_t ctr = ((uint64_t)ctr_hi << 32 | ctr_lo) + (uint64_t)k;
    ctr_lo = (uint32_t)ctr;
    ctr_hi = (uint32_t)(ctr >> 32);
    const int S = rb.S, A = rb.A;
    if (idx_out) idx_out += (int64_t)k * B;
    if (s) s += (int64_t)k * B * S;
    if (a) a += (int64_t)k * B * A;
    if (r) r += (int64_t)k * B;
    if (s2) s2 += (int64_t)k * B * S;
    if (done) done += (int64_t)k * B;
    if (xsa) xsa += (int64_t)k * B * (S + A);
    if (eff) eff += (int64_t)k * B;
  }
  const uint32_t c2 = RLMD_TAG_REPLAY_IDX | (ctr_hi << 8);
  if (M <= kSortPopulation) {
    int npow = 1;
    while (npow < M) npow <<= 1;
    for (int e = i; e < npow; e += kSampleThreads) {
      if (e < M) {
        const rlmd_u32x4 v = rlmd_philox(seed, (uint32_t)e, ctr_lo, c2, 0xFFFFFFFFu);
        keys[e] = ((uint64_t)v.x << 32) | (uint64_t)e;
      } else {
        keys[e] = ~0ull;
      }
    }
    __syncthreads();
    for (int k = 2; k <= npow; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int e = i; e < npow; e += kSampleThreads) {
          const int exj = e ^ j;
          if (exj > e) {
            const uint64_t x = keys[e], y = keys[exj];
            const bool up = (e & k) == 0;
            if ((x > y) == up) {
              keys[e] = y;
              keys[exj] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    if (i < B) cand[i] = (int64_t)(keys[i] & 0xFFFFFFFFu);
  } else {
    // rounds of: hash every candidate into an LDS table; the smallest slot per
    // index owns it (atomicMin: order-independent); the other slots redraw
    __shared__ unsigned long long tab_key[2 * kSampleThreads];
    __shared__ int tab_own[2 * kSampleThreads];
    constexpr int H = 2 * kSampleThreads;
    if (i < B) {
      const rlmd_u32x4 v = rlmd_philox(seed, (uint32_t)i, ctr_lo, c2, 0u);
      cand[i] = (int64_t)rlmd_below(v.x, v.y, (uint64_t)M);
    }
    for (int round = 1; round <= kMaxRounds; ++round) {
      for (int e = i; e < H; e += kSampleThreads) {
        tab_key[e] = ~0ull;
        tab_own[e] = 0x7fffffff;
      }
      __syncthreads();
      int h = 0;
      const unsigned long long c = i < B ? (unsigned long long)cand[i] : 0ull;
      if (i < B) {
        h = (int)((c * 0x9E3779B97F4A7C15ull) >> 52) & (H - 1);
        for (int probe = 0; probe < H; ++probe) {
          const unsigned long long old = atomicCAS(&tab_key[h], ~0ull, c);
          if (old == ~0ull || old == c) break;
          h = (h + 1) & (H - 1);
        }
        atomicMin(&tab_own[h], i);
      }
      __syncthreads();
      const bool dup = i < B && tab_own[h] != i;
      if (dup) {
        const rlmd_u32x4 v = rlmd_philox(seed, (uint32_t)i, ctr_lo, c2, (uint32_t)round);
        cand[i] = (int64_t)rlmd_below(v.x, v.y, (uint64_t)M);
      }
      if (!__syncthreads_or(dup)) break;
    }
  }
  __syncthreads();
  const int per = (B + G - 1) / G;
  if (i >= B || i < part * per || i >= (part + 1) * per) return;
  const int64_t row = cand[i];
  if (idx_out) idx_out[i] = row;
  if (rb.n_steps > 1)
    gather_row(rb, row, i, s, a, r, s2, done, xsa, eff);
  else
    gather_row1(rb, row, i, s, a, r, s2, done, xsa, eff);
}

__global__ void replay_gather_kernel(rlmd::ReplayView rb, int n, const int64_t* rows, float* s, float* a,
                                     float* r, float* s2, uint8_t* done, int32_t* eff) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) gather_row(rb, rows[i], i, s, a, r, s2, done, nullptr, eff);
}

__global__ void replay_insert_kernel(rlmd::ReplayView rb, int64_t base, int64_t n, const float* s,
                                     const float* a, const float* r, const float* s2,
                                     const uint8_t* d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t row = (base + i) % rb.capacity;
  for (int k = 0; k < rb.S; ++k) {
    rb.state[row * rb.S + k] = s[i * rb.S + k];
    rb.next_state[row * rb.S + k] = s2[i * rb.S + k];
  }
  for (int k = 0; k < rb.A; ++k) rb.action[row * rb.A + k] = a[i * rb.A + k];
  rb.reward[row] = r[i];
  rb.done[row] = d[i];
  if (rb.n_steps > 1) rlmd::ms_record(rb, (int)((base + i) % rb.lanes), row, d[i] != 0);
}

__global__ void replay_read_kernel(rlmd::ReplayView rb, int64_t start, int64_t n, float* s, float* a,
                                   float* r, float* s2, uint8_t* d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t row = (start + i) % rb.capacity;
  for (int k = 0; k < rb.S; ++k) {
    if (s) s[i * rb.S + k] = rb.state[row * rb.S + k];
    if (s2) s2[i * rb.S + k] = rb.next_state[row * rb.S + k];
  }
  for (int k = 0; k < rb.A; ++k)
    if (a) a[i * rb.A + k] = rb.action[row * rb.A + k];
  if (r) r[i] = rb.reward[row];
  if (d) d[i] = rb.done[row];
}

}  // namespace

namespace rlmd {

ReplayView replay_view(rlmd_replay_t rb) { return rb->v; }
int64_t replay_mem_idx(rlmd_replay_t rb) { return rb->mem_idx; }
void replay_advance(rlmd_replay_t rb, int64_t n) { rb->mem_idx += n; }

int replay_sample_launch(const ReplayView& rb, int64_t M, int B, int K, uint64_t seed, uint64_t ctr,
                         int64_t* idx, float* s, float* a, float* r, float* s2, uint8_t* done, float* xsa,
                         int32_t* eff, hipStream_t stream) {
  RLMD_CHECK(B >= 1 && B <= RLMD_MAX_BATCH, "batch must be in [1, 1024]");
  RLMD_CHECK(K >= 1, "need at least one mini-batch");
  RLMD_CHECK(M >= B, "replay holds fewer transitions than the mini-batch");
  RLMD_CHECK(M <= (int64_t)1 << 52, "replay too large");
  const int G = B >= 256 ? 8 : 1;  // gather parts per mini-batch
  hipLaunchKernelGGL(replay_sample_kernel, dim3(K * G), dim3(kSampleThreads), 0, stream, rb, M, B, G, seed,
                     (uint32_t)ctr, (uint32_t)(ctr >> 32), idx, s, a, r, s2, done, xsa, eff);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace rlmd

extern "C" {

int rlmd_replay_create(int64_t capacity, int32_t S, int32_t A, rlmd_replay_t* out) {
  RLMD_CHECK(out && capacity > 0 && S > 0 && A > 0, "bad replay arguments");
  auto* rb = new rlmd_replay_s();
  rb->v.capacity = capacity;
  rb->v.S = S;
  rb->v.A = A;
  RLMD_HIP(hipMalloc(&rb->v.state, sizeof(float) * capacity * S));
  RLMD_HIP(hipMalloc(&rb->v.next_state, sizeof(float) * capacity * S));
  RLMD_HIP(hipMalloc(&rb->v.action, sizeof(float) * capacity * A));
  RLMD_HIP(hipMalloc(&rb->v.reward, sizeof(float) * capacity));
  RLMD_HIP(hipMalloc(&rb->v.done, capacity));
  rb->v.n_steps = 1;
  rb->v.lanes = 1;
  rb->v.additive = 1;
  rb->v.gamma = 0.99;
  *out = rb;
  return 0;
}

int rlmd_replay_set_multistep(rlmd_replay_t rb, int32_t lanes, int32_t n_steps, int32_t additive,
                              double gamma) {
  RLMD_CHECK(rb, "null replay");
  RLMD_CHECK(rb->mem_idx == 0, "multi-step mode must be set before the first insert");
  RLMD_CHECK(lanes >= 1 && rb->v.capacity % lanes == 0, "capacity must be a multiple of the lane count");
  RLMD_CHECK(n_steps >= 1, "multi_steps must be >= 1");
  rb->v.n_steps = n_steps;
  rb->v.lanes = lanes;
  rb->v.additive = additive ? 1 : 0;
  rb->v.gamma = gamma;
  if (n_steps > 1) {
    if (!rb->v.tag) RLMD_HIP(hipMalloc(&rb->v.tag, sizeof(int32_t) * 3 * rb->v.capacity));
    if (rb->v.lane) RLMD_HIP(hipFree(rb->v.lane));
    RLMD_HIP(hipMalloc(&rb->v.lane, sizeof(int32_t) * 4 * lanes));
    std::vector<int32_t> init(4 * (size_t)lanes, 0);
    for (int32_t l = 0; l < lanes; ++l) init[4 * l + 3] = -1;
    RLMD_HIP(hipMemcpy(rb->v.lane, init.data(), sizeof(int32_t) * init.size(), hipMemcpyHostToDevice));
  }
  return 0;
}

int rlmd_replay_destroy(rlmd_replay_t rb) {
  if (!rb) return 0;
  (void)hipFree(rb->v.state);
  (void)hipFree(rb->v.next_state);
  (void)hipFree(rb->v.action);
  (void)hipFree(rb->v.reward);
  (void)hipFree(rb->v.done);
  if (rb->v.tag) (void)hipFree(rb->v.tag);
  if (rb->v.lane) (void)hipFree(rb->v.lane);
  delete rb;
  return 0;
}

int rlmd_replay_insert(rlmd_replay_t rb, int64_t n, const float* s, const float* a, const float* r,
                       const float* s2, const uint8_t* d, void* stream) {
  RLMD_CHECK(rb && s && a && r && s2 && d, "null argument");
  if (n <= 0) return 0;
  RLMD_CHECK(rb->v.n_steps <= 1 || n <= rb->v.lanes, "multi-step insert: at most one transition per lane per call");
  hipLaunchKernelGGL(replay_insert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, rb->v, rb->mem_idx, n, s, a, r, s2, d);
  RLMD_LAUNCH_CHECK();
  rb->mem_idx += n;
  return 0;
}

int rlmd_replay_read(rlmd_replay_t rb, int64_t start, int64_t n, float* s, float* a, float* r,
                     float* s2, uint8_t* d, void* stream) {
  RLMD_CHECK(rb && start >= 0, "bad argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(replay_read_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, rb->v, start, n, s, a, r, s2, d);
  RLMD_LAUNCH_CHECK();
  return 0;
}

int rlmd_replay_mem_idx(rlmd_replay_t rb, int64_t* m) {
  RLMD_CHECK(rb && m, "null argument");
  *m = rb->mem_idx;
  return 0;
}

int rlmd_replay_sample(rlmd_replay_t rb, int32_t B, uint64_t seed, uint64_t ctr, int64_t* idx,
                       float* s, float* a, float* r, float* s2, uint8_t* done, int32_t* eff, void* stream) {
  RLMD_CHECK(rb, "null replay");
  const int64_t M = rb->mem_idx < rb->v.capacity ? rb->mem_idx : rb->v.capacity;
  return rlmd::replay_sample_launch(rb->v, M, B, 1, seed, ctr, idx, s, a, r, s2, done, nullptr, eff,
                                    (hipStream_t)stream);
}

int rlmd_replay_gather(rlmd_replay_t rb, int32_t n, const int64_t* rows, float* s, float* a, float* r,
                       float* s2, uint8_t* done, int32_t* eff, void* stream) {
  RLMD_CHECK(rb && rows, "null argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(replay_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     rb->v, n, rows, s, a, r, s2, done, eff);
  RLMD_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
