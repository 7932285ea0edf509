// rlmd_common.h — shared device/host helpers for the rlmd_amd HIP library (gfx950).
//
// Counter-based randomness: every random draw in the library is
//   Philox4x32-10(key = seed, counter = (c0, c1, c2, c3))
// with a fixed meaning per draw site (see RLMD_TAG_*), so a draw is a pure
// function of (seed, lane/row, step, site, index).  No per-lane RNG state lives
// in HBM, graph replays stay deterministic, and the CPU oracle (oracle/philox.py)
// regenerates the same bits.  The generator core is the standard Philox4x32-10
// (Salmon et al., SC'11) — the same core rocRAND's philox4x32_10 uses; the
// uniform and normal transforms below are ours and are restated in the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RLMD_TAG_ENV_DRAW 1u       // env gamble outcomes (c0 = lane, c1 = step, c3 = pair index)
#define RLMD_TAG_WARMUP_ACTION 2u  // warm-up random actions (c0 = lane, c1 = step)
#define RLMD_TAG_ACT_NOISE 3u      // acting noise (SAC eps / TD3 policy noise)
#define RLMD_TAG_REPLAY_IDX 4u     // replay sample indices (c0 = slot, c1 = update, c3 = round)
#define RLMD_TAG_EPS_NEXT 5u       // SAC eps for next-state actions in the target
#define RLMD_TAG_EPS_CUR 6u        // SAC eps for current-state actions in the actor update
#define RLMD_TAG_TD3_TARGET 7u     // TD3 target policy smoothing noise
#define RLMD_TAG_MKT_START 8u      // market episode start index (c0 = lane, c1 = episode)
#define RLMD_TAG_MKT_PERM 9u       // market in-block shuffles (c0 = lane, c1 = episode, c3 = block)

struct rlmd_u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ uint32_t rlmd_mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__host__ __device__ __forceinline__ rlmd_u32x4 rlmd_philox(uint64_t seed, uint32_t c0, uint32_t c1,
                                                           uint32_t c2, uint32_t c3) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * x0, hi0 = rlmd_mulhi32(0xD2511F53u, x0);
    const uint32_t lo1 = 0xCD9E8D57u * x2, hi1 = rlmd_mulhi32(0xCD9E8D57u, x2);
    const uint32_t n0 = hi1 ^ x1 ^ k0, n2 = hi0 ^ x3 ^ k1;
    x0 = n0;
    x1 = lo1;
    x2 = n2;
    x3 = lo0;
  }
  return {x0, x1, x2, x3};
}

// 53-bit uniform in [0, 1) from two words (NumPy's random_sample construction).
__host__ __device__ __forceinline__ double rlmd_u01(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// Box–Muller pair from one Philox block: z0 = r cos(2πu2), z1 = r sin(2πu2),
// r = sqrt(-2 ln(1 - u1)) (1 - u1 in (0, 1], so the log is finite).
__device__ __forceinline__ void rlmd_normal2(rlmd_u32x4 v, double& z0, double& z1) {
  const double u1 = rlmd_u01(v.x, v.y), u2 = rlmd_u01(v.z, v.w);
  const double r = sqrt(-2.0 * log(1.0 - u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// Uniform integer in [0, n) from one 32-bit word and a second for 64-bit range
// (multiply-shift; bias < n / 2^64, negligible).
__host__ __device__ __forceinline__ uint64_t rlmd_below(uint32_t a, uint32_t b, uint64_t n) {
  const uint64_t x = ((uint64_t)a << 32) | b;
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(x, n);
#else
  return (uint64_t)(((unsigned __int128)x * n) >> 64);
#endif
}

// ---------------------------------------------------------------------------
// Block-wide ascending bitonic sort of one u64 key per thread over the first n
// (power of two, n <= blockDim.x) threads; returns this thread's sorted key.
// Strides < 64 exchange through wave shuffles (no barrier); strides >= 64
// through `lds` (>= blockDim.x entries).  Every thread of the block must call
// it; threads >= n sort their own n-aligned segments, each ascending, so several
// independent sorts of n keys can share one call.
// ---------------------------------------------------------------------------
// DPP lane moves (VALU rate, no LDS crossbar): a 16-lane row reduction with
// quad butterflies then the half-row and row mirrors; every lane of the row
// ends with the row's result (quad [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E,
// row_half_mirror = 0x141, row_mirror = 0x140).
template <int CTRL>
__device__ __forceinline__ float rlmd_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rlmd_row16_sum(float v) {
  v += rlmd_dpp<0xB1>(v);
  v += rlmd_dpp<0x4E>(v);
  v += rlmd_dpp<0x141>(v);
  v += rlmd_dpp<0x140>(v);
  return v;
}
__device__ __forceinline__ float rlmd_row16_max(float v) {
  v = fmaxf(v, rlmd_dpp<0xB1>(v));
  v = fmaxf(v, rlmd_dpp<0x4E>(v));
  v = fmaxf(v, rlmd_dpp<0x141>(v));
  v = fmaxf(v, rlmd_dpp<0x140>(v));
  return v;
}

__device__ __forceinline__ uint64_t rlmd_shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}

// The value of lane (l ^ J) for a compile-time J, by the cheapest lane move:
// DPP for J < 16 (quad permutes [1,0,3,2] / [2,3,0,1]; J = 4 as the half-row
// mirror l ^ 7 then the quad reversal l ^ 3; J = 8 as row_ror:8), ds_swizzle's
// xor mode for J = 16 (no address VGPR), ds_bpermute only for J = 32.  A
// bitonic stage otherwise waits a bpermute round trip per 32-bit half.
template <int J>
__device__ __forceinline__ uint32_t rlmd_xor_lane(uint32_t v) {
  // every lane's source lies inside its row, so no lane keeps an old value
  // (mov_dpp: no "old" operand to initialise)
  const int x = (int)v;
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);
  else if constexpr (J == 4)
    return (uint32_t)__builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF,
                                              false);
  else if constexpr (J == 8) return (uint32_t)__builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false);
  else if constexpr (J == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle(x, 0x401F);
  else return (uint32_t)__shfl_xor(x, J, 64);
}
template <int J>
__device__ __forceinline__ uint64_t rlmd_xor_lane_u64(uint64_t v) {
  return ((uint64_t)rlmd_xor_lane<J>((uint32_t)(v >> 32)) << 32) | rlmd_xor_lane<J>((uint32_t)v);
}

// Range-checked buffer loads: an element load is always issued (no exec-masked
// branch, whose s_waitcnt vmcnt(0) would serialise a run of conditional loads);
// ok == false turns the byte offset out of range and the hardware returns 0.
//
// A buffer resource must sit in scalar registers.  Every resource here is
// wave-uniform by construction (workgroup / job / wave pointers and sizes), but
// where the compiler cannot prove it — a size chosen by a select it placed on the
// VALU, a pointer picked by the wave index — it wraps each load in a
// readfirstlane "waterfall" loop (one trip per distinct value, a dependent round
// of scalar moves, compares and exec branches around every single load).  The
// explicit readfirstlane below states the uniformity; on values already in
// scalar registers it folds to a move.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rlmd_rsrc_wave(const void* base, int bytes) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rlmd_rsrc(const void* base, int64_t bytes) {
  return rlmd_rsrc_wave(base, (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
}
__device__ __forceinline__ float rlmd_ldf(__amdgpu_buffer_rsrc_t r, int64_t idx, bool ok) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, ok ? (int)(idx * 4) : 0x7fffffff, 0, 0));
}

// Kernel-argument prefetch.  The learner kernels take structs of 0.5-1 KB by
// value; the compiler loads each field (s_load) next to its first use, behind the
// role branches, so a prologue walked ~6-9 dependent scalar round trips, each a
// miss on a fresh kernarg line (the host writes the segment per dispatch: no
// cache holds it).  One dword of every 64-byte line, loaded together at entry and
// waited for once, turns those into scalar-cache hits.  Loads only (the scalar
// cache is never written).  The loads and their wait are ONE asm statement with
// early-clobber outputs: left to the compiler they came in clauses of 8 with a
// wait after each, and split asm loads would let it reuse an output register
// while its load is still in flight.
// Line offsets are clamped to the last dword of the explicit arguments
// (LAST = BYTES - 4, rounded down to a dword): lines past the end repeat that
// dword instead of reading past the arguments, where the kernarg allocation of a
// kernel whose hidden arguments the compiler trimmed may end.
template <int NL, int LAST>
struct rlmd_karg_lines;
template <int LAST>
struct rlmd_karg_lines<4, LAST> {
  static __device__ __forceinline__ void run(const void* kp) {
  uint32_t v[4];
  __asm__ volatile("s_load_dword %0, %4, %5\n""s_load_dword %1, %4, %6\n""s_load_dword %2, %4, %7\n""s_load_dword %3, %4, %8\n"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&s"(v[0]), "=&s"(v[1]), "=&s"(v[2]), "=&s"(v[3])
                   : "s"(kp), "i"(0 < LAST ? 0 : LAST), "i"(64 < LAST ? 64 : LAST), "i"(128 < LAST ? 128 : LAST), "i"(192 < LAST ? 192 : LAST)
                   : "memory");
  }
};
template <int LAST>
struct rlmd_karg_lines<8, LAST> {
  static __device__ __forceinline__ void run(const void* kp) {
  uint32_t v[8];
  __asm__ volatile("s_load_dword %0, %8, %9\n""s_load_dword %1, %8, %10\n""s_load_dword %2, %8, %11\n""s_load_dword %3, %8, %12\n""s_load_dword %4, %8, %13\n""s_load_dword %5, %8, %14\n""s_load_dword %6, %8, %15\n""s_load_dword %7, %8, %16\n"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&s"(v[0]), "=&s"(v[1]), "=&s"(v[2]), "=&s"(v[3]), "=&s"(v[4]), "=&s"(v[5]), "=&s"(v[6]), "=&s"(v[7])
                   : "s"(kp), "i"(0 < LAST ? 0 : LAST), "i"(64 < LAST ? 64 : LAST), "i"(128 < LAST ? 128 : LAST), "i"(192 < LAST ? 192 : LAST), "i"(256 < LAST ? 256 : LAST), "i"(320 < LAST ? 320 : LAST), "i"(384 < LAST ? 384 : LAST), "i"(448 < LAST ? 448 : LAST)
                   : "memory");
  }
};
template <int LAST>
struct rlmd_karg_lines<12, LAST> {
  static __device__ __forceinline__ void run(const void* kp) {
  uint32_t v[12];
  __asm__ volatile("s_load_dword %0, %12, %13\n""s_load_dword %1, %12, %14\n""s_load_dword %2, %12, %15\n""s_load_dword %3, %12, %16\n""s_load_dword %4, %12, %17\n""s_load_dword %5, %12, %18\n""s_load_dword %6, %12, %19\n""s_load_dword %7, %12, %20\n""s_load_dword %8, %12, %21\n""s_load_dword %9, %12, %22\n""s_load_dword %10, %12, %23\n""s_load_dword %11, %12, %24\n"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&s"(v[0]), "=&s"(v[1]), "=&s"(v[2]), "=&s"(v[3]), "=&s"(v[4]), "=&s"(v[5]), "=&s"(v[6]), "=&s"(v[7]), "=&s"(v[8]), "=&s"(v[9]), "=&s"(v[10]), "=&s"(v[11])
                   : "s"(kp), "i"(0 < LAST ? 0 : LAST), "i"(64 < LAST ? 64 : LAST), "i"(128 < LAST ? 128 : LAST), "i"(192 < LAST ? 192 : LAST), "i"(256 < LAST ? 256 : LAST), "i"(320 < LAST ? 320 : LAST), "i"(384 < LAST ? 384 : LAST), "i"(448 < LAST ? 448 : LAST), "i"(512 < LAST ? 512 : LAST), "i"(576 < LAST ? 576 : LAST), "i"(640 < LAST ? 640 : LAST), "i"(704 < LAST ? 704 : LAST)
                   : "memory");
  }
};
template <int LAST>
struct rlmd_karg_lines<16, LAST> {
  static __device__ __forceinline__ void run(const void* kp) {
  uint32_t v[16];
  __asm__ volatile("s_load_dword %0, %16, %17\n""s_load_dword %1, %16, %18\n""s_load_dword %2, %16, %19\n""s_load_dword %3, %16, %20\n""s_load_dword %4, %16, %21\n""s_load_dword %5, %16, %22\n""s_load_dword %6, %16, %23\n""s_load_dword %7, %16, %24\n""s_load_dword %8, %16, %25\n""s_load_dword %9, %16, %26\n""s_load_dword %10, %16, %27\n""s_load_dword %11, %16, %28\n""s_load_dword %12, %16, %29\n""s_load_dword %13, %16, %30\n""s_load_dword %14, %16, %31\n""s_load_dword %15, %16, %32\n"
                   "s_waitcnt lgkmcnt(0)"
                   : "=&s"(v[0]), "=&s"(v[1]), "=&s"(v[2]), "=&s"(v[3]), "=&s"(v[4]), "=&s"(v[5]), "=&s"(v[6]), "=&s"(v[7]), "=&s"(v[8]), "=&s"(v[9]), "=&s"(v[10]), "=&s"(v[11]), "=&s"(v[12]), "=&s"(v[13]), "=&s"(v[14]), "=&s"(v[15])
                   : "s"(kp), "i"(0 < LAST ? 0 : LAST), "i"(64 < LAST ? 64 : LAST), "i"(128 < LAST ? 128 : LAST), "i"(192 < LAST ? 192 : LAST), "i"(256 < LAST ? 256 : LAST), "i"(320 < LAST ? 320 : LAST), "i"(384 < LAST ? 384 : LAST), "i"(448 < LAST ? 448 : LAST), "i"(512 < LAST ? 512 : LAST), "i"(576 < LAST ? 576 : LAST), "i"(640 < LAST ? 640 : LAST), "i"(704 < LAST ? 704 : LAST), "i"(768 < LAST ? 768 : LAST), "i"(832 < LAST ? 832 : LAST), "i"(896 < LAST ? 896 : LAST), "i"(960 < LAST ? 960 : LAST)
                   : "memory");
  }
};
template <int BYTES>
__device__ __forceinline__ void rlmd_kernarg_prefetch() {
  // lines of the explicit arguments, rounded up to a multiple of 4 (<= 16: 1 KB)
  constexpr int nl = (BYTES + 63) / 64, n4 = ((nl + 3) / 4) * 4;
  static_assert(n4 <= 16, "kernel arguments above 1 KB");
  static_assert(BYTES >= 4, "kernel arguments below one dword");
  rlmd_karg_lines<n4, ((BYTES - 4) / 4) * 4>::run((const void*)__builtin_amdgcn_kernarg_segment_ptr());
}
#ifndef RLMD_KARG_PF
#define RLMD_KARG_PF 1
#endif
#if RLMD_KARG_PF
#define RLMD_KERNARG_PREFETCH(args) rlmd_kernarg_prefetch<(int)sizeof(args)>()
#else
#define RLMD_KERNARG_PREFETCH(args) \
  do {                              \
  } while (0)
#endif

// Write-through stores for data the next kernel reads (optimiser state, compute
// copies, row-packed activations, bases): a device-scope store (sc1) sends each
// line on to memory as it is written, instead of leaving it dirty in the XCD's
// L2 for the release at the end of the kernel, which writes every dirty line
// back after the last workgroup has finished (≈1 µs per MB at the update
// kernels' sizes, on the critical path of every launch).
#ifndef RLMD_WT_STORES
#define RLMD_WT_STORES 1
#endif
#if RLMD_WT_STORES
#define RLMD_WT_AUX 16  // buffer-store cache policy: sc1 (device scope)
#else
#define RLMD_WT_AUX 0
#endif
template <class T>
__device__ __forceinline__ void rlmd_st_wt(T* p, T v) {
#if RLMD_WT_STORES
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = v;
#endif
}
// 16 bytes (16-byte aligned) as two 8-byte device-scope stores
__device__ __forceinline__ void rlmd_st_wt16(void* p, float a, float b, float c, float d) {
  uint64_t* q = static_cast<uint64_t*>(p);
  rlmd_st_wt(q, (uint64_t)__float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32));
  rlmd_st_wt(q + 1, (uint64_t)__float_as_uint(c) | ((uint64_t)__float_as_uint(d) << 32));
}

__device__ inline uint64_t rlmd_block_bitonic(uint64_t key, int n, uint64_t* lds) {
  const int i = threadIdx.x;
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      uint64_t other;
      if (j >= 64) {
        __syncthreads();
        lds[i] = key;
        __syncthreads();
        other = lds[i ^ j];
      } else {
        other = rlmd_shfl_xor_u64(key, j);
      }
      // ascending sub-sequences alternate with descending ones while merging;
      // the final merge (k == n) is ascending in every n-aligned segment
      const bool up = k == n || (i & k) == 0;
      const bool keep_min = ((i & j) == 0) == up;
      key = keep_min ? (key < other ? key : other) : (key < other ? other : key);
    }
  }
  return key;
}

// ---------------------------------------------------------------------------
// host-side error plumbing for the C ABI
// ---------------------------------------------------------------------------
#include <string>
namespace rlmd {
void set_error(const std::string& msg);
}
#define RLMD_HIP(call)                                                                     \
  do {                                                                                     \
    hipError_t _e = (call);                                                                \
    if (_e != hipSuccess) {                                                                \
      rlmd::set_error(std::string(#call) + " failed: " + hipGetErrorString(_e) + " at " + \
                      __FILE__ + ":" + std::to_string(__LINE__));                          \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)
#define RLMD_CHECK(cond, msg)                                          \
  do {                                                                 \
    if (!(cond)) {                                                     \
      rlmd::set_error(std::string("rlmd: ") + (msg) + " [" #cond "]"); \
      return 1;                                                        \
    }                                                                  \
  } while (0)
#define RLMD_LAUNCH_CHECK()                                                                   \
  do {                                                                                        \
    hipError_t _e = hipGetLastError();                                                        \
    if (_e != hipSuccess) {                                                                   \
      rlmd::set_error(std::string("kernel launch failed: ") + hipGetErrorString(_e) + " at " + \
                      __FILE__ + ":" + std::to_string(__LINE__));                             \
      return 3;                                                                               \
    }                                                                                         \
  } while (0)
