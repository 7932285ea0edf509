// rlmd_block.h — workgroup-level building blocks shared by the loss kernels
// (learn.hip) and the row kernels (rows.hip): wave sums, orderable float keys,
// deterministic block all-reduces and block-wide ranks of distinct 64-bit keys.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rlmd_common.h"

namespace rlmd {
namespace {

// 64-lane sum: DPP within each 16-lane row, then two cross-row shuffles
__device__ __forceinline__ float wave_sum(float v) {
  v = rlmd_row16_sum(v);
  v += __uint_as_float(rlmd_xor_lane<16>(__float_as_uint(v)));
  v += __shfl_xor(v, 32, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  v = rlmd_row16_max(v);
  v = fmaxf(v, __uint_as_float(rlmd_xor_lane<16>(__float_as_uint(v))));
  v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

// orderable key of a float (ascending unsigned order == ascending float order)
__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Block all-reduce of NS sums and NM maxima at once (3 barriers).  Each wave
// reduces with shuffles and parks its partial in red[v][16]; lanes of the first
// waves fold the per-wave partials of one value each (a fixed tree, so the
// result is deterministic) and every thread reads the NS + NM results back.
// red: 16 * (NS + NM) + 16 floats.
template <int NS, int NM>
__device__ __forceinline__ void block_allreduce(float* sm, float* mx, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  constexpr int NV = NS + NM;
  float* res = red + 16 * NV;
#pragma unroll
  for (int v = 0; v < NS; ++v) sm[v] = wave_sum(sm[v]);
#pragma unroll
  for (int v = 0; v < NM; ++v) mx[v] = wave_max(mx[v]);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < NS; ++v) red[v * 16 + w] = sm[v];
#pragma unroll
    for (int v = 0; v < NM; ++v) red[(NS + v) * 16 + w] = mx[v];
  }
  __syncthreads();
  if ((int)threadIdx.x < 16 * NV) {
    const int v = threadIdx.x >> 4, q = threadIdx.x & 15;
    const bool is_sum = v < NS;
    const float t = q < nw ? red[threadIdx.x] : (is_sum ? 0.f : -INFINITY);
    const float r = is_sum ? rlmd_row16_sum(t) : rlmd_row16_max(t);  // one 16-lane row per value
    if (q == 0) res[v] = r;
  }
  __syncthreads();
#pragma unroll
  for (int v = 0; v < NS; ++v) sm[v] = res[v];
#pragma unroll
  for (int v = 0; v < NM; ++v) mx[v] = res[NS + v];
  __syncthreads();  // red / res reusable
}

// Ascending bitonic sort of one 64-bit key per lane across the wave (registers):
// merge stage (K, J) exchanges with lane l ^ J, the stride a compile-time
// constant so that 18 of the 21 stages move lanes by DPP (rlmd_xor_lane).  Which
// lanes keep the minimum depends on the lane index only: a 64-bit constant per
// stage, applied to the compare's lane mask on the scalar unit (ballot ->
// s_xnor -> inverse ballot), so a stage costs the two lane moves, one 64-bit
// compare and two selects on the VALU.
template <int K, int J>
constexpr uint64_t bitonic_keep_min() {
  uint64_t m = 0;
  for (int l = 0; l < 64; ++l) {
    const bool up = (l & K) == 0 || K == 64;
    if (((l & J) == 0) == up) m |= 1ull << l;
  }
  return m;
}
template <int K, int J>
__device__ __forceinline__ uint64_t bitonic_stage(uint64_t key) {
  const uint64_t other = rlmd_xor_lane_u64<J>(key);
  // this lane keeps its own key exactly when (key < other) agrees with keeping
  // the minimum (keys are distinct but for absent ~0 ones)
  const uint64_t lt = __builtin_amdgcn_ballot_w64(key < other);
  key = __builtin_amdgcn_inverse_ballot_w64(~(lt ^ bitonic_keep_min<K, J>())) ? key : other;
  if constexpr (J > 1) return bitonic_stage<K, J / 2>(key);
  else if constexpr (K < 64) return bitonic_stage<2 * K, K>(key);
  else return key;
}
__device__ __forceinline__ uint64_t wave_sort64(uint64_t key) { return bitonic_stage<2, 1>(key); }

// Ranks of distinct 64-bit keys across the block (ascending; key ~0 = absent):
// each wave sorts its 64 keys in registers, parks the sorted run in LDS, and the
// key at lane l of run w gets rank l + sum over the other NW - 1 runs of a
// binary search (6 probes over the first 63 entries + the last entry).  The
// searches over the other runs are independent: each probe step reads all of
// them at once, so the dependent LDS chain is 6 probes long, not 6 per run.  A
// search position is kept as a byte address (the run's base folded in), so a
// probe is one LDS read with a constant offset, one 64-bit compare, one select
// and one add: the rank is VALU-bound at two waves per SIMD.  The rank is
// scattered to out[key & 0xffffffff] (the caller's index in the low word) and
// read back by the key's owner after the barrier.
// runs: LDS [blockDim.x] uint64; out: LDS int [blockDim.x].  NW: the block's
// waves (blockDim.x == 64 NW), a compile-time constant.
template <int NW>
__device__ __forceinline__ void block_rank(uint64_t key, uint64_t* runs, int* out) {
  typedef const __attribute__((address_space(3))) uint64_t lds_u64;
  const int l = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform: scalar run bases
  const uint64_t sk = wave_sort64(key);
  runs[threadIdx.x] = sk;
  __syncthreads();
  if constexpr (NW == 1) {
    if (sk != ~0ull) out[(int)(sk & 0xffffffffu)] = l;
    __syncthreads();
    return;
  }
  // LDS byte address of each other run's search position
  const uint32_t r0 = (uint32_t)(uintptr_t)(lds_u64*)runs;
  uint32_t at[NW > 1 ? NW - 1 : 1];
#pragma unroll
  for (int i = 0; i < NW - 1; ++i) at[i] = r0 + (uint32_t)(512 * ((w + 1 + i) % NW));
#pragma unroll
  for (int st = 32; st > 0; st >>= 1) {
    uint64_t probe[NW > 1 ? NW - 1 : 1];
#pragma unroll
    for (int i = 0; i < NW - 1; ++i) probe[i] = *(lds_u64*)(uintptr_t)(at[i] + 8u * (st - 1));
#pragma unroll
    for (int i = 0; i < NW - 1; ++i) at[i] += probe[i] < sk ? 8u * st : 0u;
    // keep each step's reads together (one LDS round per step): unconstrained,
    // the scheduler ran one run's six dependent probes after another
    __builtin_amdgcn_sched_barrier(0);
  }
  int rank = l;
#pragma unroll
  for (int i = 0; i < NW - 1; ++i) {
    const uint32_t run0 = r0 + (uint32_t)(512 * ((w + 1 + i) % NW));
    rank += (int)((at[i] - run0) >> 3) + (*(lds_u64*)(uintptr_t)(run0 + 504u) < sk ? 1 : 0);
  }
  if (sk != ~0ull) out[(int)(sk & 0xffffffffu)] = rank;
  __syncthreads();
}

}  // namespace
}  // namespace rlmd
