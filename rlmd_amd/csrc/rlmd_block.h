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
// constant so that 18 of the 21 stages move lanes by DPP (rlmd_xor_lane).
template <int K, int J>
__device__ __forceinline__ uint64_t bitonic_stage(uint64_t key, int l) {
  const uint64_t other = rlmd_xor_lane_u64<J>(key);
  const bool up = (l & K) == 0 || K == 64;
  const bool keep_min = ((l & J) == 0) == up;
  // one compare: this lane keeps its own key exactly when (key < other) agrees
  // with keeping the minimum (keys are distinct but for absent ~0 ones)
  key = ((key < other) == keep_min) ? key : other;
  if constexpr (J > 1) return bitonic_stage<K, J / 2>(key, l);
  else if constexpr (K < 64) return bitonic_stage<2 * K, K>(key, l);
  else return key;
}
__device__ __forceinline__ uint64_t wave_sort64(uint64_t key) {
  return bitonic_stage<2, 1>(key, (int)(threadIdx.x & 63));
}

// Ranks of distinct 64-bit keys across the block (ascending; key ~0 = absent):
// each wave sorts its 64 keys in registers, parks the sorted run in LDS, and the
// key at lane l of run w gets rank l + sum over the other runs of a binary
// search (6 probes over the first 63 entries + the last entry).  The searches
// over the other runs are independent: each probe step reads all of them at
// once, so the dependent LDS chain is 6 probes long, not 6 per run.  The rank is
// scattered to out[key & 0xffffffff] (the caller's index in the low word) and
// read back by the key's owner after the barrier.
// runs: LDS [blockDim.x] uint64; out: LDS int [blockDim.x].  NW: the block's
// waves (blockDim.x == 64 NW), a compile-time constant so that every probe is
// an unconditional LDS read (one wait per probe step for all runs).
template <int NW>
__device__ __forceinline__ void block_rank(uint64_t key, uint64_t* runs, int* out) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t sk = wave_sort64(key);
  runs[threadIdx.x] = sk;
  __syncthreads();
  int pos[NW];
#pragma unroll
  for (int v = 0; v < NW; ++v) pos[v] = 0;
#pragma unroll
  for (int st = 32; st > 0; st >>= 1) {
    uint64_t probe[NW];
#pragma unroll
    for (int v = 0; v < NW; ++v) probe[v] = runs[64 * v + pos[v] + st - 1];
#pragma unroll
    for (int v = 0; v < NW; ++v) pos[v] += probe[v] < sk ? st : 0;
  }
  int rank = l;
#pragma unroll
  for (int v = 0; v < NW; ++v) rank += v == w ? 0 : pos[v] + (runs[64 * v + 63] < sk ? 1 : 0);
  if (sk != ~0ull) out[(int)(sk & 0xffffffffu)] = rank;
  __syncthreads();
}

}  // namespace
}  // namespace rlmd
