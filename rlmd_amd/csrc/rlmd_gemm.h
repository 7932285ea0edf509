// rlmd_gemm.h — internal GEMM launch interface (see gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rlmd_abi.h"
#include "rlmd_adam.h"

#define RLMD_GEMM_MAX_PROBS 6

namespace rlmd {

enum { GEMM_FWD = 0, GEMM_BWD_X = 1, GEMM_BWD_W = 2 };

// Output C is [M, N] (BWD_W: the weight-gradient [out, in] with M = out, N = in,
// K = batch).  All pointers f32 device memory.
struct GemmProblem {
  const float* A;
  int32_t lda;
  const float* B;
  int32_t ldb;
  const float* bias;  // FWD: bias[N]
  float* C;
  int32_t ldc;
  const float* mask;  // BWD_X: ReLU mask source [M, N] (element > 0 keeps)
  int32_t ldm;
  float* bias_grad;   // BWD_W: bias gradient [M]
  // FWD (mini-batch tiles only): fused single-output head.  Each 32-column tile
  // writes head_part[tile][i] = sum over its columns j of act(C[i, j]) * head_w[j];
  // consumers add the ceil(N/32) partials in tile order (deterministic).
  const float* head_w;
  float* head_part;
};

struct GemmShape {
  int32_t M, N, K, relu;
};

// Up to RLMD_GEMM_MAX_PROBS independent problems of one mode, each with its own
// shape, share a launch: blockIdx.x runs over the concatenated output tiles of
// all problems (tile_begin is filled in by gemm_launch), blockIdx.z is the
// split-K slab.
struct GemmBatch {
  GemmShape shape[RLMD_GEMM_MAX_PROBS];
  GemmProblem prob[RLMD_GEMM_MAX_PROBS];
  int32_t nprob;
  int32_t tiles_n[RLMD_GEMM_MAX_PROBS];         // set by gemm_launch
  int32_t tile_begin[RLMD_GEMM_MAX_PROBS + 1];  // set by gemm_launch
  int32_t splits;        // BWD_W split-K: slabs written at C + s*split_stride (and bias_grad)
  int64_t split_stride;  // floats between slabs
  // BWD_W with fuse_adam (32x32 tiles): each split publishes its partial to a
  // private slab (slabs: [tiles][splits][256 threads] x 16 B) and takes an
  // arrival ticket on tile_ctr[tile] (monotonic, zero-initialised once); the
  // tile's last arrival sums the slabs in order (the rounding of adam_kernel)
  // and steps the parameters it covers (rlmd_adam.h).  Parameter index = (C or
  // bias_grad) - adam.g + element offset.
  int32_t fuse_adam;
  AdamArgs adam;
  __attribute__((ext_vector_type(4))) float* slabs;
  unsigned* tile_ctr;
  int32_t max_tiles;  // capacity of slabs / tile_ctr
};

// Appends one problem; returns its index.
inline int gemm_add(GemmBatch& b, const GemmShape& s, const GemmProblem& p) {
  b.shape[b.nprob] = s;
  b.prob[b.nprob] = p;
  return b.nprob++;
}

int gemm_launch(int prec, int mode, const GemmBatch& b, hipStream_t stream);

// 32x32 output tiles of a weight-gradient problem [M = out, N = in] (+ the db column)
inline int bwd_w_tiles(int M, int N) { return ((N + 1 + 31) / 32) * ((M + 31) / 32); }

}  // namespace rlmd
