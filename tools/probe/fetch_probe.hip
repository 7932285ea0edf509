// fetch_probe.hip — how long does one workgroup take to pull a 128 KB weight
// matrix (as the learn row kernels' fragment prefetch does: 8 waves x 16 loads
// of 16 B per lane, all issued up front) right after another launch wrote it,
// and when it is already cache-warm?  Prints cycles (s_memtime) from the first
// issue to the last landed load, max over the workgroup's waves, median over
// workgroups.  Experiment tool (tools/probe), not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef short bf16x8 __attribute__((ext_vector_type(8)));

__global__ void writer(bf16x8* w, int n, short v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    w[i] = bf16x8{v, v, v, v, v, v, v, v};
}

// each workgroup: 8 waves, wave q loads fragments [q * 16, q * 16 + 16) x 64 lanes
// scat: also 48 scattered 4-B loads per lane (every lane its own cache line),
// as the row kernels' first load round issues for masks / fc1 columns / scalars
template <int SCAT>
__global__ void __launch_bounds__(512) reader(const bf16x8* w, int nfrag_per_wave, unsigned long long* out,
                                              float* sink, const float* sc) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bf16x8* p = w + (size_t)(wave * nfrag_per_wave) * 64 + lane;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float sv[SCAT > 0 ? SCAT : 1];
#pragma unroll
  for (int j = 0; j < SCAT; ++j) sv[j] = sc[((threadIdx.x * 37 + j * 4099 + blockIdx.x * 613) & 65535) * 32];
  bf16x8 acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = p[j * 64];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < SCAT; ++j) s += sv[j];
#pragma unroll
  for (int j = 0; j < 16; ++j) s += (float)acc[j][0] + (float)acc[j][7];
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __shared__ unsigned long long dt[8];
  if (lane == 0) dt[wave] = t1 - t0;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = 0;
    for (int q = 0; q < 8; ++q) m = dt[q] > m ? dt[q] : m;
    out[blockIdx.x] = m;
  }
  if (s == 12345.f) sink[threadIdx.x] = s;
}

static unsigned long long median(std::vector<unsigned long long> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int nfrag = 8 * 16 * 64;  // 128 KB of 16-B fragments
  bf16x8* w;
  unsigned long long* out;
  float* sink;
  hipMalloc(&w, sizeof(bf16x8) * nfrag);
  hipMalloc(&out, sizeof(unsigned long long) * 1024);
  hipMalloc(&sink, 4096);
  float* sc;
  hipMalloc(&sc, sizeof(float) * 65536 * 32);
  hipMemset(sc, 0, sizeof(float) * 65536 * 32);
  std::vector<unsigned long long> h(1024);
  for (int scat = 0; scat < 2; ++scat)
  for (int nwg : {1, 32, 160}) {
    for (int mode = 0; mode < 2; ++mode) {  // 0: right after a writer launch, 1: after another reader (warm)
      std::vector<unsigned long long> med;
      for (int it = 0; it < 20; ++it) {
        hipLaunchKernelGGL(writer, dim3(256), dim3(256), 0, 0, w, nfrag, (short)it);
        if (scat) {
          if (mode == 1) hipLaunchKernelGGL(reader<48>, dim3(nwg), dim3(512), 0, 0, w, 16, out, sink, sc);
          hipLaunchKernelGGL(reader<48>, dim3(nwg), dim3(512), 0, 0, w, 16, out, sink, sc);
        } else {
          if (mode == 1) hipLaunchKernelGGL(reader<0>, dim3(nwg), dim3(512), 0, 0, w, 16, out, sink, sc);
          hipLaunchKernelGGL(reader<0>, dim3(nwg), dim3(512), 0, 0, w, 16, out, sink, sc);
        }
        hipMemcpy(h.data(), out, sizeof(unsigned long long) * nwg, hipMemcpyDeviceToHost);
        if (it >= 4) med.push_back(median(std::vector<unsigned long long>(h.begin(), h.begin() + nwg)));
      }
      printf("%s workgroups %4d  %-28s  128 KB per workgroup: median %6llu cycles (%.1f B/cycle/CU)\n",
             scat ? "+48 scattered 4-B loads/lane" : "fragments only              ", nwg,
             mode == 0 ? "after a writer launch" : "after a reader (warm)", median(med),
             131072.0 / (double)median(med));
    }
  }
  return 0;
}
