// Microbenchmark: per-item scattered atomics (the counting-sort histogram / cursor pattern):
// n items each add 1 to bin hash(i) % K, non-returning (hist) or returning (cursor -> scatter).
// hipcc --offload-arch=gfx950 -O3 tools/atomic_bench2.hip -o tools/atomic_bench2
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ unsigned hsh(unsigned i) { i *= 2654435761u; i ^= i >> 15; i *= 2246822519u; return i ^ (i >> 13); }
__global__ void k_bins(unsigned* c, unsigned K, unsigned n, unsigned* out, int mode, unsigned clus) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned key = clus ? (i / clus) % K : hsh(i) % K;
    if (mode == 0) {
      out[i] = key;
    } else if (mode == 1) {
      __hip_atomic_fetch_add(c + key, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const unsigned r = __hip_atomic_fetch_add(c + key, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      out[i] = r;
    }
  }
}
__global__ void k_empty(unsigned* p) { if (p && threadIdx.x == 1024) *p = 0; }
int main() {
  unsigned *c, *out;
  hipMalloc(&c, 1u << 22);
  hipMalloc(&out, 800000 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const unsigned n = 800000;
  auto timeit = [&](auto launch) {
    float best = 1e9;
    for (int rep = 0; rep < 7; ++rep) {
      hipMemset(c, 0, 1u << 22);
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); best = ms < best ? ms : best;
    }
    return best * 1e3;
  };
  printf("empty kernel x1: %.1f us\n", timeit([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, c); }));
  printf("empty kernel x20: %.1f us\n", timeit([&] { for (int k = 0; k < 20; ++k) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, c); }));
  for (unsigned clus : {0u, 8u})
    for (unsigned K : {1024u, 100000u})
      for (int mode = 0; mode < 3; ++mode)
        printf("clus=%u K=%6u mode=%d (0 none,1 add,2 fetch-add): %7.1f us\n", clus, K, mode,
               timeit([&] { hipLaunchKernelGGL(k_bins, dim3(2048), dim3(256), 0, 0, c, K, n, out, mode, clus); }));
  return 0;
}
