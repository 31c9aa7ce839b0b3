// Microbenchmark: cost of wave-aggregated returning atomics on K counters (128 B apart), the
// append pattern of the simulator's sharded queues. hipcc --offload-arch=gfx950 -O3 tools/atomic_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k_append(unsigned* ctr, int K, int n, unsigned* out, int mode) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    unsigned sub = ((i >> 6) + blockIdx.x) % K;
    unsigned* c = ctr + sub * 32;
    unsigned long long m = __ballot(1);
    int leader = __ffsll(m) - 1;
    unsigned base = 0;
    if (mode == 0) {  // returning, agent scope
      if ((int)(threadIdx.x & 63) == leader)
        base = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)c, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      base = __shfl(base, leader);
    } else if (mode == 1) {  // returning, workgroup scope (not correct across blocks; cost probe only)
      if ((int)(threadIdx.x & 63) == leader)
        base = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)c, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      base = __shfl(base, leader);
    } else {  // no atomic
      base = i & ~63u;
    }
    out[(base + (threadIdx.x & 63)) & ((1u << 22) - 1)] = i;
  }
}
int main() {
  unsigned *ctr, *out;
  hipMalloc(&ctr, 4096 * 128);
  hipMalloc(&out, (1u << 22) * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int n = 800000;
  for (int mode = 0; mode < 3; ++mode)
    for (int K : {1, 8, 64, 512, 4096}) {
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(ctr, 0, 4096 * 128);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_append, dim3(2048), dim3(256), 0, 0, ctr, K, n, out, mode);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
      }
      printf("mode=%d K=%5d  %8.1f us\n", mode, K, best * 1e3);
    }
  return 0;
}
