// Microbenchmark: block reservations on C append counters (the Queues sub-queue pattern): every
// block, each round, one returning agent-scope atomicAdd by thread 0 on counter (block + round) % C,
// a barrier, then a 16-B store per thread at the reserved place. Counters `stride` bytes apart:
// does the counters' spacing (lines of one memory channel or of many) change the rate?
// hipcc --offload-arch=gfx950 -O3 tools/atomic_bench3.hip -o tools/atomic_bench3
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_res(unsigned* c, unsigned C, unsigned stride_w, unsigned rounds, uint4* out, unsigned cap) {
  __shared__ unsigned base;
  for (unsigned r = 0; r < rounds; ++r) {
    if (threadIdx.x == 0) {
      const unsigned k = (blockIdx.x + r * 7u) % C;
      base = __hip_atomic_fetch_add(c + (size_t)k * stride_w, blockDim.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const unsigned at = (base + threadIdx.x) % cap;
    out[at] = make_uint4(at, r, blockIdx.x, 0);
    __syncthreads();
  }
}
int main() {
  unsigned* c;
  uint4* out;
  const size_t cbytes = 64ull << 20;
  hipMalloc(&c, cbytes);
  const unsigned cap = 1u << 22;
  hipMalloc(&out, (size_t)cap * 16);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  auto timeit = [&](auto launch) {
    float best = 1e9;
    for (int rep = 0; rep < 7; ++rep) {
      hipMemset(c, 0, cbytes);
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); best = ms < best ? ms : best;
    }
    return best * 1e3;
  };
  for (unsigned C : {1u, 8u, 16u, 64u, 192u})
    for (unsigned stride : {4u, 128u, 256u, 512u, 1024u, 2048u, 4096u, 8192u, 65536u}) {
      if (C == 1 && stride > 4) continue;
      if ((size_t)C * stride > cbytes) continue;
      const float us = timeit([&] { hipLaunchKernelGGL(k_res, dim3(2048), dim3(256), 0, 0, c, C, stride / 4, 8u, out, cap); });
      printf("C=%4u stride=%6u B: %7.1f us  (%.1f reservations/us)\n", C, stride, us, 2048.0 * 8 / us);
    }
  return 0;
}
