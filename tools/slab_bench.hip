// Microbenchmark for VERDICT r5 item 1 (producers appending token-bucket-bound copies straight into
// per-sender-bucket slabs): the producer-side cost of the two append forms on the storm's shape -
// 800k 32-B records from 2048 workgroups of 256 threads, each record's consumer bucket uniform over
// B = 1020 buckets (the extraction's due records arrive in wheel-slot order, so a wave's 64 records
// name ~62 distinct buckets):
//   subq  - the product's form: a wave appends its records to one of 64 sub-queues with ONE
//           returning atomic per wave (Queues::push_batch), 32-B stores in wave order;
//   slab  - wave-aggregated reservations per (wave, bucket) on the bucket's own slab cursor (one
//           128-B line per bucket: wave_append's leader loop), then the 32-B store into the slab;
//   slabx - as slab, with the buckets' cursors in 8 replicas by XCD (blockIdx % 8) and 8 slab parts.
// Prints the kernel time of each (best of 7), and the reservations made (per-wave counts summed on the
// host: one counter for all waves would itself serialise ~8k atomics on one line, ~96 us).
//   hipcc --offload-arch=gfx950 -O3 tools/slab_bench.hip -o tools/slab_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr unsigned kN = 800000, kB = 1020, kSlab = 2048;

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ unsigned lane() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ unsigned rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__global__ void k_subq(unsigned* ctr, uint4* out, unsigned* nres) {
  unsigned res = 0;
  for (unsigned i0 = blockIdx.x * blockDim.x; i0 < kN; i0 += gridDim.x * blockDim.x) {
    const unsigned i = i0 + threadIdx.x;
    const bool act = i < kN;
    const uint64_t m = __ballot(act);
    const unsigned sub = ((blockIdx.x & 7u) << 3) | ((threadIdx.x >> 6) & 7u);
    unsigned base = 0;
    if (lane() == 0) { base = atomicAdd(ctr + (sub << 5), (unsigned)__popcll(m)); ++res; }
    base = __shfl(base, 0);
    if (act) {
      const unsigned at = (sub * (kN / 32) + base + rank(m)) % (64u * (kN / 32));
      out[2 * at] = make_uint4(i, hash(i), 0, 0);
      out[2 * at + 1] = make_uint4(i, 0, 0, 0);
    }
  }
  for (int o = 32; o > 0; o >>= 1) res += __shfl_xor(res, o);
  if (lane() == 0) nres[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = res;  // summed on the host
}

template <int R>
__global__ void k_slab(unsigned* ctr, uint4* out, unsigned* nres) {
  unsigned res = 0;
  const unsigned rep = R > 1 ? (blockIdx.x & (R - 1)) : 0u;
  for (unsigned i0 = blockIdx.x * blockDim.x; i0 < kN; i0 += gridDim.x * blockDim.x) {
    const unsigned i = i0 + threadIdx.x;
    bool pend = i < kN;
    const unsigned b = hash(i) % kB;
    unsigned pos = 0;
    for (;;) {  // wave_append: one leader atomic per distinct bucket of the wave
      const uint64_t m = __ballot(pend);
      if (!m) break;
      const int ld = __ffsll((unsigned long long)m) - 1;
      const unsigned lb = __shfl(b, ld);
      const bool mine = pend && b == lb;
      const uint64_t mm = __ballot(mine);
      unsigned base = 0;
      if ((int)lane() == ld) { base = atomicAdd(ctr + ((lb * R + rep) << 5), (unsigned)__popcll(mm)); ++res; }
      base = __shfl(base, ld);
      if (mine) { pos = base + rank(mm); pend = false; }
    }
    if (i < kN) {
      const unsigned at = ((b * R + rep) * (kSlab / R) + pos % (kSlab / R));
      out[2 * at] = make_uint4(i, hash(i), 0, 0);
      out[2 * at + 1] = make_uint4(i, 0, 0, 0);
    }
  }
  for (int o = 32; o > 0; o >>= 1) res += __shfl_xor(res, o);
  if (lane() == 0) nres[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = res;  // summed on the host
}

int main() {
  unsigned *ctr, *nres;
  uint4* out;
  hipMalloc(&ctr, (size_t)kB * 8 * 128 + 64 * 128);
  const unsigned nw = 2048 * 4;
  hipMalloc(&nres, nw * 4);
  unsigned* hres = new unsigned[nw];
  hipMalloc(&out, (size_t)kB * kSlab * 32 + (size_t)64 * (kN / 32) * 32);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  auto timeit = [&](const char* name, auto launch) {
    float best = 1e9;
    unsigned r = 0;
    for (int rep = 0; rep < 7; ++rep) {
      hipMemset(ctr, 0, (size_t)kB * 8 * 128 + 64 * 128);
      hipDeviceSynchronize();
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); best = ms < best ? ms : best;
      hipMemcpy(hres, nres, nw * 4, hipMemcpyDeviceToHost);
      r = 0;
      for (unsigned w = 0; w < nw; ++w) r += hres[w];
    }
    printf("%-6s %8.1f us  reservations %u (%.0f per us)\n", name, best * 1e3, r, r / (best * 1e3));
  };
  const dim3 g(2048), t(256);
  timeit("subq", [&] { hipLaunchKernelGGL(k_subq, g, t, 0, 0, ctr, out, nres); });
  timeit("slab", [&] { hipLaunchKernelGGL(k_slab<1>, g, t, 0, 0, ctr, out, nres); });
  timeit("slabx", [&] { hipLaunchKernelGGL(k_slab<8>, g, t, 0, 0, ctr, out, nres); });
  return 0;
}
