// tgsim_flood.hip — device side of the flood workload (tgsim_flood_*):
// every instance forwards a publication, on its first receipt, to each neighbour but the sender.
//
// The reaction reads the last window's deliveries where the receive stage left them (SoA in inbox
// order, o_*), so a wave of forwards never leaves HBM:
//   k_flood_count  one thread per delivery: publication p = seq / D; first receipt iff the (p, v)
//                  bit is clear and no earlier delivery of v's inbox run carries p (the run is in
//                  (t, src, seq) order, so "earlier" is the oracle's sequential order); forwards =
//                  neighbours of v other than the sender.
//   scan           hipcub exclusive sum over the counts -> staged offsets (deterministic order:
//                  delivery index, then neighbour slot — the oracle's append order).
//   k_flood_emit   sets the seen bit of each first receipt and writes its forwards into the staged
//                  SoA (src, dst, seq, size, t) after the messages already staged.
// Bytes per delivery: 12 B read (dst, src, seq) + the receiver's row (≈ 4 B·deg, L2-resident for
// the graph's 32 MB at 1M × 8) + 1 bit; per forward 24 B written. HBM-bound streaming work.
#include <hipcub/hipcub.hpp>

#include "tgsim_dev.h"

namespace tgsim {

namespace {

__global__ __launch_bounds__(kBlock) void k_flood_count(const uint32_t* __restrict__ o_dst,
                                                        const uint32_t* __restrict__ o_src,
                                                        const uint32_t* __restrict__ o_seq,
                                                        const uint32_t* __restrict__ inbox, uint32_t n, uint32_t lo,
                                                        Flood f, DevScalars* sc) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i > n) return;
  if (i == n) { f.cnt[n] = 0; return; }
  const uint32_t v = o_dst[i] - lo, s = o_src[i], p = o_seq[i] / f.D;
  uint32_t c = 0, first = 0;
  if (p >= f.max_pubs) {
    atomicOr(&sc->err, ERR_BAD_MSG);
  } else if (!((f.seen[(size_t)p * f.wpp + (v >> 5)] >> (v & 31)) & 1u)) {
    first = 1;
    for (uint32_t j = i; j > inbox[v]; --j)
      if (o_seq[j - 1] / f.D == p) { first = 0; break; }
    if (first)
      for (uint32_t k = f.off[v]; k < f.off[v + 1]; ++k) c += f.nbr[k] != s;
  }
  f.cnt[i] = c;
  f.first[i] = (uint8_t)first;
}

__global__ __launch_bounds__(kBlock) void k_flood_emit(const uint32_t* __restrict__ o_dst,
                                                       const uint32_t* __restrict__ o_src,
                                                       const uint32_t* __restrict__ o_seq,
                                                       const int64_t* __restrict__ o_t, uint32_t n, uint32_t lo,
                                                       Flood f, uint32_t base, uint32_t size, int64_t horizon,
                                                       uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                       uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                       int64_t* __restrict__ m_t) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || !f.first[i]) return;
  const uint32_t g = o_dst[i], v = g - lo, s = o_src[i], p = o_seq[i] / f.D;
  atomicOr(&f.seen[(size_t)p * f.wpp + (v >> 5)], 1u << (v & 31));
  const int64_t t = o_t[i] > horizon ? o_t[i] : horizon;
  uint32_t w = base + f.pos[i];
  const uint32_t k0 = f.off[v], k1 = f.off[v + 1];
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t u = f.nbr[k];
    if (u == s) continue;
    m_src[w] = g; m_dst[w] = u; m_seq[w] = p * f.D + (k - k0); m_size[w] = size; m_t[w] = t;
    ++w;
  }
}

__global__ __launch_bounds__(kBlock) void k_flood_mark(const uint32_t* __restrict__ pairs, uint32_t n, Flood f) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = pairs[2 * i], p = pairs[2 * i + 1];
  atomicOr(&f.seen[(size_t)p * f.wpp + (v >> 5)], 1u << (v & 31));
}

inline unsigned blocks(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

hipError_t launch_flood_count(Dev& d, uint32_t n, uint32_t* total) {
  Flood& f = d.fl;
  {
    ProfScope ps_(d, KID_FLOOD_COUNT);
    hipLaunchKernelGGL(k_flood_count, dim3(blocks((uint64_t)n + 1)), dim3(kBlock), 0, d.stream, d.o_dst, d.o_src,
                       d.o_seq, d.inbox, n, d.lo, f, d.sc);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t bytes = f.scan_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(f.scan_tmp, bytes, f.cnt, f.pos, n + 1, d.stream);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(total, f.pos + n, sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(d.stream);
}

hipError_t launch_flood_emit(Dev& d, uint32_t n, uint32_t staged_base, uint32_t size, int64_t horizon) {
  if (!n) return hipSuccess;
  ProfScope ps_(d, KID_FLOOD_EMIT);
  hipLaunchKernelGGL(k_flood_emit, dim3(blocks(n)), dim3(kBlock), 0, d.stream, d.o_dst, d.o_src, d.o_seq, d.o_t, n,
                     d.lo, d.fl, staged_base, size, horizon, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_flood_mark(Dev& d, uint32_t n) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_flood_mark, dim3(blocks(n)), dim3(kBlock), 0, d.stream, d.fl.mark, n, d.fl);
  return hipGetLastError();
}

// scan scratch for up to n + 1 items (the runtime sizes it with the reaction's item capacity)
size_t flood_scan_bytes(uint32_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, n + 1);
  return bytes;
}

}  // namespace tgsim
