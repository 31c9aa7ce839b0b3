// tgsim_flood.hip — device side of the flood workload (tgsim_flood_*):
// every instance forwards a publication, on its first receipt, to each neighbour but the sender.
//
// The reaction reads the last window's deliveries where the receive stage left them (SoA in inbox
// order, o_*) and their count from the device (sc->n_out), so a wave of forwards needs no host
// round trip. The deliveries split into kFloodBlocks contiguous chunks:
//   k_flood_count  per delivery: publication p = seq / D; first receipt iff the (p, v) bit is clear
//                  and no earlier delivery of v's inbox run carries p (the run is in (t, src, seq)
//                  order, so "earlier" is the oracle's sequential order); forwards = neighbours of
//                  v other than the sender; the chunk's total -> bsum[chunk].
//   k_flood_scan   one block: exclusive scan of the chunk totals + the staging base (host-known, or
//                  the device count sc->n_msgs_dev) -> each chunk's first staged slot; new count.
//   k_flood_emit   per chunk, tile by tile (block scan of the counts): the seen bit of each first
//                  receipt and its forwards in the staged SoA (src, dst, seq, size, t) — the
//                  oracle's append order (delivery index, then neighbour slot).
// Bytes per delivery: 12 B read (dst, src, seq) + the receiver's row (≈ 4 B·deg, L2-resident for
// the graph's 32 MB at 1M × 8) + 5 B of scratch written and read + 1 bit; per forward 24 B written.
// HBM-bound streaming work.
#include <algorithm>

#include "tgsim_dev.h"

namespace tgsim {

namespace {

constexpr uint32_t kWalkMax = 32;  // k_flood_emit: rows up to this long are written one slot per thread
constexpr uint32_t kMultiSender = 0xFFFFFFFFu;  // k_flood_emit: the sender occurs more than once in the row

// Chunk c of the n deliveries: [c * per, min(n, (c + 1) * per)).
__device__ __forceinline__ void chunk_range(uint32_t n, uint32_t& i0, uint32_t& i1) {
  const uint32_t per = (n + kFloodBlocks - 1) / kFloodBlocks;
  i0 = min(n, blockIdx.x * per);
  i1 = min(n, i0 + per);
}

__global__ __launch_bounds__(kBlock) void k_flood_count(const uint32_t* __restrict__ o_dst,
                                                        const uint32_t* __restrict__ o_src,
                                                        const uint32_t* __restrict__ o_seq,
                                                        const uint32_t* __restrict__ inbox, uint32_t lo, Flood f,
                                                        DevScalars* sc) {
  __shared__ uint32_t red[kBlock / 64];
  uint32_t i0, i1;
  chunk_range(sc->n_out, i0, i1);
  uint32_t sum = 0;
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += kBlock) {
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
    sum += c;
  }
  uint32_t total;
  (void)block_excl_scan(sum, red, total);
  if (threadIdx.x == 0) f.bsum[blockIdx.x] = total;
}

// One block: chunk totals -> staged offsets of the chunks (in place), the new staged count.
__global__ __launch_bounds__(kBlock) void k_flood_scan(Flood f, DevScalars* sc, uint32_t base_dev, uint32_t base_host,
                                                       uint32_t cap) {
  __shared__ uint32_t red[kBlock / 64];
  constexpr uint32_t per = kFloodBlocks / kBlock;
  static_assert(kFloodBlocks % kBlock == 0, "chunks per thread");
  uint32_t v[per], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < per; ++k) { v[k] = f.bsum[threadIdx.x * per + k]; sum += v[k]; }
  uint32_t total;
  uint32_t run = block_excl_scan(sum, red, total);
  const uint32_t base = base_dev ? sc->n_msgs_dev : base_host;
#pragma unroll
  for (uint32_t k = 0; k < per; ++k) { f.bsum[threadIdx.x * per + k] = base + run; run += v[k]; }
  if (threadIdx.x == 0) {
    const uint64_t end = (uint64_t)base + total;
    if (end > cap) atomicOr(&sc->err, ERR_CAP_M);  // emit writes only below cap
    sc->n_msgs_dev = (uint32_t)(end < cap ? end : cap);
    sc->fl_total = total;
  }
}

__global__ __launch_bounds__(kBlock) void k_flood_emit(const uint32_t* __restrict__ o_dst,
                                                       const uint32_t* __restrict__ o_src,
                                                       const uint32_t* __restrict__ o_seq,
                                                       const int64_t* __restrict__ o_t, uint32_t lo, Flood f,
                                                       const DevScalars* sc, uint32_t size, int64_t horizon,
                                                       uint32_t cap, uint32_t* __restrict__ m_src,
                                                       uint32_t* __restrict__ m_dst, uint32_t* __restrict__ m_seq,
                                                       uint32_t* __restrict__ m_size, int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  // the tile's first receipts in LDS; their forwards are then written one output slot per thread
  // (consecutive lanes, consecutive slots) instead of one delivery per thread (lanes ≈deg slots apart)
  __shared__ uint32_t s_off[kBlock], s_g[kBlock], s_s[kBlock], s_p[kBlock], s_k0[kBlock], s_k1[kBlock];
  __shared__ uint32_t s_pos[kBlock];  // the sender's place in a short row (kMultiSender: more than one)
  __shared__ int64_t s_t[kBlock];
  uint32_t i0, i1;
  chunk_range(sc->n_out, i0, i1);
  uint32_t run = f.bsum[blockIdx.x];
  for (uint32_t t0 = i0; t0 < i1; t0 += kBlock) {  // block-uniform trip count: the scan's barriers
    const uint32_t i = t0 + threadIdx.x;
    const bool in = i < i1;
    const bool first = in && f.first[i];
    uint32_t tile;
    s_off[threadIdx.x] = block_excl_scan(first ? f.cnt[i] : 0u, red, tile);
    if (first) {
      const uint32_t g = o_dst[i], v = g - lo, p = o_seq[i] / f.D;
      atomicOr(&f.seen[(size_t)p * f.wpp + (v >> 5)], 1u << (v & 31));
      s_g[threadIdx.x] = g; s_s[threadIdx.x] = o_src[i]; s_p[threadIdx.x] = p;
      s_k0[threadIdx.x] = f.off[v]; s_k1[threadIdx.x] = f.off[v + 1];
      s_t[threadIdx.x] = o_t[i] > horizon ? o_t[i] : horizon;
      const uint32_t k0 = s_k0[threadIdx.x], k1 = s_k1[threadIdx.x];
      if (k1 - k0 > kWalkMax) {  // a long row: its own thread writes it (the walk below is O(row) per slot)
        const uint32_t s = s_s[threadIdx.x];
        uint32_t w = run + s_off[threadIdx.x];
        for (uint32_t k = k0; k < k1; ++k) {
          const uint32_t u = f.nbr[k];
          if (u == s) continue;
          if (w < cap) { m_src[w] = g; m_dst[w] = u; m_seq[w] = p * f.D + (k - k0); m_size[w] = size; m_t[w] = s_t[threadIdx.x]; }
          ++w;
        }
      } else {  // one pass over the short row: where the sender sits, so a slot needs one row load
        const uint32_t s = s_s[threadIdx.x];
        uint32_t pos = k1 - k0, mult = 0;
        for (uint32_t k = k0; k < k1; ++k) {
          const bool hit = f.nbr[k] == s;
          pos = hit && !mult ? k - k0 : pos;
          mult += hit;
        }
        s_pos[threadIdx.x] = mult > 1 ? kMultiSender : pos;
      }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < tile; j += kBlock) {
      // the delivery d whose forwards cover j: the last offset <= j (a delivery with forwards has a
      // larger offset than every one before it)
      uint32_t lo_d = 0, hi_d = kBlock;
      while (hi_d - lo_d > 1) {
        const uint32_t mid = (lo_d + hi_d) >> 1;
        if (s_off[mid] <= j) lo_d = mid; else hi_d = mid;
      }
      const uint32_t d = lo_d, s = s_s[d], k0 = s_k0[d], k1 = s_k1[d];
      if (k1 - k0 > kWalkMax) continue;
      uint32_t r = j - s_off[d], k = k0;
      const uint32_t pos = s_pos[d];
      if (pos != kMultiSender) {  // the r-th neighbour other than the sender (row order)
        k = k0 + r + (r >= pos ? 1u : 0u);
      } else {
        for (; k < k1; ++k) {
          if (f.nbr[k] == s) continue;
          if (r == 0) break;
          --r;
        }
      }
      const uint32_t w = run + j;
      if (w < cap) {
        m_src[w] = s_g[d]; m_dst[w] = f.nbr[k]; m_seq[w] = s_p[d] * f.D + (k - k0); m_size[w] = size;
        m_t[w] = s_t[d];
      }
    }
    run += tile;
    __syncthreads();  // the next tile rewrites the LDS arrays
  }
}

__global__ __launch_bounds__(kBlock) void k_flood_mark(const uint32_t* __restrict__ pairs, uint32_t n, Flood f) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = pairs[2 * i], p = pairs[2 * i + 1];
  atomicOr(&f.seen[(size_t)p * f.wpp + (v >> 5)], 1u << (v & 31));
}

// Appends behind the device-side staged count (sc non-null: every thread reads the same base, nothing
// in this launch writes it; k_append_commit moves the count afterwards), or at the host-known base
// (sc null: tgsim_enqueue_device, one launch for the five arrays instead of five copies).
__global__ __launch_bounds__(kBlock) void k_append(const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                                   const uint32_t* __restrict__ seq,
                                                   const uint32_t* __restrict__ size, const int64_t* __restrict__ t,
                                                   uint32_t n, uint32_t cap, const DevScalars* sc, uint32_t base_host,
                                                   uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                   uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                   int64_t* __restrict__ m_t) {
  const uint32_t base = sc ? sc->n_msgs_dev : base_host;
  if ((uint64_t)base + n > cap) return;  // k_append_commit reports it (the host checked its own base)
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    m_src[base + i] = src[i]; m_dst[base + i] = dst[i]; m_seq[base + i] = seq[i]; m_size[base + i] = size[i];
    m_t[base + i] = t[i];
  }
}

__global__ void k_append_commit(uint32_t n, uint32_t cap, DevScalars* sc) {
  const uint64_t end = (uint64_t)sc->n_msgs_dev + n;
  if (end > cap) atomicOr(&sc->err, ERR_CAP_M);
  else sc->n_msgs_dev = (uint32_t)end;
}

}  // namespace

hipError_t launch_flood_react(Dev& d, bool base_dev, uint32_t base_host, uint32_t size, int64_t horizon) {
  Flood& f = d.fl;
  {
    ProfScope ps_(d, KID_FLOOD_COUNT);
    hipLaunchKernelGGL(k_flood_count, dim3(kFloodBlocks), dim3(kBlock), 0, d.stream, d.o_dst, d.o_src, d.o_seq,
                       d.inbox, d.lo, f, d.sc);
    hipLaunchKernelGGL(k_flood_scan, dim3(1), dim3(kBlock), 0, d.stream, f, d.sc, (uint32_t)base_dev, base_host,
                       d.cap_msgs);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  ProfScope ps_(d, KID_FLOOD_EMIT);
  hipLaunchKernelGGL(k_flood_emit, dim3(kFloodBlocks), dim3(kBlock), 0, d.stream, d.o_dst, d.o_src, d.o_seq, d.o_t,
                     d.lo, f, d.sc, size, horizon, d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_append(Dev& d, const uint32_t* src, const uint32_t* dst, const uint32_t* seq, const uint32_t* size,
                         const int64_t* t, uint32_t n) {
  if (!n) return hipSuccess;
  const unsigned g = std::min<unsigned>((n + kBlock - 1) / kBlock, (unsigned)kStreamBlocks);
  hipLaunchKernelGGL(k_append, dim3(g), dim3(kBlock), 0, d.stream, src, dst, seq, size, t, n, d.cap_msgs, d.sc, 0u,
                     d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  hipLaunchKernelGGL(k_append_commit, dim3(1), dim3(1), 0, d.stream, n, d.cap_msgs, d.sc);
  return hipGetLastError();
}

hipError_t launch_stage(Dev& d, const uint32_t* src, const uint32_t* dst, const uint32_t* seq, const uint32_t* size,
                        const int64_t* t, uint32_t n, uint32_t base) {
  if (!n) return hipSuccess;
  const unsigned g = std::min<unsigned>((n + kBlock - 1) / kBlock, (unsigned)kStreamBlocks);
  hipLaunchKernelGGL(k_append, dim3(g), dim3(kBlock), 0, d.stream, src, dst, seq, size, t, n, d.cap_msgs,
                     (const DevScalars*)nullptr, base, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_flood_mark(Dev& d, uint32_t n) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_flood_mark, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, d.stream, d.fl.mark, n, d.fl);
  return hipGetLastError();
}

}  // namespace tgsim
