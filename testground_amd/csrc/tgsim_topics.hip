// tgsim_topics.hip — device side of sync.Client Subscribe for many subscribers at once
// (tgsim_sync_subscribe_device): the address-exchange fan-out of every plan (storm.go:232-255,
// pingpong.go:219-245, splitbrain/main.go:91-103), where each of N instances reads the N entries of
// one topic — N^2 deliveries — without a host round trip.
//
// The topic log is the arena tgsim_sync_publish appends to: one entry per publication, grouped per
// publish batch by (topic, position), so a topic's positions 1..count are a short list of runs
// (pos0, len, first entry) — one per batch that published to it. Entry times never decrease along a
// topic's positions (batches cannot go back in time; a batch orders by (t, instance)).
//   k_sub_count  one thread per subscriber: binary search over the topic's runs (by first time) and
//                inside the last visible run -> the last position with t <= until_t; count =
//                min(last - from + 1, cap_each) (0 if negative).
//   scan         hipcub exclusive sum (64-bit: N^2 overflows 32 bits at 66k subscribers).
//   k_sub_fill   block per subscriber (grid-stride): the entry ids of positions from .. from+count-1,
//                run by run, as contiguous coalesced 16-B stores into the subscriber's inbox slice.
// Bytes per delivery: 4 B written (the id; the entry itself is read from the shared, L2-resident
// arena by whoever consumes the inbox). Per subscriber: 24 B read + 8 B offset written.
#include <hipcub/hipcub.hpp>

#include "tgsim_dev.h"

namespace tgsim {

namespace {

// Number of positions of the run list [r0, r1) whose time is <= until (times non-decreasing).
__device__ __forceinline__ uint32_t visible_positions(const TopicIndex& ti, uint32_t r0, uint32_t r1, int64_t until) {
  // last run whose first entry is visible
  uint32_t lo = r0, hi = r1;  // invariant: runs < lo visible, runs >= hi not
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ti.t[ti.entry[mid]] <= until) lo = mid + 1;
    else hi = mid;
  }
  if (lo == r0) return 0;
  const uint32_t j = lo - 1;
  const uint64_t e = ti.entry[j];
  uint32_t a = 1, b = ti.len[j];  // invariant: entries < a of the run visible (the first is), >= b not
  while (a < b) {
    const uint32_t mid = (a + b) >> 1;
    if (ti.t[e + mid] <= until) a = mid + 1;
    else b = mid;
  }
  return ti.pos0[j] - 1u + a;  // positions 1..pos0-1 (earlier runs) + a of run j
}

__global__ __launch_bounds__(kBlock) void k_sub_count(TopicIndex ti, uint32_t n, const uint32_t* __restrict__ topics,
                                                      const uint32_t* __restrict__ from,
                                                      const int64_t* __restrict__ until, uint32_t cap_each,
                                                      uint64_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i > n) return;
  if (i == n) { cnt[n] = 0; return; }
  const uint32_t k = topics[i], f = from[i];
  uint32_t c = 0;
  if (k < ti.n_topics && f >= 1) {
    const uint32_t last = visible_positions(ti, ti.run_off[k], ti.run_off[k + 1], until[i]);
    if (last >= f) c = min(last - f + 1u, cap_each);
  }
  cnt[i] = c;
}

// Runs are ordered by pos0 and tile positions 1..count: the run holding position p.
__device__ __forceinline__ uint32_t run_of(const TopicIndex& ti, uint32_t r0, uint32_t r1, uint32_t p) {
  uint32_t lo = r0, hi = r1;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ti.pos0[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

// out[q] = v + q for q < len by the block: 4-B stores up to a 16-B boundary, then 16-B stores.
__device__ __forceinline__ void fill_iota(uint32_t* out, uint32_t len, uint32_t v) {
  const uint32_t head = min(len, (uint32_t)((16u - ((uintptr_t)out & 15u)) & 15u) >> 2);
  if (threadIdx.x < head) out[threadIdx.x] = v + threadIdx.x;
  const uint32_t body = (len - head) >> 2;
  uint4* o4 = reinterpret_cast<uint4*>(out + head);
  const uint32_t vb = v + head;
  for (uint32_t q = threadIdx.x; q < body; q += kBlock) {
    const uint32_t x = vb + 4u * q;
    o4[q] = make_uint4(x, x + 1u, x + 2u, x + 3u);
  }
  const uint32_t done = head + 4u * body;
  if (threadIdx.x < len - done) out[done + threadIdx.x] = v + done + threadIdx.x;
}

__global__ __launch_bounds__(kBlock) void k_sub_fill(TopicIndex ti, uint32_t n, const uint32_t* __restrict__ topics,
                                                     const uint32_t* __restrict__ from,
                                                     const uint64_t* __restrict__ off, uint32_t* __restrict__ out,
                                                     uint64_t cap) {
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {  // block-uniform: every wave reaches the exit
    const uint64_t o = off[i];
    if (o >= cap) continue;
    const uint64_t m = min(off[i + 1] - o, cap - o);
    if (!m) continue;
    const uint32_t k = topics[i], r1 = ti.run_off[k + 1];
    uint32_t p = from[i];
    const uint32_t p_end = p + (uint32_t)m;  // m <= visible positions, so no wrap
    uint64_t w = o;
    for (uint32_t j = run_of(ti, ti.run_off[k], r1, p); p < p_end && j < r1; ++j) {
      const uint32_t q_end = min(p_end, ti.pos0[j] + ti.len[j]);
      const uint32_t e0 = (uint32_t)(ti.entry[j] + (p - ti.pos0[j]));
      const uint32_t len = q_end - p;
      fill_iota(out + w, len, e0);
      w += len;
      p = q_end;
    }
  }
}

inline unsigned blocks(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

}  // namespace

hipError_t launch_subscribe(Dev& d, const TopicIndex& ti, uint32_t n, const uint32_t* topics, const uint32_t* from,
                            const int64_t* until, uint32_t cap_each, uint64_t* cnt, void* scan_tmp, size_t scan_bytes,
                            uint64_t* offsets, uint32_t* entries, uint64_t entries_cap) {
  hipLaunchKernelGGL(k_sub_count, dim3(blocks((uint64_t)n + 1)), dim3(kBlock), 0, d.stream, ti, n, topics, from, until,
                     cap_each, cnt);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, cnt, offsets, n + 1, d.stream);
  if (e != hipSuccess || !entries || !entries_cap || !n) return e;
  hipLaunchKernelGGL(k_sub_fill, dim3(n < 16384u ? n : 16384u), dim3(kBlock), 0, d.stream, ti, n, topics, from,
                     (const uint64_t*)offsets, entries, (uint64_t)entries_cap);
  return hipGetLastError();
}

size_t subscribe_scan_bytes(uint32_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, n + 1);
  return bytes;
}

}  // namespace tgsim
