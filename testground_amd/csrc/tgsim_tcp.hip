// tgsim_tcp.hip — TCP mode (tgsim_tcp_*): segmentation and loss recovery over the
// per-packet path, for the reference plans that move data over TCP (plans/benchmarks/storm.go:
// 127-180, plans/network/pingpong.go:73-104). Packets are ordinary staged messages with
// seq = segment * 16 + attempt; after every window the reaction reads the window's packet statuses
// and deliveries where the pipeline left them:
//   k_tcp_status   per packet: the copies that entered the egress queue (status flags) are the
//                  attempt's copies (s_w bits 28-29, s_out); none: refused route (the write fails) or a
//                  retransmission at t_a + rto * 2^a. A segment is staged at most once per window
//                  (its next attempt is scheduled only once every copy is accounted for), so these are
//                  plain stores
//   k_tcp_arrive   per delivery. An attempt with one copy (the common case) has one delivery, whose
//                  thread alone settles the segment: intact -> the segment arrived (a one-segment
//                  write is delivered by one store of its time; the last segment of a longer one
//                  delivers it), corrupted -> retransmission at
//                  max(t_a + rto * 2^a, its arrival). A duplicated attempt's copies take atomics
//                  (first intact arrival, latest corrupted copy, one outstanding copy fewer) and
//                  append the segment to the settle list
//   k_tcp_settle   per duplicated delivery, one thread per segment (epoch claim): the same decision
//                  once the window's copies are counted
//   k_tcp_release  at the next window start: due retransmissions appended to the staged messages
//                  (device-side count), the rest kept for a later window
// Queue limit: a sender's pending retransmissions (pend_by, including those released into the open
// window until their packet is accounted) join its queue occupancy in the per-window test
// (Heavy::retx) and in the host's exact refresh, mult * (occupancy + pending): that bounds mult *
// (the sender's unsettled segments), which only new segments raise, so the host bound needs no
// read-back of the TCP state.
// Device-scope atomics execute at the memory side, one request per lane, so the common case uses
// none: a delivery reads one segment word (write, copies, one-segment flag) and stores the write's
// time; a write is delivered once its time is set. Every decision is order-independent: the result equals the oracle's
// sequential pass although threads race.
#include "tgsim_dev.h"

namespace tgsim {

namespace {

constexpr uint32_t kArrived = 0xFFFFFFFFu;  // s_mark of a duplicated segment that has arrived (above every epoch)
constexpr uint32_t kSoleSeg = 0x80000000u;  // s_w: the segment is its write's only one
constexpr uint32_t kWMask = 0x0FFFFFFFu;    // s_w: the write
constexpr uint32_t kQShift = 28;            // s_w: copies of the current attempt (2 bits)

__device__ __forceinline__ uint32_t tcp_copies(uint8_t st) {
  const uint32_t code = st & 0x0Fu;
  if (code == TGSIM_ST_LOCAL) return 1u;
  if (code != TGSIM_ST_QUEUED) return 0u;
  uint32_t q = (st & TGSIM_ST_FLAG_OVERLIMIT) ? 0u : 1u;
  if ((st & TGSIM_ST_FLAG_DUP) && !(st & TGSIM_ST_FLAG_CLONE_LOST)) ++q;
  return q;
}

// the write fails (earliest failure kept; the first transition from pending counts it)
__device__ __forceinline__ void tcp_fail(TcpDev& t, uint32_t w, int64_t tf, uint32_t state) {
  atomicMin(reinterpret_cast<long long*>(&t.w_fail[w]), (long long)(tf * 2 + (state == TGSIM_TCP_TIMEOUT ? 1 : 0)));
  if (atomicCAS(&t.w_state[w], (uint32_t)TGSIM_TCP_PENDING, state) == TGSIM_TCP_PENDING) {
    atomicAdd(&t.sc->done, 1u);
    atomicAdd(&t.sc->failed, 1ull);
  }
}

// attempt s_att[sid] failed, known at t_known: the next attempt (true: it joins the pending list), or
// the write times out
__device__ __forceinline__ bool tcp_next(TcpDev& t, uint32_t sid, int64_t t_known) {
  const uint32_t a = t.s_att[sid];
  int64_t tn = t.s_tatt[sid] + (t.rto << a);
  tn = tn < t_known ? t_known : tn;
  const uint32_t w = t.s_w[sid] & kWMask;
  if (a + 1u >= t.max_att) {
    tcp_fail(t, w, tn, TGSIM_TCP_TIMEOUT);
    return false;
  }
  t.s_att[sid] = a + 1u;
  t.s_tatt[sid] = tn;
  t.s_tlast[sid] = INT64_MIN;
  atomicAdd(&t.pend_by[t.w_src[w]], 1u);
  return true;
}

// Per-item kernels record their decisions as bits, one word per wave (lanes beyond the count are
// inactive, so their bits are 0): a hot counter updated per wave would serialise every wave on one
// address. k_tcp_collect turns the bits into list entries with one slot reservation per block.
__device__ __forceinline__ void put_bits(uint64_t* bm, uint32_t i, bool f) {
  const uint64_t b = __ballot(f);
  if (lane_id() == 0) bm[i >> 6] = b;
}

// block sum of v into part[blockIdx.x] (a plain store; k_tcp_collect adds the partials)
__device__ __forceinline__ void block_partial(uint32_t v, uint32_t* part) {
  __shared__ uint32_t red[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor(v, o);
  if (lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(kBlock) void k_tcp_status(const uint8_t* __restrict__ status,
                                                       const uint32_t* __restrict__ seq, uint32_t n_host,
                                                       const uint32_t* n_dev, TcpDev t) {
  const uint32_t n = n_dev ? *n_dev : n_host;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sq = seq[i], sid = sq >> 4;
    const uint8_t st = status[i];
    const uint32_t q = tcp_copies(st), code = st & 0x0Fu;
    bool retx = false;
    // a released retransmission leaves its sender's pending count once its packet is accounted
    if (sq & 15u) atomicSub(&t.pend_by[t.w_src[t.s_w[sid] & kWMask]], 1u);
    if (q) {
      t.s_out[sid] = q;
      t.s_w[sid] = (t.s_w[sid] & ~(3u << kQShift)) | (q << kQShift);
    } else if (code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) {
      tcp_fail(t, t.s_w[sid] & kWMask, t.s_tatt[sid], TGSIM_TCP_REFUSED);
    } else {
      retx = tcp_next(t, sid, t.s_tatt[sid]);
    }
    put_bits(t.bm_s, i, retx);
  }
}

// a segment of write sw (its s_w word) arrived intact at arr: 1 when that delivers the write. A write
// whose every segment arrived cannot fail, so its time alone marks it delivered
__device__ __forceinline__ uint32_t tcp_arrived(TcpDev& t, uint32_t sw, int64_t arr) {
  const uint32_t w = sw & kWMask;
  if (sw & kSoleSeg) {  // no other segment: nothing else writes the write's entries
    t.w_tarr[w] = arr;
    return 1u;
  }
  // running max, then the count; the last segment reads the max back after its count (the fences
  // order each thread's max before its count, and the counts are totally ordered)
  atomicMax(reinterpret_cast<long long*>(&t.w_tmax[w]), (long long)arr);
  __threadfence();
  if (atomicSub(&t.w_rem[w], 1u) != 1u) return 0u;
  __threadfence();
  const long long m = atomicMax(reinterpret_cast<long long*>(&t.w_tmax[w]), (long long)arr);
  t.w_tarr[w] = m > (long long)arr ? (int64_t)m : arr;
  return 1u;
}

__global__ __launch_bounds__(kBlock) void k_tcp_arrive(const uint32_t* __restrict__ o_seq,
                                                       const int64_t* __restrict__ o_t,
                                                       const uint32_t* __restrict__ o_flags, const DevScalars* sc,
                                                       TcpDev t) {
  const uint32_t n = sc->n_out;
  uint32_t ndel = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sid = o_seq[i] >> 4;
    const int64_t ti = o_t[i];
    const bool corrupt = o_flags[i] & TGSIM_F_CORRUPT;
    const uint32_t sw = t.s_w[sid];
    const bool sole = ((sw >> kQShift) & 3u) == 1u;
    bool retx = false;
    if (sole) {  // the attempt's only copy: this thread settles the segment
      if (!corrupt) ndel += tcp_arrived(t, sw, ti);
      else retx = tcp_next(t, sid, ti);
    } else {
      // a duplicated attempt: the latest copy matters only to a segment whose copies all arrived
      // corrupted; k_tcp_settle decides once the window's copies are counted
      if (!corrupt) atomicMin(reinterpret_cast<long long*>(&t.s_arr[sid]), (long long)ti);
      else atomicMax(reinterpret_cast<long long*>(&t.s_tlast[sid]), (long long)ti);
      atomicSub(&t.s_out[sid], 1u);
    }
    put_bits(t.bm_r, i, retx);
    put_bits(t.bm_d, i, !sole);
  }
  block_partial(ndel, t.part);
}

// duplicated deliveries (bm_d), one thread per segment and epoch; an arrived segment is never
// settled again. Few: these take direct list slots
__global__ __launch_bounds__(kBlock) void k_tcp_settle(const uint32_t* __restrict__ o_seq, const DevScalars* sc,
                                                       TcpDev t, uint32_t epoch, uint32_t cur) {
  const uint32_t nw = (sc->n_out + 63u) >> 6;
  uint32_t ndel = 0;
  for (uint32_t wi = blockIdx.x * kBlock + threadIdx.x; wi < nw; wi += gridDim.x * kBlock) {
    for (uint64_t m = t.bm_d[wi]; m; m &= m - 1) {
      const uint32_t sid = o_seq[wi * 64u + (uint32_t)__builtin_ctzll(m)] >> 4;
      if (atomicMax(&t.s_mark[sid], epoch) >= epoch) continue;
      const int64_t arr = t.s_arr[sid];
      if (arr != INT64_MAX) {
        t.s_mark[sid] = kArrived;
        ndel += tcp_arrived(t, t.s_w[sid], arr);
      } else if (t.s_out[sid] == 0 && tcp_next(t, sid, t.s_tlast[sid])) {
        t.pend[cur][atomicAdd(&t.sc->pend_n[cur], 1u)] = sid;
        atomicAdd(&t.sc->retx, 1ull);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ndel += (uint32_t)__shfl_xor(ndel, o);
  if (lane_id() == 0 && ndel) {
    atomicAdd(&t.sc->done, ndel);
    atomicAdd(&t.sc->delivered, (unsigned long long)ndel);
  }
}

// The window's retransmissions (bits over the packets, then over the deliveries) into the pending
// list: per block a scan of the words' bit counts and one slot reservation; and the delivered
// partials of k_tcp_arrive.
__global__ __launch_bounds__(kBlock) void k_tcp_collect(const uint32_t* __restrict__ m_seq, uint32_t n_host,
                                                        const uint32_t* n_dev, const uint32_t* __restrict__ o_seq,
                                                        const DevScalars* sc, TcpDev t, uint32_t cur,
                                                        uint32_t nparts) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sbase;
  const uint32_t ws = ((n_dev ? *n_dev : n_host) + 63u) >> 6, wr = (sc->n_out + 63u) >> 6, nw = ws + wr;
  uint32_t nretx = 0;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < nw; b0 += gridDim.x * kBlock) {  // uniform per block
    const uint32_t wi = b0 + threadIdx.x;
    uint64_t m = 0;
    const uint32_t* seq = m_seq;
    uint32_t i0 = wi * 64u;
    if (wi < ws) {
      m = t.bm_s[wi];
    } else if (wi < nw) {
      m = t.bm_r[wi - ws];
      seq = o_seq;
      i0 = (wi - ws) * 64u;
    }
    uint32_t tot;
    uint32_t p = block_excl_scan((uint32_t)__popcll(m), red, tot);
    if (threadIdx.x == 0 && tot) sbase = atomicAdd(&t.sc->pend_n[cur], tot);
    __syncthreads();
    p += sbase;
    for (; m; m &= m - 1) t.pend[cur][p++] = seq[i0 + (uint32_t)__builtin_ctzll(m)] >> 4;
    nretx += tot;
    __syncthreads();  // sbase is rewritten by the next round
  }
  uint32_t nd = 0;
  if (blockIdx.x == 0)
    for (uint32_t k = threadIdx.x; k < nparts; k += kBlock) nd += t.part[k];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nd += (uint32_t)__shfl_xor(nd, o);
  if (lane_id() == 0 && nd) {
    atomicAdd(&t.sc->done, nd);
    atomicAdd(&t.sc->delivered, (unsigned long long)nd);
  }
  if (threadIdx.x == 0 && nretx) atomicAdd(&t.sc->retx, (unsigned long long)nretx);
}

__global__ __launch_bounds__(kBlock) void k_tcp_reset(TcpDev t, uint32_t cur) {
  if (threadIdx.x == 0) { t.sc->done = 0; t.sc->pend_n[cur ^ 1u] = 0; }
}

__global__ __launch_bounds__(kBlock) void k_tcp_base(DevScalars* sc, uint32_t base_host) {
  if (threadIdx.x == 0) sc->n_msgs_dev = base_host;
}

__global__ __launch_bounds__(kBlock) void k_tcp_release(TcpDev t, uint32_t cur, DevScalars* sc, uint32_t cap,
                                                        uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                        uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                        int64_t* __restrict__ m_t) {
  const uint32_t n = t.sc->pend_n[cur], nxt = cur ^ 1u;
  const int64_t t_end = sc->t_end;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sid = t.pend[cur][i], w = t.s_w[sid] & kWMask;
    const int64_t ta = t.s_tatt[sid];
    if (t.w_state[w] == TGSIM_TCP_PENDING && ta >= t_end) {
      t.pend[nxt][atomicAdd(&t.sc->pend_n[nxt], 1u)] = sid;
      continue;
    }
    if (t.w_state[w] != TGSIM_TCP_PENDING) {  // the write has failed: nothing more is sent
      atomicSub(&t.pend_by[t.w_src[w]], 1u);
      continue;
    }
    const uint32_t p = atomicAdd(&sc->n_msgs_dev, 1u);
    if (p >= cap) {
      atomicOr(&sc->err, ERR_CAP_M);
      continue;
    }
    m_src[p] = t.w_src[w]; m_dst[p] = t.w_dst[w]; m_seq[p] = (sid << 4) | t.s_att[sid]; m_size[p] = t.s_wire[sid];
    m_t[p] = ta;
    atomicAdd(&t.sc->released, 1ull);
  }
}

// A generated storm round (staged [base, base + n)) becomes TCP writes: one segment each.
__global__ __launch_bounds__(kBlock) void k_tcp_adopt(TcpDev t, uint32_t base, uint32_t n, uint32_t wbase,
                                                      uint32_t sbase, uint32_t* __restrict__ m_src,
                                                      uint32_t* __restrict__ m_dst, uint32_t* __restrict__ m_seq,
                                                      uint32_t* __restrict__ m_size, const int64_t* __restrict__ m_t) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t m = base + i, w = wbase + i, sid = sbase + i;
    t.w_src[w] = m_src[m]; t.w_dst[w] = m_dst[m]; t.w_rem[w] = 1u;
    t.s_w[sid] = w | kSoleSeg; t.s_wire[sid] = m_size[m] + t.hdr; t.s_tatt[sid] = m_t[m];
    m_seq[m] = sid << 4;
    m_size[m] += t.hdr;
  }
}

}  // namespace

hipError_t launch_tcp_adopt(Dev& d, TcpDev& t, uint32_t base, uint32_t n, uint32_t wbase, uint32_t sbase) {
  if (!n) return hipSuccess;
  const unsigned g = std::min<unsigned>((n + kBlock - 1) / kBlock, (unsigned)kStreamBlocks);
  hipLaunchKernelGGL(k_tcp_adopt, dim3(g), dim3(kBlock), 0, d.stream, t, base, n, wbase, sbase, d.m_src, d.m_dst,
                     d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_tcp_react(Dev& d, TcpDev& t, uint32_t cur, uint32_t n_host, const uint32_t* n_dev, uint32_t epoch) {
  hipLaunchKernelGGL(k_tcp_reset, dim3(1), dim3(kBlock), 0, d.stream, t, cur);
  hipLaunchKernelGGL(k_tcp_status, dim3(kStreamBlocks), dim3(kBlock), 0, d.stream, d.status, d.m_seq, n_host, n_dev, t);
  hipLaunchKernelGGL(k_tcp_arrive, dim3(kTcpArriveBlocks), dim3(kBlock), 0, d.stream, d.o_seq, d.o_t, d.o_flags, d.sc, t);
  hipLaunchKernelGGL(k_tcp_settle, dim3(64), dim3(kBlock), 0, d.stream, d.o_seq, d.sc, t, epoch, cur);
  hipLaunchKernelGGL(k_tcp_collect, dim3(64), dim3(kBlock), 0, d.stream, d.m_seq, n_host, n_dev, d.o_seq, d.sc, t, cur,
                     (uint32_t)kTcpArriveBlocks);
  return hipGetLastError();
}

hipError_t launch_tcp_release(Dev& d, TcpDev& t, uint32_t cur, bool base_dev, uint32_t base_host) {
  if (!base_dev) hipLaunchKernelGGL(k_tcp_base, dim3(1), dim3(kBlock), 0, d.stream, d.sc, base_host);
  // the pending count is device-side: a fixed grid, grid-stride
  hipLaunchKernelGGL(k_tcp_release, dim3(256), dim3(kBlock), 0, d.stream, t, cur, d.sc, d.cap_msgs, d.m_src,
                     d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

}  // namespace tgsim
