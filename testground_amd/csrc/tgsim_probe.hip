// tgsim_probe.hip — device side of the sequential probes (tgsim_probe_*): every
// local instance probes the instances of `order` one at a time, as plans/splitbrain/main.go:153-175
// does with one httpclient.Get after another (Timeout: 1 minute). Oracle twin: tgo_probe_*.
//
// After each window, with no host round trip:
//   k_probe_pre     per staged packet of the window: a request its prober's route refused
//                   (blackhole / prohibit / no route) ends the probe at its send time; per delivery:
//                   a request at its peer - a position of its prober beyond the last one answered
//                   here: the highest such position and its copies' first arrival (atomicMax /
//                   atomicMin) - and the reply's first arrival at its prober
//   k_probe_step    per prober: the reply its peer owes (at max(arrival, horizon); on one shard the
//                   prober's thread answers for the peer), the probe's end (refused / reply before the
//                   deadline / deadline passed), the next request; the staged slots reserved once per
//                   block behind sc->n_msgs_dev; the last workgroup proposes the next window's end (one
//                   window_ns while messages are staged or in flight, else the earliest deadline + 1)
//   sharded: k_probe_answer (the peers answer, listed by k_probe_pre) before the step, its notices
//   to the probers' shards through the exchange blocks (k_probe_notices), the proposal collective
// A prober's state lives in its own slots on its shard; the answering state per prober on every
// shard. The only shared updates are the arrival extrema, the notices and the reservations.
#include <algorithm>

#include "tgsim_dev.h"

namespace tgsim {

namespace {

constexpr uint32_t kTagMask = 0x3FFFFFFFu;
constexpr uint64_t kArrSpan = 1ull << 40;  // request arrivals packed relative to the window end (answer)
constexpr int64_t kNone = INT64_MAX;
enum : uint8_t { kIdle = 0, kWait = 1, kDone = 2 };

// the next position after pos (pos = ~0u: the first) whose instance is not the prober g
__device__ __forceinline__ uint32_t next_pos(const ProbeDev& p, uint32_t g, uint32_t pos) {
  uint32_t j = pos == ~0u ? 0u : pos + 1u;
  while (j < p.n_order && p.order[j] == g) ++j;
  return j;
}

__global__ void k_probe_base(DevScalars* sc, uint32_t base_host) { sc->n_msgs_dev = base_host; }


// Stage up to two messages per thread (a reply, then a request) with one reservation per block.
struct Staged {
  uint32_t src[2], dst[2], seq[2], size[2];
  int64_t t[2];
  uint32_t n = 0;
  __device__ void add(uint32_t s, uint32_t d, uint32_t q, uint32_t z, int64_t tt) {
    src[n] = s; dst[n] = d; seq[n] = q; size[n] = z; t[n] = tt; ++n;
  }
};

__device__ __forceinline__ void flush_block(const Staged& st, uint32_t* red, uint32_t* sbase, DevScalars* sc,
                                            uint32_t cap, uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                            uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                            int64_t* __restrict__ m_t) {
  uint32_t tot;
  const uint32_t ex = block_excl_scan(st.n, red, tot);
  if (threadIdx.x == 0) *sbase = tot ? reserve_staged(&sc->n_msgs_dev, tot, cap) : 0u;
  __syncthreads();
  for (uint32_t k = 0; k < st.n; ++k) {
    const uint32_t w = *sbase + ex + k;
    if (w < cap) {
      m_src[w] = st.src[k]; m_dst[w] = st.dst[k]; m_seq[w] = st.seq[k]; m_size[w] = st.size[k]; m_t[w] = st.t[k];
    } else {
      atomicOr(&sc->err, ERR_CAP_M);
    }
  }
  __syncthreads();  // sbase is rewritten by the next round
}

// per block: the minimum deadline of its waiting probers and their count
__device__ __forceinline__ void block_waiting(ProbeDev& p, int64_t dl, uint32_t waiting) {
  __shared__ int64_t s_dl[kBlock / 64];
  __shared__ uint32_t s_n[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_xor(dl, o);
    dl = y < dl ? y : dl;
    waiting += (uint32_t)__shfl_xor(waiting, o);
  }
  if (lane_id() == 0) { s_dl[threadIdx.x >> 6] = dl; s_n[threadIdx.x >> 6] = waiting; }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t m = s_dl[0];
    uint32_t n = s_n[0];
    for (int w = 1; w < kBlock / 64; ++w) { m = s_dl[w] < m ? s_dl[w] : m; n += s_n[w]; }
    if (m != kNone) atomicMin(reinterpret_cast<long long*>(&p.sc->min_dl), (long long)m);
    if (n) atomicAdd(&p.sc->active, n);
  }
}

// the previous probe of prober l ended at te: probe pos leaves at max(te, H); or l has no probe left
// and is done at te
__device__ __forceinline__ void begin_probe(ProbeDev& p, uint32_t l, uint32_t g, uint32_t pos, int64_t te, int64_t H,
                                            Staged& st) {
  if (pos >= p.n_order) {
    p.state[l] = kDone;
    p.t_done[l] = te;
    p.pos[l] = p.n_order;
    return;
  }
  const int64_t t = te > H ? te : H;
  p.state[l] = kWait;
  p.pos[l] = pos;
  p.t_req[l] = t;
  p.refused[l] = 0;
  p.replied[l] = 0;
  p.t_reparr[l] = kNone;
  st.add(g, p.order[pos], TGSIM_PROBE_REQ | pos, p.req_bytes, t);
}

__global__ __launch_bounds__(kBlock) void k_probe_start(ProbeDev p, DevScalars* sc, uint32_t lo, uint32_t nloc,
                                                        int64_t t0, uint32_t cap, uint32_t* __restrict__ m_src,
                                                        uint32_t* __restrict__ m_dst, uint32_t* __restrict__ m_seq,
                                                        uint32_t* __restrict__ m_size, int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sbase;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < nloc; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t l = b0 + threadIdx.x;
    Staged st;
    if (l < nloc && p.state[l] == kIdle) begin_probe(p, l, lo + l, next_pos(p, lo + l, ~0u), t0, t0, st);
    flush_block(st, red, &sbase, sc, cap, m_src, m_dst, m_seq, m_size, m_t);
  }
}

__device__ __forceinline__ void probe_status(const uint8_t* __restrict__ status, const uint32_t* __restrict__ m_src,
                                             const uint32_t* __restrict__ m_dst, const uint32_t* __restrict__ m_seq,
                                             uint32_t n_host, const uint32_t* n_dev, ProbeDev& p, uint32_t lo,
                                             uint32_t bid, uint32_t nb) {
  const uint32_t n = n_dev ? *n_dev : n_host;
  for (uint32_t i = bid * kBlock + threadIdx.x; i < n; i += nb * kBlock) {
    const uint32_t sq = m_seq[i];
    if ((sq >> 30) != 1u) continue;
    const uint32_t code = status[i] & 0x0Fu;
    if (code != TGSIM_ST_DROPPED && code != TGSIM_ST_REJECTED && code != TGSIM_ST_UNREACHABLE) continue;
    const uint32_t l = m_src[i] - lo;
    if (p.state[l] == kWait && p.pos[l] == (sq & kTagMask) && p.order[sq & kTagMask] == m_dst[i]) p.refused[l] = 1;
  }
}

__device__ __forceinline__ void probe_arrive(const uint32_t* __restrict__ o_src, const uint32_t* __restrict__ o_dst,
                                             const uint32_t* __restrict__ o_seq, const int64_t* __restrict__ o_t,
                                             const DevScalars* sc, ProbeDev& p, uint32_t lo, uint32_t bid,
                                             uint32_t nb) {
  const uint32_t n = sc->n_out;
  for (uint32_t i0 = bid * kBlock; i0 < n; i0 += nb * kBlock) {  // wave-uniform trip count
    const uint32_t i = i0 + threadIdx.x;
    bool listed = false;
    uint32_t g = 0;
    if (i < n) {
      const uint32_t sq = o_seq[i], tag = sq >> 30;
      if (tag == 1u) {  // a request at its peer (a position beyond the last one answered here)
        const uint32_t j = sq & kTagMask;
        g = o_src[i];
        if (g < p.N && j < p.n_order && p.order[j] == o_dst[i] && j + 1u > p.ans[g]) {
          const uint32_t old = atomicMax(&p.cur[g], j + 1u);
          // the highest position, and the first arrival of that position's request only: a request
          // j delayed past its timeout that lands in the window of request j + 1 does not stamp
          // j + 1's reply before j + 1 arrived
          const uint64_t off = (uint64_t)(sc->t_end - 1 - o_t[i]);  // >= 0: delivered in this window
          if (off >= kArrSpan) atomicOr(const_cast<uint32_t*>(&sc->err), ERR_PROBE_SPAN);
          atomicMax(reinterpret_cast<unsigned long long*>(&p.rqa[g]),
                    (unsigned long long)(((uint64_t)(j + 1u) << 40) | min(off, kArrSpan - 1u)));  // max off = first
          listed = old == 0u && p.S > 1;
        }
      } else if (tag == 3u && (sq & kTagMask) == o_dst[i]) {  // a reply at its prober
        const uint32_t l = o_dst[i] - lo;
        if (p.state[l] == kWait && p.replied[l] && p.order[p.pos[l]] == o_src[i])
          atomicMin(reinterpret_cast<long long*>(&p.t_reparr[l]), (long long)o_t[i]);
      }
    }
    const uint64_t lm = __ballot(listed);  // sharded: the probers to answer, one reservation per wave
    if (lm) {
      const int leader = __ffsll((unsigned long long)lm) - 1;
      uint32_t base = 0;
      if ((int)lane_id() == leader) base = atomicAdd(&p.sc->n_ans, (uint32_t)__popcll(lm));
      base = __shfl(base, leader);
      if (listed) p.alist[base + mask_rank(lm)] = g;
    }
  }
}

// The reaction's first launch: the window's refused requests (blocks [0, nb)) and first arrivals
// (blocks [nb, 2 nb)) are independent of each other; block 0 also resets the step's reductions and
// (host-counted staging) sets the staged base - four launches of ~5 us each became one.
__global__ __launch_bounds__(kBlock) void k_probe_pre(const uint8_t* __restrict__ status,
                                                      const uint32_t* __restrict__ m_src,
                                                      const uint32_t* __restrict__ m_dst,
                                                      const uint32_t* __restrict__ m_seq, uint32_t n_host,
                                                      const uint32_t* n_dev, const uint32_t* __restrict__ o_src,
                                                      const uint32_t* __restrict__ o_dst,
                                                      const uint32_t* __restrict__ o_seq,
                                                      const int64_t* __restrict__ o_t, DevScalars* sc, ProbeDev p,
                                                      uint32_t lo, uint32_t nb, uint32_t set_base, uint32_t base_host) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.sc->min_dl = kNone;
    p.sc->active = 0;
    p.sc->done = 0;
    if (set_base) sc->n_msgs_dev = base_host;  // nothing in this launch reads it
  }
  if (blockIdx.x < nb) probe_status(status, m_src, m_dst, m_seq, n_host, n_dev, p, lo, blockIdx.x, nb);
  else probe_arrive(o_src, o_dst, o_seq, o_t, sc, p, lo, blockIdx.x - nb, nb);
}

__device__ __forceinline__ void probe_end(ProbeDev& p, const DevScalars* sc);

// On the prober's shard: its current request `pos` was answered with a reply sent at t
__device__ __forceinline__ void reply_staged(ProbeDev& p, uint32_t g, uint32_t pos, int64_t t) {
  const uint32_t l = g - p.lo;
  if (g < p.lo || l >= p.nloc || p.state[l] != kWait || p.pos[l] != pos) return;  // moved past it
  p.replied[l] = 2;
  p.t_rep[l] = t;
}

// The peer answers prober g's highest new request: the reply at max(first arrival, horizon), staged
// in st; returns the answered position. The prober's shard learns of it (reply_staged) here on one
// shard, by a notice when sharded.
__device__ __forceinline__ uint32_t answer(ProbeDev& p, uint32_t g, int64_t H, int64_t t_end, Staged& st) {
  const uint64_t key = p.rqa[g];  // (position + 1, first arrival) of the highest position (probe_arrive)
  const uint32_t j = (uint32_t)(key >> 40) - 1u;
  const int64_t ra = t_end - 1 - (int64_t)(key & (kArrSpan - 1u));
  const int64_t trep = ra > H ? ra : H;
  st.add(p.order[j], g, TGSIM_PROBE_REP | g, p.rep_bytes, trep);
  p.ans[g] = j + 1u;
  p.cur[g] = 0;
  p.rqa[g] = 0;
  if (p.S == 1) reply_staged(p, g, j, trep);
  return j;
}

constexpr uint32_t kNoticeReply = 3u;

// Sharded: the local peers answer the probers listed by k_probe_pre; notices to their shards
__global__ __launch_bounds__(kBlock) void k_probe_answer(ProbeDev p, DevScalars* sc, uint32_t cap,
                                                         uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                         uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                         int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sbase;
  const uint32_t n = p.sc->n_ans;
  const int64_t H = sc->T, t_end = sc->t_end;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < n; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t i = b0 + threadIdx.x;
    Staged st;
    uint32_t g = 0, j = 0, peer = kNoPeer;
    int64_t trep = 0;
    if (i < n) {
      g = p.alist[i];
      j = answer(p, g, H, t_end, st);
      trep = st.t[0];
      const uint32_t k = shard_of(g, p.N, p.S);
      if (k == p.shard) reply_staged(p, g, j, trep);
      else peer = k;
    }
    notice_push(p.xq, p.xsend, p.xcap, sc, peer, g, j, kNoticeReply, trep);
    flush_block(st, red, &sbase, sc, cap, m_src, m_dst, m_seq, m_size, m_t);
  }
}

__global__ void k_probe_xheaders(ProbeDev p) {
  const uint32_t k = threadIdx.x;
  if (k >= p.S) return;
  const uint32_t n = min(p.xq[k << 5], p.xcap - 1);
  tgsim_record h;
  h.t = (int64_t)n; h.src = h.dst = h.seq = h.size = h.meta = h.corrupt_off = 0;
  p.xsend[(size_t)k * p.xcap] = h;
}

__global__ __launch_bounds__(kBlock) void k_probe_notices(DevScalars* sc, ProbeDev p) {
  const uint64_t total = (uint64_t)p.S * p.xcap;
  for (uint64_t x = (uint64_t)blockIdx.x * kBlock + threadIdx.x; x < total; x += (uint64_t)gridDim.x * kBlock) {
    const uint32_t k = (uint32_t)(x / p.xcap), i = (uint32_t)(x % p.xcap);
    if (k == p.shard || i == 0) continue;
    const int64_t n = p.xrecv[(size_t)k * p.xcap].t;
    if (n < 0 || n >= (int64_t)p.xcap) {
      if (i == 1) atomicOr(&sc->err, ERR_EXCH_HDR);
      continue;
    }
    if ((int64_t)i > n) continue;
    const tgsim_record r = p.xrecv[x];
    if (r.seq == kNoticeReply) reply_staged(p, r.src, r.dst, r.t);
  }
}

__global__ __launch_bounds__(kBlock) void k_probe_step(ProbeDev p, DevScalars* sc, uint32_t lo, uint32_t nloc,
                                                       uint32_t cap, uint32_t* __restrict__ m_src,
                                                       uint32_t* __restrict__ m_dst, uint32_t* __restrict__ m_seq,
                                                       uint32_t* __restrict__ m_size, int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sbase;
  const int64_t H = sc->T, t_end = sc->t_end;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < nloc; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t l = b0 + threadIdx.x;
    Staged st;
    int64_t dl_wait = kNone;
    uint32_t waiting = 0;
    if (l < nloc && p.S == 1 && p.cur[l]) answer(p, lo + l, H, t_end, st);  // one shard: for the peer
    if (l < nloc && p.state[l] == kWait) {
      const uint32_t g = lo + l, pos = p.pos[l];
      const int64_t tr = p.t_req[l], dl = tr + p.timeout, ra = p.t_reparr[l];
      // a reply staged now, before the deadline, may still beat it: its arrival decides next window
      // (a request arriving within one window of the deadline is not a timeout)
      const uint8_t rp = p.replied[l];
      const bool reply_pending = rp == 2 && p.t_rep[l] < dl;
      if (rp == 2) p.replied[l] = 1;
      uint8_t out = TGSIM_PROBE_NONE;
      int64_t te = 0;
      if (p.refused[l]) { out = TGSIM_PROBE_REFUSED; te = tr; }
      else if (ra != kNone && ra < dl) { out = TGSIM_PROBE_OK; te = ra; }
      else if (dl < t_end && !reply_pending) { out = TGSIM_PROBE_TIMEOUT; te = dl; }
      if (out != TGSIM_PROBE_NONE) {
        p.out[(size_t)l * p.n_order + pos] = out;
        begin_probe(p, l, g, next_pos(p, g, pos), te, H, st);
      }
      if (p.state[l] == kWait) {
        waiting = 1;
        dl_wait = p.t_req[l] + p.timeout;
      }
    }
    flush_block(st, red, &sbase, sc, cap, m_src, m_dst, m_seq, m_size, m_t);
    block_waiting(p, dl_wait, waiting);
  }
  // the last workgroup to finish proposes the next window's end (the former k_probe_end launch)
  __shared__ uint32_t s_last;
  if (block_release_for_count()) s_last = atomicAdd(&p.sc->done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(s_last) && threadIdx.x == 0) {
    fence_acquire_agent();
    probe_end(p, sc);
  }
}

// every k_probe_step workgroup's reductions and reservations are done: the counters are read with
// device-scope atomic loads (another XCD's L2 may hold the lines)
__device__ __forceinline__ void probe_end(ProbeDev& p, const DevScalars* sc) {
  const int64_t t_end = sc->t_end;
  int64_t ne = t_end + p.window;
  const uint32_t act = __hip_atomic_load(&p.sc->active, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t m = __hip_atomic_load(&p.sc->min_dl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t staged = __hip_atomic_load(const_cast<uint32_t*>(&sc->n_msgs_dev), __ATOMIC_ACQUIRE,
                                            __HIP_MEMORY_SCOPE_AGENT);
  const bool busy = staged != 0 || sc->arena_used != 0;
  if (!busy && act && m != kNone && m + 1 > ne) ne = m + 1;
  p.sc->next_end = ne;
  p.sc->n_active = act;
  p.sc->prop[0] = busy ? 1 : 0;  // sharded: the same rule over every shard's inputs (k_probe_prop)
  p.sc->prop[1] = act;
  p.sc->prop[2] = m;
}

__global__ void k_probe_prop(ProbeDev p, const DevScalars* sc) {
  if (threadIdx.x != 0) return;
  int64_t busy = 0, act = 0, m = kNone;
  for (uint32_t k = 0; k < p.S; ++k) {
    busy |= p.prop_all[3 * k];
    act += p.prop_all[3 * k + 1];
    m = p.prop_all[3 * k + 2] < m ? p.prop_all[3 * k + 2] : m;
  }
  int64_t ne = sc->t_end + p.window;
  if (!busy && act && m != kNone && m + 1 > ne) ne = m + 1;
  p.sc->next_end = ne;
  p.sc->n_active = (uint32_t)act;
}

unsigned grid_for(uint32_t n) {
  return std::max(1u, std::min<unsigned>((n + kBlock - 1) / kBlock, (unsigned)kStreamBlocks));
}

}  // namespace

hipError_t launch_probe_start(Dev& d, bool base_dev, uint32_t base_host, int64_t t0) {
  if (!base_dev) hipLaunchKernelGGL(k_probe_base, dim3(1), dim3(1), 0, d.stream, d.sc, base_host);
  hipLaunchKernelGGL(k_probe_start, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, d.pr, d.sc, d.lo, d.nloc, t0,
                     d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_probe_react(Dev& d, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                              const uint32_t* n_status_dev) {
  ProbeDev& p = d.pr;
  ProfScope ps_(d, KID_PROBE);
  constexpr uint32_t nb = kStreamBlocks / 2;
  hipLaunchKernelGGL(k_probe_pre, dim3(2 * nb), dim3(kBlock), 0, d.stream, d.status, d.m_src, d.m_dst, d.m_seq,
                     n_status_host, n_status_dev, d.o_src, d.o_dst, d.o_seq, d.o_t, d.sc, p, d.lo, nb,
                     base_dev ? 0u : 1u, base_host);
  hipLaunchKernelGGL(k_probe_step, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, p, d.sc, d.lo, d.nloc,
                     d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_probe_react_pre(Dev& d, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                                  const uint32_t* n_status_dev) {
  ProbeDev& p = d.pr;
  ProfScope ps_(d, KID_PROBE);
  constexpr uint32_t nb = kStreamBlocks / 2;
  if (hipMemsetAsync(&p.sc->n_ans, 0, sizeof(uint32_t), d.stream) != hipSuccess) return hipGetLastError();
  if (hipMemsetAsync(p.xq, 0, (size_t)p.S * 128, d.stream) != hipSuccess) return hipGetLastError();
  hipLaunchKernelGGL(k_probe_pre, dim3(2 * nb), dim3(kBlock), 0, d.stream, d.status, d.m_src, d.m_dst, d.m_seq,
                     n_status_host, n_status_dev, d.o_src, d.o_dst, d.o_seq, d.o_t, d.sc, p, d.lo, nb,
                     base_dev ? 0u : 1u, base_host);
  hipLaunchKernelGGL(k_probe_answer, dim3(grid_for(p.N)), dim3(kBlock), 0, d.stream, p, d.sc, d.cap_msgs, d.m_src,
                     d.m_dst, d.m_seq, d.m_size, d.m_t);
  hipLaunchKernelGGL(k_probe_xheaders, dim3(1), dim3(kMaxShards), 0, d.stream, p);
  return hipGetLastError();
}

hipError_t launch_probe_react_post(Dev& d) {
  ProbeDev& p = d.pr;
  ProfScope ps_(d, KID_PROBE);
  const uint64_t total = (uint64_t)p.S * p.xcap;
  hipLaunchKernelGGL(k_probe_notices, dim3(grid_for((uint32_t)std::min<uint64_t>(total, 0xFFFFFFFFu))), dim3(kBlock), 0,
                     d.stream, d.sc, p);
  hipLaunchKernelGGL(k_probe_step, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, p, d.sc, d.lo, d.nloc,
                     d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_probe_prop(Dev& d) {
  hipLaunchKernelGGL(k_probe_prop, dim3(1), dim3(64), 0, d.stream, d.pr, d.sc);
  return hipGetLastError();
}

}  // namespace tgsim
