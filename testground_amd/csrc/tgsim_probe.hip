// tgsim_probe.hip — device side of the sequential probes (tgsim_probe_*): every
// local instance probes the instances of `order` one at a time, as plans/splitbrain/main.go:153-175
// does with one httpclient.Get after another (Timeout: 1 minute). Oracle twin: tgo_probe_*.
//
// After each window, with no host round trip:
//   k_probe_status  per staged packet of the window: a request its prober's route refused
//                   (blackhole / prohibit / no route) ends the probe at its send time
//   k_probe_arrive  per delivery: the first arrival of the current request at its peer and of the
//                   reply at the prober (atomicMin: the earliest copy whatever thread sees it)
//   k_probe_step    per prober: the reply its peer owes (at max(arrival, horizon)), the probe's end
//                   (refused / reply before the deadline / deadline passed), the next request; the
//                   staged slots reserved once per block behind sc->n_msgs_dev
//   k_probe_end     one thread: the next window's proposed end (one window_ns while messages are
//                   staged or in flight, else the earliest deadline + 1)
// A prober's state lives in its own slots (one thread writes them in k_probe_step); the only shared
// updates are the arrival minima and the per-block reservation.
#include <algorithm>

#include "tgsim_dev.h"

namespace tgsim {

namespace {

constexpr uint32_t kTagMask = 0x3FFFFFFFu;
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
  p.t_reqarr[l] = kNone;
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
  for (uint32_t i = bid * kBlock + threadIdx.x; i < n; i += nb * kBlock) {
    const uint32_t sq = o_seq[i], tag = sq >> 30;
    if (tag == 1u) {  // a request at its peer
      const uint32_t l = o_src[i] - lo, j = sq & kTagMask;
      if (p.state[l] == kWait && p.pos[l] == j && p.order[j] == o_dst[i])
        atomicMin(reinterpret_cast<long long*>(&p.t_reqarr[l]), (long long)o_t[i]);
    } else if (tag == 3u && (sq & kTagMask) == o_dst[i]) {  // a reply at its prober
      const uint32_t l = o_dst[i] - lo;
      if (p.state[l] == kWait && p.replied[l] && p.order[p.pos[l]] == o_src[i])
        atomicMin(reinterpret_cast<long long*>(&p.t_reparr[l]), (long long)o_t[i]);
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
    if (l < nloc && p.state[l] == kWait) {
      const uint32_t g = lo + l, pos = p.pos[l];
      const int64_t rq = p.t_reqarr[l];
      const int64_t tr = p.t_req[l], dl = tr + p.timeout, ra = p.t_reparr[l];
      // a reply staged now, before the deadline, may still beat it: its arrival decides next window
      // (a request arriving within one window of the deadline is not a timeout)
      bool reply_pending = false;
      if (rq != kNone && !p.replied[l]) {  // the peer answers the request's first arrival
        const int64_t trep = rq > H ? rq : H;
        st.add(p.order[pos], g, TGSIM_PROBE_REP | g, p.rep_bytes, trep);
        p.replied[l] = 1;
        reply_pending = trep < dl;
      }
      p.t_reqarr[l] = kNone;
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
  if (staged == 0 && sc->arena_used == 0 && act && m != kNone && m + 1 > ne) ne = m + 1;
  p.sc->next_end = ne;
  p.sc->n_active = act;
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

}  // namespace tgsim
