// tgsim_storm.hip — device side of the storm plan reactor (tgsim_storm_*): the dial
// and write pacing of plans/benchmarks/storm.go:117-190 for every instance at once, so a storm plan
// run costs the host O(1) per window whatever its instance count. Oracle twin: tgo_storm_*.
//
// After each window, with no host round trip:
//   k_storm_pre    blocks [0, nb): the window's staged packets - a SYN its dialler's route refused,
//                  a chunk that failed (no copy queued: its buffer slot frees, its instance failed);
//                  blocks [nb, 2 nb): the window's deliveries - a SYN's first arrival at its listener
//                  (atomicMin; the connection listed to be answered), a SYN-ACK's at its dialler, a
//                  chunk's arrival (to its dialler: the first copy of a written chunk frees a buffer
//                  slot, by a claim bit); block 0 also resets the step's reductions
//   k_storm_answer the listeners answer the listed SYNs: a SYN-ACK at max(first arrival, horizon) each,
//                  and a notice of it to the dialler (its timeout waits a window if the SYN-ACK may
//                  still beat the deadline)
//   (sharded: the notices for other shards' diallers cross in the exchange blocks, k_storm_notices
//    applies them; on one shard a notice is applied where it is made)
//   k_storm_step   one thread per instance: dial phase - each waiting dial's end (refused / SYN-ACK
//                  before the deadline / deadline passed), then the dial semaphore's FIFO admits dials
//                  into the free slots (those due before the next window's end); write phase - the
//                  writesem round (storm.go:158-183) over the room the buffers have; the staged slots
//                  reserved once per block behind sc->n_msgs_dev; the last workgroup proposes the next
//                  window's end (sharded: every shard's proposal inputs are gathered, k_storm_prop)
// A connection's dialler state lives on its instance's shard, written by its instance's thread; its
// listener state (the SYN's first arrival, answered) on its peer's. The only shared updates are the
// arrival minima, the claim bits, the buffer counts, the notices and the per-block reductions.
#include <algorithm>

#include "tgsim_dev.h"

namespace tgsim {

namespace {

constexpr uint32_t kTagMask = 0x3FFFFFFFu;
constexpr int64_t kNone = INT64_MAX;
constexpr int64_t kBusy = INT64_MAX;  // a held semaphore slot
enum : uint8_t { kSleep = 0, kWait = 1, kDone = 2 };
enum : uint32_t { kEmitSyn = 2u };  // (the listener's SYN-ACKs are staged by k_storm_answer)
enum : uint32_t { kModeStart = 0, kModeReact = 1, kModeWrites = 2 };

__device__ __forceinline__ bool failed_code(uint32_t st) {
  const uint32_t code = st & 0x0Fu;
  return code != TGSIM_ST_QUEUED && code != TGSIM_ST_LOCAL;
}
__device__ __forceinline__ bool refused_code(uint32_t st) {
  const uint32_t code = st & 0x0Fu;
  return code == TGSIM_ST_DROPPED || code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE;
}

// per block: the sum of v into *dst with one atomic
__device__ __forceinline__ void block_add(unsigned long long* dst, unsigned long long v, unsigned long long* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if (lane_id() == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += red[w];
    if (t) atomicAdd(dst, t);
  }
  __syncthreads();
}

// The connection a chunk packet (src -> dst, chunk id c = k * nchunks + j) belongs to on its
// dialler's shard, or kNoConn when no written chunk of the storm matches it (a message the
// host staged beside the reactor with the chunk tag must not index past the tables or free another
// chunk's buffer slot). rem[h] is not written before k_storm_step, so "written" is the count before
// this reaction.
constexpr size_t kNoConn = ~(size_t)0;
__device__ __forceinline__ size_t chunk_conn(const StormDev& s, uint32_t src, uint32_t dst, uint32_t c) {
  if (s.nchunks == 0) return kNoConn;
  const uint32_t k = c / s.nchunks, j = c - k * s.nchunks;
  const size_t h = (size_t)src * s.O + k;
  if (k >= s.O || h >= s.n_conn || s.dst[h] != dst || j >= s.nchunks - s.rem[h]) return kNoConn;
  return h;
}

// Notices to a connection's dialler (records: t = value, src = connection, seq = kind)
enum : uint32_t { kNoticeSynAck = 1u, kNoticeChunk = 2u };

// on the dialler's shard: chunk j of connection h arrived (its first copy frees a buffer slot);
// returns 1 when it counted
__device__ __forceinline__ uint32_t chunk_arrived(StormDev& s, size_t h, uint32_t j) {
  if (h >= s.n_conn || s.nchunks == 0 || j >= s.nchunks) return 0u;
  if (chunk_conn(s, (uint32_t)(h / s.O), s.dst[h], (uint32_t)(h % s.O) * s.nchunks + j) == kNoConn) return 0u;
  const uint64_t bit = (uint64_t)h * s.nchunks + j;
  const uint32_t m = 1u << (bit & 31u);
  if (atomicOr(&s.claim[bit >> 5], m) & m) return 0u;
  atomicSub(&s.infl[h], 1u);
  return 1u;
}
// on the dialler's shard: the listener staged connection h's SYN-ACK at trep
__device__ __forceinline__ void synack_staged(StormDev& s, size_t h, int64_t trep) {
  if (h >= s.n_conn) return;
  s.t_rep[h] = trep;
  s.flags[h] |= 2u | 8u;
}

__device__ __forceinline__ uint32_t dialler_shard(const StormDev& s, size_t h) {
  return s.S == 1 ? 0u : shard_of((uint32_t)(h / s.O), s.N, s.S);
}

__global__ __launch_bounds__(kBlock) void k_storm_pre(const uint8_t* __restrict__ status,
                                                      const uint32_t* __restrict__ m_src,
                                                      const uint32_t* __restrict__ m_dst,
                                                      const uint32_t* __restrict__ m_seq, uint32_t n_host,
                                                      const uint32_t* n_dev, const uint32_t* __restrict__ o_src,
                                                      const uint32_t* __restrict__ o_dst,
                                                      const uint32_t* __restrict__ o_seq,
                                                      const int64_t* __restrict__ o_t, DevScalars* sc, StormDev s,
                                                      uint32_t nb, uint32_t set_base, uint32_t base_host) {
  __shared__ unsigned long long red[kBlock / 64];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    s.sc->min_dl = kNone;
    s.sc->next_start = kNone;
    s.sc->active = 0;
    s.sc->waiting = 0;
    s.sc->done = 0;
    if (set_base) sc->n_msgs_dev = base_host;  // nothing in this launch reads it
  }
  const uint32_t O = s.O;
  unsigned long long cnt = 0;
  if (blockIdx.x < nb) {  // the window's packets
    const uint32_t n = n_dev ? *n_dev : n_host;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += nb * kBlock) {
      const uint32_t sq = m_seq[i], tag = sq >> 30;
      if (tag == 1u) {  // a SYN: refused by the dialler's route
        if (!refused_code(status[i])) continue;
        const uint32_t k = sq & kTagMask;
        const size_t h = (size_t)m_src[i] * O + k;
        if (k < O && h < s.n_conn && s.state[h] == kWait && s.dst[h] == m_dst[i]) s.flags[h] |= 1u;
      } else if (tag == 2u) {  // a chunk that no copy of entered the egress queue
        if (!failed_code(status[i])) continue;
        const size_t h = chunk_conn(s, m_src[i], m_dst[i], sq & kTagMask);
        if (h == kNoConn) continue;
        atomicSub(&s.infl[h], 1u);
        s.failed[m_src[i] - s.lo] = 1;
        ++cnt;
      }
    }
    block_add(&s.sc->failed, cnt, red);
  } else {  // the window's deliveries (local receivers)
    const uint32_t n = sc->n_out;
    for (uint32_t i0 = (blockIdx.x - nb) * kBlock; i0 < n; i0 += nb * kBlock) {  // wave-uniform trip count
      const uint32_t i = i0 + threadIdx.x;
      uint32_t peer = kNoPeer, nh = 0, nj = 0;
      bool listed = false;
      if (i < n) {
        const uint32_t sq = o_seq[i], tag = sq >> 30;
        if (tag == 1u) {  // a SYN at its listener: the connection's first arrival is answered
          const uint32_t k = sq & kTagMask;
          const size_t h = (size_t)o_src[i] * O + k;
          if (k < O && h < s.n_conn && s.dst[h] == o_dst[i] && s.ans[h] != 1u) {
            atomicMin(reinterpret_cast<long long*>(&s.t_synarr[h]), (long long)o_t[i]);
            if (atomicCAS(&s.ans[h], 0u, 2u) == 0u) { listed = true; nh = (uint32_t)h; }
          }
        } else if (tag == 3u) {  // a SYN-ACK at its dialler
          const size_t h = sq & kTagMask;
          if (h < s.n_conn && h / O == o_dst[i] && s.dst[h] == o_src[i] && s.state[h] == kWait)
            atomicMin(reinterpret_cast<long long*>(&s.t_ackarr[h]), (long long)o_t[i]);
        } else if (tag == 2u && s.nchunks) {  // a chunk at its listener: to its dialler
          const uint32_t c = sq & kTagMask, k = c / s.nchunks;
          const size_t h = (size_t)o_src[i] * O + k;
          if (k < O && h < s.n_conn && s.dst[h] == o_dst[i]) {
            const uint32_t p = dialler_shard(s, h);
            if (p == s.shard) cnt += chunk_arrived(s, h, c - k * s.nchunks);
            else { peer = p; nh = (uint32_t)h; nj = c - k * s.nchunks; }
          }
        }
      }
      const uint64_t lm = __ballot(listed);  // the SYNs to answer: one reservation per wave
      if (lm) {
        const int leader = __ffsll((unsigned long long)lm) - 1;
        uint32_t base = 0;
        if ((int)lane_id() == leader) base = atomicAdd(&s.sc->n_ans, (uint32_t)__popcll(lm));
        base = __shfl(base, leader);
        if (listed) s.alist[base + mask_rank(lm)] = nh;
      }
      if (s.S > 1) notice_push(s.xq, s.xsend, s.xcap, sc, peer, nh, 0u, kNoticeChunk, nj);
    }
    block_add(&s.sc->delivered, cnt, red);
  }
}

// The listeners answer the connections listed by k_storm_pre: the SYN-ACK at max(first arrival,
// horizon), staged behind the device-side count (one reservation per block), and its notice to the
// dialler (applied here on one shard)
__global__ __launch_bounds__(kBlock) void k_storm_answer(DevScalars* sc, StormDev s, uint32_t cap,
                                                         uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                         uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                         int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sbase;
  const uint32_t n = s.sc->n_ans;
  const int64_t H = sc->T;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < n; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t i = b0 + threadIdx.x;
    uint32_t h = 0, peer = kNoPeer;
    int64_t trep = 0;
    if (i < n) {
      h = s.alist[i];
      const int64_t sa = s.t_synarr[h];
      trep = sa > H ? sa : H;
      s.ans[h] = 1u;
      const uint32_t p = dialler_shard(s, h);
      if (p == s.shard) synack_staged(s, h, trep);
      else peer = p;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan(i < n ? 1u : 0u, red, tot);
    if (threadIdx.x == 0) sbase = tot ? reserve_staged(&sc->n_msgs_dev, tot, cap) : 0u;
    __syncthreads();
    if (i < n) {
      const uint32_t w = sbase + ex;
      if (w < cap) {  // from the listener, on the dialler's connection id
        m_src[w] = s.dst[h]; m_dst[w] = h / s.O; m_seq[w] = TGSIM_STORM_SYNACK | h; m_size[w] = s.syn; m_t[w] = trep;
      } else {
        atomicOr(&sc->err, ERR_CAP_M);
      }
    }
    if (s.S > 1) notice_push(s.xq, s.xsend, s.xcap, sc, peer, h, 0u, kNoticeSynAck, trep);
    __syncthreads();  // sbase is rewritten by the next round
  }
}

// Sharded: the headers of the notice blocks (counts from the cursors), as k_xheaders does for a window
__global__ void k_storm_xheaders(StormDev s) {
  const uint32_t p = threadIdx.x;
  if (p >= s.S) return;
  const uint32_t n = min(s.xq[p << 5], s.xcap - 1);
  tgsim_record h;
  h.t = (int64_t)n; h.src = h.dst = h.seq = h.size = h.meta = h.corrupt_off = 0;
  s.xsend[(size_t)p * s.xcap] = h;
}

// Sharded: the notices the other shards sent this shard's diallers
__global__ __launch_bounds__(kBlock) void k_storm_notices(DevScalars* sc, StormDev s) {
  __shared__ unsigned long long red[kBlock / 64];
  unsigned long long cnt = 0;
  const uint64_t total = (uint64_t)s.S * s.xcap;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j += (uint64_t)gridDim.x * kBlock) {
    const uint32_t p = (uint32_t)(j / s.xcap), i = (uint32_t)(j % s.xcap);
    if (p == s.shard || i == 0) continue;
    const int64_t n = s.xrecv[(size_t)p * s.xcap].t;
    if (n < 0 || n >= (int64_t)s.xcap) {
      if (i == 1) atomicOr(&sc->err, ERR_EXCH_HDR);
      continue;
    }
    if ((int64_t)i > n) continue;
    const tgsim_record r = s.xrecv[j];
    if (r.seq == kNoticeSynAck) synack_staged(s, r.src, r.t);
    else if (r.seq == kNoticeChunk) cnt += chunk_arrived(s, r.src, (uint32_t)r.t);
  }
  block_add(&s.sc->delivered, cnt, red);
}

// per block: the minimum deadline / start time of its instances and the active count
__device__ __forceinline__ void block_reduce(StormDev& s, int64_t dl, int64_t ns, uint32_t act, uint32_t waiting) {
  __shared__ int64_t s_dl[kBlock / 64], s_ns[kBlock / 64];
  __shared__ uint32_t s_n[kBlock / 64], s_w[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_xor(dl, o), z = __shfl_xor(ns, o);
    dl = y < dl ? y : dl;
    ns = z < ns ? z : ns;
    act += (uint32_t)__shfl_xor(act, o);
    waiting += (uint32_t)__shfl_xor(waiting, o);
  }
  if (lane_id() == 0) {
    s_dl[threadIdx.x >> 6] = dl; s_ns[threadIdx.x >> 6] = ns; s_n[threadIdx.x >> 6] = act; s_w[threadIdx.x >> 6] = waiting;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t m = s_dl[0], q = s_ns[0];
    uint32_t n = s_n[0], wt = s_w[0];
    for (int w = 1; w < kBlock / 64; ++w) {
      m = s_dl[w] < m ? s_dl[w] : m;
      q = s_ns[w] < q ? s_ns[w] : q;
      n += s_n[w];
      wt += s_w[w];
    }
    if (wt) atomicAdd(&s.sc->waiting, wt);
    if (m != kNone) atomicMin(reinterpret_cast<long long*>(&s.sc->min_dl), (long long)m);
    if (q != kNone) atomicMin(reinterpret_cast<long long*>(&s.sc->next_start), (long long)q);
    if (n) atomicAdd(&s.sc->active, n);
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t chunk_payload(const StormDev& s, uint32_t j) {
  return j + 1 < s.nchunks ? s.chunk : (uint32_t)(s.data - (uint64_t)j * s.chunk);
}

// TCP mode: the ids reserved at setup for connection h's SYN write and chunk c's
// write, and the link of a write's segments onto the connection's send queue (what tgsim_tcp_write
// and k_tcp_link do for a host write; one instance's thread owns its connections' queues)
__device__ __forceinline__ uint32_t tcp_wid(const StormDev& s, size_t h, uint32_t j) {  // j = 0: the SYN
  return s.W0 + (uint32_t)h * (s.nchunks + 1) + j;
}
__device__ __forceinline__ uint32_t tcp_syn_seg(const StormDev& s, size_t h) { return s.S0 + (uint32_t)h * s.spcon; }
__device__ __forceinline__ uint32_t tcp_chunk_seg(const StormDev& s, size_t h, uint32_t c) {
  return tcp_syn_seg(s, h) + 1 + c * s.spc;
}
__device__ __forceinline__ uint32_t tcp_nseg(const StormDev& s, uint32_t c) {
  return (chunk_payload(s, c) + s.mss - 1) / s.mss;
}
// a write's outcome as tgsim_tcp_writes decodes it: delivered once its arrival time is set, else
// failed (the earliest failure's kind in w_fail) once its state left PENDING
__device__ __forceinline__ uint32_t tcp_write_state(const TcpDev& t, uint32_t w) {
  if (t.w_tarr[w] != INT64_MIN) return TGSIM_TCP_DELIVERED;
  if (t.w_state[w] == TGSIM_TCP_PENDING) return TGSIM_TCP_PENDING;
  return (t.w_fail[w] & 1) ? TGSIM_TCP_TIMEOUT : TGSIM_TCP_REFUSED;
}
__device__ __forceinline__ void tcp_link(TcpDev& t, size_t h, uint32_t prev, uint32_t first, uint32_t n, int64_t tw) {
  for (uint32_t x = first; x < first + n; ++x) t.s_tatt[x] = tw;
  if (prev != kTcpNoSeg) t.s_next[prev] = first;
  if (t.c_head[h] == kTcpNoSeg) t.c_head[h] = first;
  if (t.c_una[h] == kTcpNoSeg) t.c_una[h] = first;
  t.c_queued[h] += n;
}

__device__ __forceinline__ void storm_end(StormDev& s, const TcpDev& t, const DevScalars* sc, int64_t t_end);

// Dial phase of instance l: resolve its waiting dials (react), then admit dials. Returns the messages
// to stage (emit[h] bits); dl / ns / act: its reductions.
__device__ __forceinline__ uint32_t dial_step(StormDev& s, TcpDev& t, uint32_t l, uint32_t g, bool resolve,
                                              int64_t H, int64_t t_end, int64_t& dl_min, int64_t& ns_min,
                                              uint32_t& act, uint32_t& waiting) {
  const uint32_t O = s.O, C = s.C;
  const size_t base = (size_t)g * O;
  uint32_t cnt = 0;
  for (uint32_t k = 0; k < O; ++k) {
    const size_t h = base + k;
    s.emit[h] = 0;
    if (!resolve || s.state[h] != kWait) continue;
    if (s.tcp) {  // the SYN write: ACKed (connect() returned, seen at the window's end) or failed
      uint8_t out = TGSIM_PROBE_NONE;
      int64_t te = t_end;
      if (t.c_acked[h] >= 1) {
        out = TGSIM_PROBE_OK;
      } else {
        const uint32_t w = tcp_wid(s, h, 0);
        const uint32_t ws = tcp_write_state(t, w);
        out = ws == TGSIM_TCP_TIMEOUT ? TGSIM_PROBE_TIMEOUT : ws == TGSIM_TCP_REFUSED ? TGSIM_PROBE_REFUSED : out;
        const int64_t dl = s.t_start[h] + s.timeout;
        if (out == TGSIM_PROBE_NONE && dl < t_end) {  // net.DialTimeout (storm.go:144): the SYN write fails
          out = TGSIM_PROBE_TIMEOUT;                  // at the deadline, its slot frees then
          te = dl;
          // a SYN that arrived (its ACK did not) is a delivered write: only a pending one fails
          if (ws == TGSIM_TCP_PENDING) {
            atomicMin(reinterpret_cast<long long*>(&t.w_fail[w]), (long long)(dl * 2 + 1));
            if (atomicCAS(&t.w_state[w], (uint32_t)TGSIM_TCP_PENDING, (uint32_t)TGSIM_TCP_TIMEOUT) == TGSIM_TCP_PENDING) {
              atomicAdd(&t.sc->done, 1u);
              atomicAdd(&t.sc->failed, 1ull);
            }
          }
        }
      }
      if (out != TGSIM_PROBE_NONE) {
        s.state[h] = kDone;
        s.res[h] = out;
        s.t_done[h] = te;
        s.slot_t[(size_t)l * C + s.slot[h]] = te;
      } else {
        ++act;
        ++waiting;
      }
      continue;
    }
    const int64_t dl = s.t_start[h] + s.timeout;
    // the listener answered the SYN's first arrival in this reaction (its notice): the SYN-ACK may
    // still beat the deadline, so a timeout waits one more window
    const uint8_t fl = s.flags[h];
    const bool reply_pending = (fl & 8u) && s.t_rep[h] < dl;
    s.flags[h] = (uint8_t)(fl & ~8u);
    const int64_t aa = s.t_ackarr[h];
    uint8_t out = TGSIM_PROBE_NONE;
    int64_t te = 0;
    if (s.flags[h] & 1u) { out = TGSIM_PROBE_REFUSED; te = s.t_start[h]; }
    else if (aa != kNone && aa < dl) { out = TGSIM_PROBE_OK; te = aa; }
    else if (dl < t_end && !reply_pending) { out = TGSIM_PROBE_TIMEOUT; te = dl; }
    if (out != TGSIM_PROBE_NONE) {
      s.state[h] = kDone;
      s.res[h] = out;
      s.t_done[h] = te;
      s.slot_t[(size_t)l * C + s.slot[h]] = te;  // `<-sem`: the slot is free from the dial's end
    } else {
      ++act;
      ++waiting;
      dl_min = dl < dl_min ? dl : dl_min;
    }
  }
  // the semaphore admits dials in FIFO order while a slot is free: dial at max(t_ready, slot free, H)
  // (TCP: the window's end, when the reaction saw the previous dial's end)
  if (s.tcp) H = t_end > H ? t_end : H;
  uint32_t q = s.dq[l];
  while (q < O) {
    uint32_t best = C;
    int64_t bt = kBusy;
    for (uint32_t c = 0; c < C; ++c) {
      const int64_t t = s.slot_t[(size_t)l * C + c];
      if (t < bt) { bt = t; best = c; }
    }
    if (best == C) break;  // every slot held by a waiting dial
    const uint32_t k = s.order[base + q];
    const size_t h = base + k;
    int64_t t0 = s.t_ready[h];
    t0 = bt > t0 ? bt : t0;
    t0 = H > t0 ? H : t0;
    if (t0 >= t_end + s.window) {  // still asleep (or queued) past the next window
      ns_min = t0 < ns_min ? t0 : ns_min;
      break;
    }
    s.slot_t[(size_t)l * C + best] = kBusy;
    s.slot[h] = best;
    s.state[h] = kWait;
    s.t_start[h] = t0;
    ++act;
    ++waiting;
    ++q;
    if (s.tcp) {  // the SYN: a bare segment written on the connection (the first on its queue)
      tcp_link(t, h, kTcpNoSeg, tcp_syn_seg(s, h), 1, t0);
      s.wsegs[h] = 1;
      continue;
    }
    s.flags[h] = 0;
    s.t_ackarr[h] = kNone;
    s.emit[h] |= kEmitSyn;
    ++cnt;
    const int64_t dl = t0 + s.timeout;
    dl_min = dl < dl_min ? dl : dl_min;
  }
  s.dq[l] = q;
  act += O - q;  // asleep, not yet admitted
  return cnt;
}

// Write phase of instance l at time t: one writesem round (storm.go:158-183). Goroutines take the
// semaphore in FIFO order; a conn.Write whose chunk fits the buffer returns and its goroutine queues
// again for the next chunk, one that does not fit blocks holding its slot (the holders retry first,
// in order). Returns the chunks written (emit[h] per connection).
//   message mode: a connection's buffer holds `win` chunks that have neither arrived nor failed;
//   TCP mode: conn.Write returns once the chunk's segments fit the socket buffer, 2 x cwnd segments
//   (Linux autotunes sk_sndbuf to about twice the window [EXT]) minus those written and not yet
//   ACKed - at most one chunk per connection per reaction, as the ACKs drain it window by window.
// TCP mode also settles the connection's written chunks in order (delivered / failed, from the write
// states) and links each new chunk's segments onto its send queue.
__device__ __forceinline__ uint32_t write_step(StormDev& s, TcpDev& t, uint32_t l, uint32_t g, int64_t t_end,
                                               uint32_t& act, unsigned long long& bytes, unsigned long long& dcnt,
                                               unsigned long long& fcnt) {
  const uint32_t O = s.O, C = s.C, win = s.win;
  const size_t base = (size_t)g * O;
  uint32_t* ring = s.ring + base;
  uint32_t* hold = s.hold + (size_t)l * s.Hc;
  uint32_t qh = s.qh[l], ql = s.ql[l], nh = s.nh[l];
  for (uint32_t k = 0; k < O; ++k) {
    const size_t h = base + k;
    s.emit[h] = 0;
    if (!s.tcp) continue;
    const uint32_t written = s.nchunks - s.rem[h];
    uint32_t st = s.settled[h];
    while (st < written) {
      const uint32_t ws = tcp_write_state(t, tcp_wid(s, h, 1 + st));
      if (ws == TGSIM_TCP_PENDING) break;
      if (ws == TGSIM_TCP_DELIVERED) {
        ++dcnt;
      } else {
        ++fcnt;
        s.failed[l] = 1;
      }
      ++st;
    }
    s.settled[h] = st;
  }
  auto room = [&](size_t h) -> bool {
    if (!s.tcp) return s.infl[h] + s.emit[h] < win;
    if (s.emit[h]) return false;
    const int64_t buffered = (int64_t)s.wsegs[h] - (int64_t)t.c_acked[h];
    return 2 * (int64_t)t.c_cwnd[h] - buffered >= (int64_t)tcp_nseg(s, s.nchunks - s.rem[h]);
  };
  uint32_t cnt = 0;
  bool progress = true;
  while (progress) {
    progress = false;
    uint32_t keep = 0;
    for (uint32_t i = 0; i < nh; ++i) {  // blocked writers whose buffer drained
      const uint32_t k = hold[i];
      const size_t h = base + k;
      if (room(h)) {
        s.emit[h] += 1;
        const uint32_t r = --s.rem[h];
        ++cnt;
        progress = true;
        if (r) { ring[(qh + ql) % O] = k; ++ql; }
      } else {
        hold[keep++] = k;
      }
    }
    nh = keep;
    while (nh < C && ql > 0) {  // free slots go to the queue's head
      const uint32_t k = ring[qh];
      qh = (qh + 1) % O;
      --ql;
      const size_t h = base + k;
      if (room(h)) {
        s.emit[h] += 1;
        const uint32_t r = --s.rem[h];
        ++cnt;
        progress = true;
        if (r) { ring[(qh + ql) % O] = k; ++ql; }
      } else {
        hold[nh++] = k;
      }
    }
  }
  s.qh[l] = qh;
  s.ql[l] = ql;
  s.nh[l] = nh;
  for (uint32_t k = 0; k < O; ++k) {
    const size_t h = base + k;
    const uint32_t e = s.emit[h];
    const uint32_t j0 = s.nchunks - s.rem[h] - e;
    for (uint32_t j = j0; j < j0 + e; ++j) bytes += chunk_payload(s, j);
    if (s.tcp) {
      if (e) {  // chunk j0 (one per reaction): its segments after the previous write's last one
        const uint32_t first = tcp_chunk_seg(s, h, j0), n = tcp_nseg(s, j0);
        tcp_link(t, h, j0 ? first - 1 : tcp_syn_seg(s, h), first, n, t_end);
        s.wsegs[h] += n;
      }
      act += (s.rem[h] || s.settled[h] < s.nchunks - s.rem[h]) ? 1u : 0u;
    } else {
      const uint32_t f = s.infl[h] + e;
      s.infl[h] = f;
      act += (s.rem[h] || f) ? 1u : 0u;
    }
  }
  return cnt;
}

__global__ __launch_bounds__(kBlock) void k_storm_step(StormDev s, TcpDev t, DevScalars* sc, uint32_t lo, uint32_t nloc,
                                                       uint32_t mode, int64_t H_host, int64_t tend_host, uint32_t cap,
                                                       uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                       uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                       int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ unsigned long long red64[kBlock / 64];
  __shared__ uint32_t sbase;
  const bool react = mode == kModeReact;
  const int64_t H = react ? sc->T : H_host, t_end = react ? sc->t_end : tend_host;
  const bool writes = s.phase == 1;
  const uint32_t O = s.O;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < nloc; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t l = b0 + threadIdx.x;
    int64_t dl = kNone, ns = kNone;
    uint32_t act = 0, waiting = 0, wrote = 0, cnt = 0;
    unsigned long long bytes = 0, dcnt = 0, fcnt = 0;
    const uint32_t g = lo + l;
    if (l < nloc) {
      if (writes) wrote = write_step(s, t, l, g, t_end, act, bytes, dcnt, fcnt);
      else cnt = dial_step(s, t, l, g, react, H, t_end, dl, ns, act, waiting);
    }
    if (wrote) s.t_last[l] = t_end;
    if (!s.tcp) cnt += wrote;  // TCP: the connections' queues send them (k_tcp_conn_release)
    uint32_t tot;
    const uint32_t ex = block_excl_scan(cnt, red, tot);
    if (threadIdx.x == 0) sbase = tot ? reserve_staged(&sc->n_msgs_dev, tot, cap) : 0u;
    __syncthreads();
    if (cnt) {
      uint32_t w = sbase + ex;
      const size_t base = (size_t)g * O;
      for (uint32_t k = 0; k < O; ++k) {
        const size_t h = base + k;
        const uint32_t e = s.emit[h];
        if (!e) continue;
        if (writes) {  // chunks j0 .. j0 + e - 1 at t_end
          const uint32_t j0 = s.nchunks - s.rem[h] - e;
          for (uint32_t j = j0; j < j0 + e; ++j, ++w) {
            const uint32_t pay = chunk_payload(s, j);
            if (w < cap) {
              m_src[w] = g; m_dst[w] = s.dst[h]; m_seq[w] = TGSIM_STORM_DATA | (k * s.nchunks + j);
              m_size[w] = pay + s.hdr; m_t[w] = t_end;
            } else {
              atomicOr(&sc->err, ERR_CAP_M);
            }
          }
        } else {
          if (e & kEmitSyn) {
            if (w < cap) {
              m_src[w] = g; m_dst[w] = s.dst[h]; m_seq[w] = TGSIM_STORM_SYN | k; m_size[w] = s.syn;
              m_t[w] = s.t_start[h];
            } else {
              atomicOr(&sc->err, ERR_CAP_M);
            }
            ++w;
          }
        }
      }
    }
    __syncthreads();  // sbase is rewritten by the next round
    if (writes) {
      block_add(&s.sc->written, wrote, red64);
      block_add(&s.sc->bytes, bytes, red64);
      if (s.tcp) {
        block_add(&s.sc->delivered, dcnt, red64);
        block_add(&s.sc->failed, fcnt, red64);
      }
    }
    block_reduce(s, dl, ns, act, waiting);
  }
  // the last workgroup to finish proposes the next window's end
  __shared__ uint32_t s_last;
  if (block_release_for_count()) s_last = atomicAdd(&s.sc->done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(s_last) && threadIdx.x == 0) {
    fence_acquire_agent();
    storm_end(s, t, sc, t_end);
  }
}

// every k_storm_step workgroup's reductions and reservations are done: read with device-scope atomic
// loads (another XCD's L2 may hold the lines)
__device__ __forceinline__ void storm_end(StormDev& s, const TcpDev& t, const DevScalars* sc, int64_t t_end) {
  int64_t ne = t_end + s.window;
  const uint32_t act = __hip_atomic_load(&s.sc->active, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  // TCP: no jump while a dial waits for its ACK (its SYN may be waiting out a retransmission timer;
  // with no dial waiting no timer is armed in the dial phase, and the write phase never jumps: it has
  // no deadlines or starts)
  const bool tcp_idle = !s.tcp || __hip_atomic_load(&s.sc->waiting, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0;
  const int64_t m = __hip_atomic_load(&s.sc->min_dl, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t q = __hip_atomic_load(&s.sc->next_start, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t staged = __hip_atomic_load(const_cast<uint32_t*>(&sc->n_msgs_dev), __ATOMIC_ACQUIRE,
                                            __HIP_MEMORY_SCOPE_AGENT);
  int64_t cand = m != kNone ? m + 1 : kNone;
  cand = q < cand ? q : cand;
  const bool busy = staged != 0 || sc->arena_used != 0 || !tcp_idle;
  if (!busy && act && cand != kNone && cand > ne) ne = cand;  // idle: jump to the next deadline or dial
  s.sc->next_end = ne;
  s.sc->n_active = act;
  s.sc->prop[0] = busy ? 1 : 0;  // sharded: the same rule over every shard's inputs (k_storm_prop)
  s.sc->prop[1] = act;
  s.sc->prop[2] = cand;
}

// Sharded: the proposal from every shard's (busy, active, earliest deadline + 1 / dial start), all-
// gathered into prop_all - the one-shard rule over the whole run
__global__ void k_storm_prop(StormDev s, const DevScalars* sc) {
  if (threadIdx.x != 0) return;
  int64_t busy = 0, act = 0, cand = kNone;
  for (uint32_t k = 0; k < s.S; ++k) {
    busy |= s.prop_all[3 * k];
    act += s.prop_all[3 * k + 1];
    cand = s.prop_all[3 * k + 2] < cand ? s.prop_all[3 * k + 2] : cand;
  }
  int64_t ne = sc->t_end + s.window;
  if (!busy && act && cand != kNone && cand > ne) ne = cand;
  s.sc->next_end = ne;
  s.sc->n_active = (uint32_t)act;
}

__global__ void k_storm_reset(StormDev s, DevScalars* sc, uint32_t set_base, uint32_t base_host) {
  if (threadIdx.x == 0) {
    s.sc->min_dl = kNone;
    s.sc->next_start = kNone;
    s.sc->active = 0;
    s.sc->waiting = 0;
    s.sc->done = 0;
    if (set_base) sc->n_msgs_dev = base_host;
  }
}

// the write phase's start: every connection's goroutine queued on writesem in connection order
__global__ __launch_bounds__(kBlock) void k_storm_write_init(StormDev s, uint32_t lo, uint32_t nloc) {
  for (uint32_t l = blockIdx.x * kBlock + threadIdx.x; l < nloc; l += gridDim.x * kBlock) {
    const size_t base = (size_t)(lo + l) * s.O;
    uint32_t n = 0;
    for (uint32_t k = 0; k < s.O; ++k) {
      s.rem[base + k] = s.nchunks;
      s.infl[base + k] = 0;
      if (s.tcp) s.settled[base + k] = 0;
      if (s.nchunks) s.ring[base + n++] = k;
    }
    s.qh[l] = 0;
    s.ql[l] = n;
    s.nh[l] = 0;
  }
}

// TCP mode: the reserved writes (the SYN, then every chunk) and their segments, as tgsim_tcp_write
// would build them; their times and links are set when they are written
__global__ __launch_bounds__(kBlock) void k_storm_tcp_init(StormDev s, TcpDev t) {
  for (uint32_t h = blockIdx.x * kBlock + threadIdx.x; h < s.n_conn; h += gridDim.x * kBlock) {
    const uint32_t g = h / s.O, d = s.dst[h];
    for (uint32_t j = 0; j <= s.nchunks; ++j) {
      const uint32_t w = tcp_wid(s, h, j);
      const uint32_t pay = j ? chunk_payload(s, j - 1) : 0u, n = j ? tcp_nseg(s, j - 1) : 1u;
      const uint32_t first = j ? tcp_chunk_seg(s, h, j - 1) : tcp_syn_seg(s, h);
      t.w_src[w] = g; t.w_dst[w] = d; t.w_rem[w] = n; t.w_conn[w] = h;
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t x = first + i;
        t.s_w[x] = w | (n == 1 ? kTcpSoleSeg : 0u);
        t.s_wire[x] = (i + 1 < n ? s.mss : pay - i * s.mss) + t.hdr;
        t.s_next[x] = i + 1 < n ? x + 1 : kTcpNoSeg;
      }
    }
  }
}

unsigned grid_for(uint32_t n) {
  return std::max(1u, std::min<unsigned>((n + kBlock - 1) / kBlock, (unsigned)kStreamBlocks));
}

}  // namespace

hipError_t launch_storm_start(Dev& d, const TcpDev& td, bool base_dev, uint32_t base_host, int64_t t_now) {
  hipLaunchKernelGGL(k_storm_reset, dim3(1), dim3(64), 0, d.stream, d.sm, d.sc, base_dev ? 0u : 1u, base_host);
  hipLaunchKernelGGL(k_storm_step, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, d.sm, td, d.sc, d.lo,
                     d.nloc, (uint32_t)kModeStart, t_now, t_now, d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_storm_write_start(Dev& d, const TcpDev& td, bool base_dev, uint32_t base_host, int64_t t0) {
  hipLaunchKernelGGL(k_storm_write_init, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, d.sm, d.lo, d.nloc);
  hipLaunchKernelGGL(k_storm_reset, dim3(1), dim3(64), 0, d.stream, d.sm, d.sc, base_dev ? 0u : 1u, base_host);
  hipLaunchKernelGGL(k_storm_step, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, d.sm, td, d.sc, d.lo,
                     d.nloc, (uint32_t)kModeWrites, t0, t0, d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_storm_react_pre(Dev& d, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                                  const uint32_t* n_status_dev) {
  ProfScope ps_(d, KID_STORM);
  constexpr uint32_t nb = kStreamBlocks / 2;
  StormDev& s = d.sm;
  if (hipMemsetAsync(&s.sc->n_ans, 0, sizeof(uint32_t), d.stream) != hipSuccess) return hipGetLastError();
  if (s.S > 1 && hipMemsetAsync(s.xq, 0, (size_t)s.S * 128, d.stream) != hipSuccess) return hipGetLastError();
  hipLaunchKernelGGL(k_storm_pre, dim3(2 * nb), dim3(kBlock), 0, d.stream, d.status, d.m_src, d.m_dst, d.m_seq,
                     n_status_host, n_status_dev, d.o_src, d.o_dst, d.o_seq, d.o_t, d.sc, s, nb,
                     base_dev ? 0u : 1u, base_host);
  hipLaunchKernelGGL(k_storm_answer, dim3(grid_for(std::max<uint32_t>(s.n_conn, 1u))), dim3(kBlock), 0, d.stream,
                     d.sc, s, d.cap_msgs, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  if (s.S > 1) hipLaunchKernelGGL(k_storm_xheaders, dim3(1), dim3(kMaxShards), 0, d.stream, s);
  return hipGetLastError();
}

hipError_t launch_storm_react_post(Dev& d, const TcpDev& td) {
  ProfScope ps_(d, KID_STORM);
  const StormDev& s = d.sm;
  if (s.S > 1) {
    const uint64_t total = (uint64_t)s.S * s.xcap;
    hipLaunchKernelGGL(k_storm_notices, dim3(grid_for((uint32_t)std::min<uint64_t>(total, 0xFFFFFFFFu))), dim3(kBlock),
                       0, d.stream, d.sc, s);
  }
  hipLaunchKernelGGL(k_storm_step, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, d.sm, td, d.sc, d.lo,
                     d.nloc, (uint32_t)kModeReact, (int64_t)0, (int64_t)0, d.cap_msgs, d.m_src, d.m_dst, d.m_seq,
                     d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_storm_prop(Dev& d) {
  hipLaunchKernelGGL(k_storm_prop, dim3(1), dim3(64), 0, d.stream, d.sm, d.sc);
  return hipGetLastError();
}

// TCP mode (one shard): the TCP reaction has settled the window's packets and deliveries
hipError_t launch_storm_react(Dev& d, const TcpDev& td, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                              const uint32_t* n_status_dev) {
  ProfScope ps_(d, KID_STORM);
  (void)n_status_host;
  (void)n_status_dev;
  hipLaunchKernelGGL(k_storm_reset, dim3(1), dim3(64), 0, d.stream, d.sm, d.sc, base_dev ? 0u : 1u, base_host);
  hipLaunchKernelGGL(k_storm_step, dim3(grid_for(d.nloc)), dim3(kBlock), 0, d.stream, d.sm, td, d.sc, d.lo,
                     d.nloc, (uint32_t)kModeReact, (int64_t)0, (int64_t)0, d.cap_msgs, d.m_src, d.m_dst, d.m_seq,
                     d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_storm_tcp_init(Dev& d, const TcpDev& td) {
  hipLaunchKernelGGL(k_storm_tcp_init, dim3(grid_for(d.sm.n_conn)), dim3(kBlock), 0, d.stream, d.sm, td);
  return hipGetLastError();
}

}  // namespace tgsim
