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
constexpr uint32_t kSoleSeg = kTcpSoleSeg;  // s_w: the segment is its write's only one
constexpr uint32_t kWMask = kTcpWMask;      // s_w: the write
constexpr uint32_t kQShift = 28;            // s_w: copies of the current attempt (2 bits)
constexpr uint32_t kRetxBit = 0x40000000u;  // s_w, acks mode: the segment was retransmitted (s_att > 0)
constexpr uint32_t kPlanLds = 1024;         // k_tcp_fire: timer plans up to this many batches are searched in LDS
constexpr uint32_t kFireRounds = 8;         // k_tcp_fire: rounds of entries per block reservation (mask bits)
constexpr uint32_t kFireUnroll = 4;         // k_tcp_fire: entries whose loads are in flight together
constexpr uint32_t kNoSeg = kTcpNoSeg;      // connections: end of a segment chain / no connection
constexpr uint32_t kCwndClamp = 65535u;    // Linux snd_cwnd_clamp (Reno window in segments)

__device__ __forceinline__ uint32_t tcp_copies(uint8_t st) {
  const uint32_t code = st & 0x0Fu;
  if (code == TGSIM_ST_LOCAL) return 1u;
  if (code != TGSIM_ST_QUEUED) return 0u;
  uint32_t q = (st & TGSIM_ST_FLAG_OVERLIMIT) ? 0u : 1u;
  if ((st & TGSIM_ST_FLAG_DUP) && !(st & TGSIM_ST_FLAG_CLONE_LOST)) ++q;
  return q;
}

// Sharded TCP: a shard numbers its own segments 0, 1, ... (its state arrays), while a
// packet's seq carries the single run's segment id, so that its netem draws (Philox keyed by (seq,
// src)) do not depend on the shard count. A sharded context carries generated storm rounds of one
// fanout F, n * F one-segment writes per round in (instance, k) order: an affine map per round, the
// identity on one shard (oracle twin: tgsim_oracle.c tcp_wire / tcp_local).
__device__ __forceinline__ uint32_t tcp_local(const TcpDev& t, uint32_t w) {
  if (t.S == 1) return w;
  const uint32_t per = t.N * t.F, r = w / per;
  return r * t.nloc * t.F + (w % per - t.lo * t.F);
}
__device__ __forceinline__ uint32_t tcp_wire(const TcpDev& t, uint32_t sid) {
  if (t.S == 1) return sid;
  const uint32_t per = t.nloc * t.F, r = sid / per;
  return r * t.N * t.F + t.lo * t.F + sid % per;
}
// a data copy whose writer (its src) lives on this shard: settled here
__device__ __forceinline__ bool tcp_mine(const TcpDev& t, uint32_t src) { return t.S == 1 || src - t.lo < t.nloc; }

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
    const uint32_t sq = seq[i];
    bool retx = false;
    if (!(t.acks && (sq & TGSIM_TCP_ACK_BIT))) {  // acks mode: an ACK packet's fate concerns nobody
      const uint32_t sid = tcp_local(t, sq >> 4);
      const uint8_t st = status[i];
      const uint32_t q = tcp_copies(st), code = st & 0x0Fu;
      // a released retransmission leaves its sender's pending count once its packet is accounted
      if (sq & 15u) atomicSub(&t.pend_by[t.w_src[t.s_w[sid] & kWMask]], 1u);
      if (q) {
        t.s_out[sid] = q;
        t.s_w[sid] = (t.s_w[sid] & ~(3u << kQShift)) | (q << kQShift);
      } else if (code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) {
        const uint32_t w = t.s_w[sid] & kWMask;
        tcp_fail(t, w, t.s_tatt[sid], TGSIM_TCP_REFUSED);
        if (t.n_conn && t.w_conn[w] != kNoSeg) t.c_broken[t.w_conn[w]] = 1u;  // the connection is reset
      } else if (!t.acks) {  // acks mode: the attempt's timer decides
        retx = tcp_next(t, sid, t.s_tatt[sid]);
      }
    }
    put_bits(t.bm_s, i, retx);
  }
}

// a segment of write sw (its s_w word) arrived intact at arr: 1 when that delivers the write. A write
// whose every segment arrived cannot fail, so its time alone marks it delivered
__device__ __forceinline__ uint32_t tcp_arrived(TcpDev& t, uint32_t sw, int64_t arr) {
  const uint32_t w = sw & kWMask;
  // acks mode: a write can fail (give up) while its data is still on the way; failed stays failed
  if (t.acks && t.w_state[w] != TGSIM_TCP_PENDING) return 0u;
  if (sw & kSoleSeg) {  // no other segment: nothing else writes the write's entries
    t.w_tarr[w] = arr;
    return 1u;
  }
  // running max, then the count as one acq_rel RMW (the hand-off: it releases this thread's max and,
  // for the last segment, acquires every other segment's; the counts are totally ordered); the last
  // segment reads the max back
  atomicMax(reinterpret_cast<long long*>(&t.w_tmax[w]), (long long)arr);
  if (__hip_atomic_fetch_sub(&t.w_rem[w], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != 1u) return 0u;
  const long long m = atomicMax(reinterpret_cast<long long*>(&t.w_tmax[w]), (long long)arr);
  t.w_tarr[w] = m > (long long)arr ? (int64_t)m : arr;
  return 1u;
}

// Sharded, the inputs are the window's own deliveries [0, n_out) and then the data copies of this
// shard's writers delivered on other shards (k_tcp_rx, [n_out, n_in)): a data copy delivered here for
// another shard's writer is only answered (its ACK leaves from here), a forwarded one only settled.
__global__ __launch_bounds__(kBlock) void k_tcp_arrive(const uint32_t* __restrict__ o_src,
                                                       const uint32_t* __restrict__ o_seq,
                                                       const int64_t* __restrict__ o_t,
                                                       const uint32_t* __restrict__ o_flags, const DevScalars* sc,
                                                       TcpDev t) {
  const uint32_t n = t.sc->n_in, nl = sc->n_out;
  uint32_t ndel = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sq = o_seq[i];
    const int64_t ti = o_t[i];
    const bool corrupt = o_flags[i] & TGSIM_F_CORRUPT;
    const bool here = i < nl, mine = !here || tcp_mine(t, o_src[i]);
    if (t.acks) {  // acks mode: ACKs settle segments, intact data is answered; timers decide the rest
      bool ack = false, dup = false;
      if (sq & TGSIM_TCP_ACK_BIT) {
        const uint32_t sid = tcp_local(t, (sq & ~TGSIM_TCP_ACK_BIT) >> 4);
        // the first intact ACK of a segment that has not given up frees its connection a flight slot;
        // what the window's ACKs release leaves at the latest intact one's arrival (every ACK counts
        // there, so which of a segment's duplicate ACKs claims it does not matter)
        if (!corrupt && t.s_done[sid] != 2) {
          t.s_done[sid] = 1;
          const uint32_t k = t.n_conn ? t.w_conn[t.s_w[sid] & kWMask] : kNoSeg;
          if (k != kNoSeg) {
            atomicMax(reinterpret_cast<long long*>(&t.c_tack[k]), (long long)ti);
            if (atomicExch(&t.s_ack1[sid], 1u) == 0u) {
              atomicAdd(&t.c_acks[k], 1u);
              if (!t.s_lost[sid]) atomicAdd(&t.c_fack[k], 1u);  // a segment marked lost holds no slot
            }
          }
        }
      } else if (!corrupt && !mine) {
        ack = true;  // answered here; the writer's shard settles it from the forwarded copy
      } else if (!corrupt) {
        ack = here;
        const uint32_t sid = tcp_local(t, sq >> 4), sw = t.s_w[sid];
        // the first attempt's only copy is the segment's only delivery (a later attempt - and with
        // it another copy - would have set kRetxBit): this thread settles it
        if (((sw >> kQShift) & 3u) == 1u && !(sw & kRetxBit)) {
          t.s_mark[sid] = kArrived;
          ndel += tcp_arrived(t, sw, ti);
        } else {
          atomicMin(reinterpret_cast<long long*>(&t.s_arr[sid]), (long long)ti);
          dup = true;
        }
      }
      put_bits(t.bm_r, i, false);
      put_bits(t.bm_d, i, dup);
      put_bits(t.bm_a, i, ack);
      continue;
    }
    if (!mine) {  // another shard's writer: forwarded there (k_tcp_fwd)
      put_bits(t.bm_r, i, false);
      put_bits(t.bm_d, i, false);
      continue;
    }
    const uint32_t sid = tcp_local(t, sq >> 4);
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

// duplicated deliveries (bm_d), one thread per delivery (a word's 64 deliveries walked by one thread
// made chains of dependent atomics where retransmitted attempts pile up: acks mode 19 us), the
// segment claimed once per epoch; an arrived segment is never settled again. The delivered count goes
// into the block's k_tcp_arrive partial (same grid), not into one shared line per wave.
__global__ __launch_bounds__(kBlock) void k_tcp_settle(const uint32_t* __restrict__ o_seq, const DevScalars* sc,
                                                       TcpDev t, uint32_t epoch, uint32_t cur) {
  const uint32_t n = t.sc->n_in;
  uint32_t ndel = 0;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    if (!((t.bm_d[i >> 6] >> (i & 63u)) & 1ull)) continue;
    const uint32_t sid = tcp_local(t, o_seq[i] >> 4);
    if (atomicMax(&t.s_mark[sid], epoch) >= epoch) continue;
    const int64_t arr = t.s_arr[sid];
    if (arr != INT64_MAX) {
      t.s_mark[sid] = kArrived;
      ndel += tcp_arrived(t, t.s_w[sid], arr);
    } else if (!t.acks && t.s_out[sid] == 0 && tcp_next(t, sid, t.s_tlast[sid])) {
      t.pend[cur][atomicAdd(&t.sc->pend_n[cur], 1u)] = sid;
      atomicAdd(&t.sc->retx, 1ull);
    }
  }
  __shared__ uint32_t red[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ndel += (uint32_t)__shfl_xor(ndel, o);
  if (lane_id() == 0) red[threadIdx.x >> 6] = ndel;
  __syncthreads();
  if (threadIdx.x == 0) t.part[blockIdx.x] += red[0] + red[1] + red[2] + red[3];  // after k_tcp_arrive's store
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
  const uint32_t ws = ((n_dev ? *n_dev : n_host) + 63u) >> 6, wr = (t.sc->n_in + 63u) >> 6, nw = ws + wr;
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
    for (; m; m &= m - 1) t.pend[cur][p++] = tcp_local(t, seq[i0 + (uint32_t)__builtin_ctzll(m)] >> 4);
    nretx += tot;
    __syncthreads();  // sbase is rewritten by the next round
  }
  if (t.acks) {  // the ACK list (delivery indices), one reservation per block and round
    for (uint32_t b0 = blockIdx.x * kBlock; b0 < wr; b0 += gridDim.x * kBlock) {  // uniform per block
      const uint32_t wi = b0 + threadIdx.x;
      uint64_t m = wi < wr ? t.bm_a[wi] : 0ull;
      uint32_t tot;
      uint32_t p = block_excl_scan((uint32_t)__popcll(m), red, tot);
      if (threadIdx.x == 0 && tot) sbase = atomicAdd(&t.sc->ack_n, tot);
      __syncthreads();
      p += sbase;
      for (; m; m &= m - 1) t.ack_idx[p++] = wi * 64u + (uint32_t)__builtin_ctzll(m);
      __syncthreads();
    }
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

__global__ __launch_bounds__(kBlock) void k_tcp_reset(TcpDev t, uint32_t cur, const DevScalars* sc, uint32_t fill) {
  if (threadIdx.x == 0) {
    t.sc->done = 0;
    t.sc->pend_n[cur ^ 1u] = 0;
    t.sc->ack_n = 0;
    t.sc->n_in = sc->n_out;  // sharded: k_tcp_rx adds the forwarded copies
    if (fill != ~0u) {  // acks mode: the window's new segments sent in [T, t_end): timers in [T, t_end) + rto
      TcpBatch& b = t.tb[fill % kTcpBatches];
      b.t_lo = sc->T + t.rto;
      b.t_hi = sc->t_end + t.rto;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_tcp_base(DevScalars* sc, uint32_t base_host) {
  if (threadIdx.x == 0) sc->n_msgs_dev = base_host;
}

__global__ __launch_bounds__(kBlock) void k_tcp_release(TcpDev t, uint32_t cur, DevScalars* sc, uint32_t cap,
                                                        uint32_t* __restrict__ m_src, uint32_t* __restrict__ m_dst,
                                                        uint32_t* __restrict__ m_seq, uint32_t* __restrict__ m_size,
                                                        int64_t* __restrict__ m_t) {
  // one reservation per block and round for the released packets and one for the kept entries
  // (per-item reservations serialise on the two counters at the memory side)
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sb_r, sb_k;
  const uint32_t n = t.sc->pend_n[cur], nxt = cur ^ 1u;
  const int64_t t_end = sc->t_end;
  uint32_t nrel = 0;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < n; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t i = b0 + threadIdx.x;
    bool rel = false, keep = false;
    uint32_t sid = 0, w = 0;
    int64_t ta = 0;
    if (i < n) {
      sid = t.pend[cur][i];
      w = t.s_w[sid] & kWMask;
      ta = t.s_tatt[sid];
      if (t.w_state[w] != TGSIM_TCP_PENDING) {  // the write has failed: nothing more is sent
        atomicSub(&t.pend_by[t.w_src[w]], 1u);
      } else if (ta >= t_end) {
        keep = true;
      } else {
        rel = true;
      }
    }
    uint32_t totr, totk;
    const uint32_t pr = block_excl_scan(rel ? 1u : 0u, red, totr);
    const uint32_t pk = block_excl_scan(keep ? 1u : 0u, red, totk);
    if (threadIdx.x == 0) {
      sb_r = totr ? reserve_staged(&sc->n_msgs_dev, totr, cap) : 0u;
      sb_k = totk ? atomicAdd(&t.sc->pend_n[nxt], totk) : 0u;
    }
    __syncthreads();
    if (keep) t.pend[nxt][sb_k + pk] = sid;
    if (rel) {
      const uint32_t p = sb_r + pr;
      if (p < cap) {
        m_src[p] = t.w_src[w]; m_dst[p] = t.w_dst[w]; m_seq[p] = (tcp_wire(t, sid) << 4) | t.s_att[sid];
        m_size[p] = t.s_wire[sid];
        m_t[p] = ta;
      } else {
        atomicOr(&sc->err, ERR_CAP_M);
      }
    }
    nrel += totr;
    __syncthreads();  // sb_r / sb_k are rewritten by the next round
  }
  if (threadIdx.x == 0 && nrel) atomicAdd(&t.sc->released, (unsigned long long)nrel);
}

// acks mode, window start (one block): the last reaction's ACKs get their staged slots; the live
// timer batches whose earliest timer falls before the window's end form the plan (per batch its
// first segment and its offset in the plan's item space; a batch whose every timer falls before the
// end is scanned for the last time and retires); the window's new segments register a batch.
__global__ __launch_bounds__(kBlock) void k_tcp_tplan(TcpDev t, DevScalars* sc, uint32_t head, uint32_t reg,
                                                      uint32_t lo, uint32_t hi, uint32_t cap) {
  __shared__ uint32_t red[kBlock / 64];
  const int64_t t_end = sc->t_end;
  const uint32_t tail = t.sc->tb_tail;
  if (threadIdx.x == 0) {
    const uint32_t base = sc->n_msgs_dev, na = t.sc->ack_n;
    t.sc->ack_base = base;
    // ACK slots beyond the capacity are not written (k_tcp_fire) and not counted
    sc->n_msgs_dev = (uint64_t)base + na > cap ? cap : base + na;
    if ((uint64_t)base + na > cap) atomicOr(&sc->err, ERR_CAP_M);
  }
  uint32_t carry = 0;
  for (uint32_t b0 = tail; b0 < head; b0 += kBlock) {  // block-uniform
    const uint32_t k = b0 + threadIdx.x;
    uint32_t len = 0, first = 0;
    if (k < head) {
      TcpBatch& b = t.tb[k % kTcpBatches];
      first = b.lo;
      if (!b.done && b.t_lo < t_end) {
        len = b.hi - b.lo;
        if (b.t_hi <= t_end) b.done = 1u;
      }
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan(len, red, tot);
    if (k < head) {
      t.plan_lo[k - tail] = first;
      t.plan_off[k - tail] = carry + ex;
    }
    carry += tot;
  }
  __syncthreads();  // the done flags above
  if (threadIdx.x == 0) {
    t.plan_off[head - tail] = carry;
    t.sc->plan_n = head - tail;
    t.sc->plan_total = carry;
    uint32_t tl = tail;
    while (tl < head && t.tb[tl % kTcpBatches].done) ++tl;
    t.sc->tb_tail = tl;
    if (reg) {
      if (head + 1u - tl > kTcpBatches) atomicOr(&sc->err, ERR_TCP_TIMERS);
      TcpBatch& b = t.tb[head % kTcpBatches];
      b.lo = lo; b.hi = hi; b.t_lo = INT64_MAX; b.t_hi = INT64_MAX; b.done = 0u; b.pad = 0u;
    }
  }
}

// acks mode, window start: the ACKs staged (at max(arrival, window start)); every planned
// attempt-0 timer and every retransmitted attempt's timer (pend[cur]) checked - settled (ACKed,
// gave up) or of a failed write: dropped; before the window's end: the next attempt at max(timer,
// window start), or the segment gives up; else kept (pend[cur ^ 1]). One reservation per block and
// round for the fired packets and one for the kept timers.
__global__ __launch_bounds__(kBlock) void k_tcp_fire(TcpDev t, DevScalars* sc, uint32_t cur, uint32_t cap,
                                                     const uint32_t* __restrict__ o_src,
                                                     const uint32_t* __restrict__ o_dst,
                                                     const uint32_t* __restrict__ o_seq,
                                                     const int64_t* __restrict__ o_t, uint32_t* __restrict__ m_src,
                                                     uint32_t* __restrict__ m_dst, uint32_t* __restrict__ m_seq,
                                                     uint32_t* __restrict__ m_size, int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sb_f, sb_k;
  const int64_t H = sc->T, t_end = sc->t_end;  // the window [T, t_end)
  const int64_t Hr = sc->H;                     // the reaction horizon: the last window's start
  const uint32_t nxt = cur ^ 1u, stride = gridDim.x * kBlock;
  const uint32_t na = t.sc->ack_n, ab = t.sc->ack_base;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < na; i += stride) {
    const uint32_t d = t.ack_idx[i], p = ab + i;
    if (p < cap) {  // an ACK leaves when its segment arrived (a late send, at or after the horizon)
      m_src[p] = o_dst[d]; m_dst[p] = o_src[d]; m_seq[p] = TGSIM_TCP_ACK_BIT | o_seq[d]; m_size[p] = t.hdr;
      m_t[p] = o_t[d] > Hr ? o_t[d] : Hr;
    }
  }
  const uint32_t np = t.sc->plan_n, nb = t.sc->plan_total, total = nb + t.sc->pend_n[cur];
  // the plan (a few dozen live batches) in LDS: locating an entry costs no global round trip
  __shared__ uint32_t s_off[kPlanLds], s_lo[kPlanLds];
  const bool lds = np <= kPlanLds;
  if (lds) {
    for (uint32_t k = threadIdx.x; k < np; k += kBlock) {
      s_off[k] = t.plan_off[k];
      s_lo[k] = t.plan_lo[k];
    }
    __syncthreads();
  }
  // entry j -> its segment: a batch entry (the last plan entry starting at or before j; empty
  // entries share offsets) or a retransmitted attempt's timer
  auto locate = [&](uint32_t j) -> uint32_t {
    if (j >= nb) return t.pend[cur][j - nb];
    uint32_t l = 0, h = np;
    if (lds) {
      while (h - l > 1) {
        const uint32_t mid = (l + h) >> 1;
        if (s_off[mid] <= j) l = mid; else h = mid;
      }
      return s_lo[l] + (j - s_off[l]);
    }
    while (h - l > 1) {
      const uint32_t mid = (l + h) >> 1;
      if (t.plan_off[mid] <= j) l = mid; else h = mid;
    }
    return t.plan_lo[l] + (j - t.plan_off[l]);
  };
  // A block takes kFireRounds rounds of entries at a time: the decisions (and their effects on the
  // segment) first, recorded as one bit per round in two masks per thread, then one reservation per
  // block for the fired packets and one for the kept timers, then the writes. A reservation per
  // round would put total / 256 updates on each of the two counters, which the memory side
  // serialises.
  const uint32_t span = kBlock * kFireRounds;
  uint32_t nfire = 0;
  for (uint32_t c0 = blockIdx.x * span; c0 < total; c0 += gridDim.x * span) {  // block-uniform
    uint32_t fmask = 0, kmask = 0;
    // kFireUnroll entries at a time, each level of their dependent loads issued together
    for (uint32_t r0 = 0; r0 < kFireRounds; r0 += kFireUnroll) {
      uint32_t sid[kFireUnroll], a[kFireUnroll], sw[kFireUnroll], wst[kFireUnroll];
      uint8_t dn[kFireUnroll];
      int64_t ta[kFireUnroll];
      bool batch[kFireUnroll], live[kFireUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kFireUnroll; ++u) {
        const uint32_t j = c0 + (r0 + u) * kBlock + threadIdx.x;
        live[u] = j < total;
        batch[u] = j < nb;
        sid[u] = live[u] ? locate(j) : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < kFireUnroll; ++u) {
        a[u] = live[u] ? t.s_att[sid[u]] : 0u;
        dn[u] = live[u] ? t.s_done[sid[u]] : (uint8_t)1;
      }
#pragma unroll
      for (uint32_t u = 0; u < kFireUnroll; ++u) {
        // a batch entry whose segment was retransmitted already has its timer on the list
        live[u] = live[u] && !(batch[u] && a[u] != 0) && dn[u] == 0;
        sw[u] = live[u] ? t.s_w[sid[u]] : 0u;
        ta[u] = live[u] ? t.s_tatt[sid[u]] : 0;
      }
#pragma unroll
      for (uint32_t u = 0; u < kFireUnroll; ++u) wst[u] = live[u] ? t.w_state[sw[u] & kWMask] : 0u;
#pragma unroll
      for (uint32_t u = 0; u < kFireUnroll; ++u) {
        if (!live[u]) continue;
        const uint32_t r = r0 + u, w = sw[u] & kWMask;
        const uint32_t k = t.n_conn ? t.w_conn[w] : kNoSeg;
        // a connection segment marked lost has no timer until it is resent (which enters it again)
        if (k != kNoSeg && t.s_lost[sid[u]]) { t.s_tq[sid[u]] = 0; continue; }
        if (wst[u] == TGSIM_TCP_TIMEOUT || wst[u] == TGSIM_TCP_REFUSED) continue;
        const int64_t T = ta[u] + (t.rto << a[u]);
        if (T >= t_end || (!batch[u] && ta[u] >= H)) {  // not due, or sent in this window
          if (!batch[u]) kmask |= 1u << r;
        } else if (a[u] + 1u >= t.max_att) {
          t.s_done[sid[u]] = 2;
          if (k != kNoSeg) atomicSub(&t.c_flight[k], 1u);
          if (t.w_tarr[w] == INT64_MIN) tcp_fail(t, w, T, TGSIM_TCP_TIMEOUT);
        } else if (k != kNoSeg) {
          // a connection's timeout: the loss episode (k_tcp_conn_release, kRelLoss) resends under cwnd
          atomicMin(reinterpret_cast<long long*>(&t.c_tloss[k]), (long long)T);
          t.s_tq[sid[u]] = 0;
        } else {
          t.s_att[sid[u]] = a[u] + 1u;
          t.s_tatt[sid[u]] = T > H ? T : H;
          if (!(sw[u] & kRetxBit)) t.s_w[sid[u]] = sw[u] | kRetxBit;
          fmask |= 1u << r;
          kmask |= 1u << r;
        }
      }
    }
    uint32_t totf, totk;
    const uint32_t pf = block_excl_scan((uint32_t)__popc(fmask), red, totf);
    const uint32_t pk = block_excl_scan((uint32_t)__popc(kmask), red, totk);
    if (threadIdx.x == 0) {
      sb_f = totf ? reserve_staged(&sc->n_msgs_dev, totf, cap) : 0u;
      sb_k = totk ? atomicAdd(&t.sc->pend_n[nxt], totk) : 0u;
    }
    __syncthreads();
    uint32_t qf = sb_f + pf, qk = sb_k + pk;
    for (uint32_t m = kmask; m; m &= m - 1) {  // every fired entry is also kept
      const uint32_t r = (uint32_t)__builtin_ctz(m);
      const uint32_t sid = locate(c0 + r * kBlock + threadIdx.x);
      t.pend[nxt][qk++] = sid;
      if (!((fmask >> r) & 1u)) continue;
      const uint32_t w = t.s_w[sid] & kWMask, src = t.w_src[w];
      const uint32_t p = qf++;
      if (p < cap) {
        m_src[p] = src; m_dst[p] = t.w_dst[w]; m_seq[p] = (tcp_wire(t, sid) << 4) | t.s_att[sid];
        m_size[p] = t.s_wire[sid];
        m_t[p] = t.s_tatt[sid];
      } else {
        atomicOr(&sc->err, ERR_CAP_M);
      }
      atomicAdd(&t.pend_by[src], 1u);  // released into this window until its status is read
    }
    nfire += totf;
    __syncthreads();  // sb_f / sb_k are rewritten by the next round
  }
  if (threadIdx.x == 0 && nfire) {
    atomicAdd(&t.sc->retx, (unsigned long long)nfire);
    atomicAdd(&t.sc->released, (unsigned long long)nfire);
  }
}

// Connections: a batch's new segments join their queues. One quad per touched connection (conn,
// its tail before the batch, the batch's first segment on it, count); the host chained the
// batch's own segments of a connection already.
__global__ __launch_bounds__(kBlock) void k_tcp_link(TcpDev t, const uint32_t* __restrict__ q, uint32_t n) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = q[4 * i], tail = q[4 * i + 1], first = q[4 * i + 2], cnt = q[4 * i + 3];
  if (tail != kNoSeg) t.s_next[tail] = first;
  if (t.c_head[k] == kNoSeg) t.c_head[k] = first;
  if (t.c_una[k] == kNoSeg) t.c_una[k] = first;
  t.c_queued[k] += cnt;
}

// Every connection sends while its flight is below cwnd, each segment at max(written, t0): first the
// segments a loss episode marked lost (in order, the next attempt; settled ones are passed over, one
// of a failed write or out of attempts gives up), then new ones. Modes (kRel*):
//   at a write: t0 = the write times;
//   after a window: first the window's ACKs (flight, slow start / congestion avoidance) and resets (a
//     reset connection fails its queued writes at the window's end), t0 = max(the window's latest
//     intact ACK arrival, horizon) - what the ACKs let out leaves when they arrived, not at the window's
//     end; then fast retransmit [EXT RFC 5681 3.2]: once three segments after the oldest outstanding
//     one have been ACKed (three duplicate ACKs in a cumulative-ACK stack) and it has not, it is resent
//     at t0 (next attempt; once per segment), ssthresh = max(flight / 2, 2) and cwnd = ssthresh;
//   loss: at a window start, the connections whose timer expired in the window just begun (k_tcp_fire:
//     c_tloss) [EXT Linux tcp_enter_loss, RFC 5681 3.1]: ssthresh = max(cwnd / 2, 2) unless cwnd is
//     already 1 (the same episode), cwnd = 1, every outstanding segment marked lost and the queue
//     restarted at the oldest, t0 = max(expiry, window start).
// One thread per connection; staged slots and timer-list slots reserved once per block. A resent
// segment that still has an entry on the timer lists keeps it (the entry reads its new attempt).
__global__ __launch_bounds__(kBlock) void k_tcp_conn_release(TcpDev t, DevScalars* sc, uint32_t mode, uint32_t list,
                                                             uint32_t cap, uint32_t* __restrict__ m_src,
                                                             uint32_t* __restrict__ m_dst,
                                                             uint32_t* __restrict__ m_seq,
                                                             uint32_t* __restrict__ m_size,
                                                             int64_t* __restrict__ m_t) {
  __shared__ uint32_t red[kBlock / 64];
  __shared__ uint32_t sb_m, sb_p;
  const int64_t H = sc->T;
  const uint32_t n = t.n_conn;
  unsigned long long nretx = 0;
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < n; b0 += gridDim.x * kBlock) {  // block-uniform
    const uint32_t k = b0 + threadIdx.x;
    uint32_t go = 0, nent = 0, head = kNoSeg, end = kNoSeg, fr = kNoSeg;
    bool slow = false;
    const int64_t tfail = sc->t_end;
    int64_t t0 = mode == kRelAfterWindow ? sc->t_end : INT64_MIN;
    bool act = k < n;
    if (act && mode == kRelLoss) {
      const int64_t tl = t.c_tloss[k];
      act = tl != INT64_MAX;
      if (act) {
        t.c_tloss[k] = INT64_MAX;
        t0 = tl > H ? tl : H;
        const uint32_t cw = t.c_cwnd[k];
        if (cw > 1u) t.c_ssth[k] = cw / 2u > 2u ? cw / 2u : 2u;
        t.c_cwnd[k] = 1u;
        t.c_cnt[k] = 0u;
        const uint32_t h0 = t.c_head[k];
        uint32_t u = t.c_una[k];
        while (u != h0 && t.s_done[u]) u = t.s_next[u];
        t.c_una[k] = u;
        for (uint32_t x = u; x != h0; x = t.s_next[x])
          if (!t.s_done[x]) t.s_lost[x] = 1;
        t.c_head[k] = u;
        t.c_flight[k] = 0u;
      }
    }
    if (act) {
      uint32_t cw = t.c_cwnd[k], fl = t.c_flight[k];
      if (mode == kRelAfterWindow) {
        const uint32_t acks = t.c_acks[k];
        if (acks) {
          const uint32_t fa = t.c_fack[k];
          const int64_t ta = t.c_tack[k];
          t.c_acks[k] = 0u;
          t.c_fack[k] = 0u;
          t.c_tack[k] = INT64_MIN;
          t0 = ta > H ? ta : H;
          fl -= fa;
          t.c_acked[k] += acks;
          uint32_t ss = t.c_ssth[k], cnt = t.c_cnt[k];
          for (uint32_t a = 0; a < acks; ++a) {
            if (cw < ss) ++cw;
            else if (++cnt >= cw) { ++cw; cnt = 0u; }
            cw = cw > kCwndClamp ? kCwndClamp : cw;
          }
          // fast retransmit: the oldest outstanding segment, past three ACKed ones
          const uint32_t h0 = t.c_head[k];
          uint32_t u = t.c_una[k];
          while (u != h0 && t.s_done[u]) u = t.s_next[u];
          t.c_una[k] = u;

          if (u != h0 && !t.c_broken[k] && !t.s_lost[u] && t.c_fr[k] != u && t.s_att[u] + 1u < t.max_att) {
            const uint32_t ws = t.w_state[t.s_w[u] & kWMask];
            uint32_t dup = 0;
            for (uint32_t x = t.s_next[u]; x != h0 && dup < 3u; x = t.s_next[x]) dup += t.s_done[x] == 1;
            // the count leaves the loop as a value: this compiler (ROCm 7.2) otherwise reused the exit
            // test's lane mask of the last iteration for `dup >= 3`, losing it for every lane that left
            // earlier (a wave of connections where one walks further than another: no fast retransmit).
            // Reproduced standalone by tools/loopexit_repro.hip (25.6k of 65.5k lanes wrong without the
            // asm, none with it; profiles/r06/loopexit_repro.txt) and found statically by
            // tools/loopexit_audit.py, which finds no other such loop exit in the product kernels
#ifndef TGSIM_NO_WALK_ASM  // experiment build: the walk without the asm (tools/loopexit_repro.hip)
            __asm__ volatile("" : "+v"(dup));
#endif
            if (dup >= 3u && ws != TGSIM_TCP_TIMEOUT && ws != TGSIM_TCP_REFUSED) {
              fr = u;
              t.c_fr[k] = u;
              ss = fl / 2u > 2u ? fl / 2u : 2u;
              cw = ss;
              cnt = 0u;
              t.c_ssth[k] = ss;
              nent += t.s_tq[u] ? 0u : 1u;
            }
          }
          t.c_cwnd[k] = cw;
          t.c_cnt[k] = cnt;
          t.c_flight[k] = fl;
        }
        if (t.c_broken[k]) {  // a reset connection: its queued (and lost) segments' writes fail
          for (uint32_t sid = t.c_head[k]; sid != kNoSeg; sid = t.s_next[sid]) {
            const int64_t tw = t.s_tatt[sid];
            const uint32_t w = t.s_w[sid] & kWMask;
            t.s_done[sid] = 2;
            if (t.w_tarr[w] == INT64_MIN) tcp_fail(t, w, tw > tfail ? tw : tfail, TGSIM_TCP_REFUSED);
          }
          t.c_head[k] = kNoSeg;
          t.c_queued[k] = 0u;
        }
      }
      head = t.c_head[k];
      // a write onto a reset connection stays queued until the next reaction fails it at that
      // window's end (tgo_tcp_write releases only connections that are not broken)
      const uint32_t room = fl < cw && !t.c_broken[k] ? cw - fl : 0u;
      if (room && head != kNoSeg && !t.s_lost[head] && !t.s_done[head]) {  // only new segments from here
        go = min(room, t.c_queued[k]);
        nent += go;
      } else if (room) {  // segments marked lost first: count the sends, give up the hopeless ones
        slow = true;
        uint32_t sid = head;
        while (sid != kNoSeg && go < room) {
          const uint32_t nx = t.s_next[sid];
          if (!t.s_done[sid]) {
            const uint32_t w = t.s_w[sid] & kWMask;
            const uint32_t ws = t.w_state[w];
            if (t.s_lost[sid] && (ws == TGSIM_TCP_TIMEOUT || ws == TGSIM_TCP_REFUSED || t.s_att[sid] + 1u >= t.max_att)) {
              const int64_t tw = t.s_tatt[sid];
              t.s_lost[sid] = 0;
              t.s_done[sid] = 2;
              if (t.w_tarr[w] == INT64_MIN) tcp_fail(t, w, tw > t0 ? tw : t0, TGSIM_TCP_TIMEOUT);
            } else {
              ++go;
              nent += t.s_tq[sid] ? 0u : 1u;
            }
          }
          sid = nx;
        }
        end = sid;  // past the last send and any segment given up behind it
        if (go == 0) t.c_head[k] = end;
      }
    }
    uint32_t tm, tp;
    const uint32_t nfr = fr != kNoSeg ? 1u : 0u;
    const uint32_t pm = block_excl_scan(go + nfr, red, tm);
    const uint32_t pp = block_excl_scan(nent, red, tp);
    if (threadIdx.x == 0) {
      sb_m = tm ? reserve_staged(&sc->n_msgs_dev, tm, cap) : 0u;
      sb_p = tp ? atomicAdd(&t.sc->pend_n[list], tp) : 0u;
    }
    __syncthreads();
    uint32_t e = 0;
    if (nfr) {  // the fast retransmission, first; it keeps its flight slot
      const uint32_t src = t.c_src[k], a = t.s_att[fr] + 1u, p = sb_m + pm;
      t.s_att[fr] = a;
      t.s_tatt[fr] = t0;
      t.s_w[fr] |= kRetxBit;
      atomicAdd(&t.pend_by[src], 1u);
      ++nretx;
      if (p < cap) {
        m_src[p] = src; m_dst[p] = t.c_dst[k]; m_seq[p] = (fr << 4) | a; m_size[p] = t.s_wire[fr]; m_t[p] = t0;
      } else {
        atomicOr(&sc->err, ERR_CAP_M);
      }
      if (!t.s_tq[fr]) {
        t.s_tq[fr] = 1;
        t.pend[list][sb_p + pp + e++] = fr;
      }
    }
    if (go) {
      uint32_t sid = head, sent = 0, qd = 0;
      const uint32_t src = t.c_src[k], dst = t.c_dst[k];
      while (sent < go) {
        const uint32_t nx = t.s_next[sid];
        if (!t.s_done[sid]) {
          const int64_t tw = t.s_tatt[sid], ts = tw > t0 ? tw : t0;
          uint32_t seq = sid << 4;
          if (t.s_lost[sid]) {  // the next attempt of a segment marked lost
            const uint32_t a = t.s_att[sid] + 1u;
            t.s_att[sid] = a;
            t.s_lost[sid] = 0;
            t.s_w[sid] |= kRetxBit;
            seq |= a;
            atomicAdd(&t.pend_by[src], 1u);  // released into the window until its status is read
            ++nretx;
          } else {
            ++qd;
          }
          t.s_tatt[sid] = ts;
          const uint32_t p = sb_m + pm + nfr + sent;
          if (p < cap) {
            m_src[p] = src; m_dst[p] = dst; m_seq[p] = seq; m_size[p] = t.s_wire[sid]; m_t[p] = ts;
          } else {
            atomicOr(&sc->err, ERR_CAP_M);
          }
          if (!t.s_tq[sid]) {  // its timer
            t.s_tq[sid] = 1;
            t.pend[list][sb_p + pp + e++] = sid;
          }
          ++sent;
        }
        sid = nx;
      }
      t.c_head[k] = slow ? end : sid;
      t.c_flight[k] += go;
      t.c_queued[k] -= qd;
    }
    __syncthreads();  // sb_m / sb_p are rewritten by the next round
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nretx += __shfl_xor(nretx, o);
  if (lane_id() == 0 && nretx) {
    atomicAdd(&t.sc->retx, nretx);
    atomicAdd(&t.sc->released, nretx);
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
    m_seq[m] = tcp_wire(t, sid) << 4;
    m_size[m] += t.hdr;
  }
}

// Sharded: the window's data copies delivered here for another shard's writers, each to its writer's
// shard as its delivery record (t, src, dst, seq; meta = the delivery flags), one reservation per wave
// and peer on the peer's cursor (xq[p << 5], zeroed by the host before)
__global__ __launch_bounds__(kBlock) void k_tcp_fwd(const uint32_t* __restrict__ o_src,
                                                    const uint32_t* __restrict__ o_dst,
                                                    const uint32_t* __restrict__ o_seq,
                                                    const int64_t* __restrict__ o_t,
                                                    const uint32_t* __restrict__ o_flags, DevScalars* sc, TcpDev t) {
  const uint32_t n = sc->n_out;
  for (uint32_t i0 = blockIdx.x * kBlock; i0 < n; i0 += gridDim.x * kBlock) {  // wave-uniform trip count
    const uint32_t i = i0 + threadIdx.x;
    uint32_t p = kNoPeer;
    if (i < n) {
      const uint32_t sq = o_seq[i], src = o_src[i];
      if (!(t.acks && (sq & TGSIM_TCP_ACK_BIT)) && !tcp_mine(t, src)) p = shard_of_inv(src, t.S, t.inv);
    }
    bool pending = p != kNoPeer;
    for (;;) {  // the lanes of one peer share a reservation
      const uint64_t m = __ballot(pending);
      if (m == 0) break;
      const int leader = __ffsll((unsigned long long)m) - 1;
      const uint32_t lp = __shfl(p, leader);
      const bool mine = pending && p == lp;
      const uint64_t mm = __ballot(mine);
      uint32_t base = 0;
      if ((int)lane_id() == leader) base = atomicAdd(t.xq + (lp << 5), (uint32_t)__popcll(mm));
      base = __shfl(base, leader);
      if (mine) {
        const uint32_t pos = base + mask_rank(mm);
        if (pos < t.xcap - 1u) {
          tgsim_record r;
          r.t = o_t[i]; r.src = o_src[i]; r.dst = o_dst[i]; r.seq = o_seq[i]; r.size = 0; r.meta = o_flags[i];
          r.corrupt_off = 0;
          t.xsend[(size_t)p * t.xcap + 1 + pos] = r;
        } else {
          atomicOr(&sc->err, ERR_CAP_X);
        }
        pending = false;
      }
    }
  }
}

// Sharded: the forward blocks' headers (counts from the cursors)
__global__ void k_tcp_xheaders(TcpDev t) {
  const uint32_t p = threadIdx.x;
  if (p >= t.S) return;
  tgsim_record h;
  h.t = (int64_t)min(t.xq[p << 5], t.xcap - 1u);
  h.src = h.dst = h.seq = h.size = h.meta = h.corrupt_off = 0;
  t.xsend[(size_t)p * t.xcap] = h;
}

// Sharded: the copies other shards delivered for this shard's writers join the reaction's inputs
// behind the window's own deliveries (o_* from n_out on: the delivery API reads [0, n_out)); every
// block takes the peers' counts (S <= 64) and their prefix itself
__global__ __launch_bounds__(kBlock) void k_tcp_rx(DevScalars* sc, TcpDev t, uint32_t cap, uint32_t* __restrict__ o_src,
                                                   uint32_t* __restrict__ o_dst, uint32_t* __restrict__ o_seq,
                                                   int64_t* __restrict__ o_t, uint32_t* __restrict__ o_flags) {
  __shared__ uint32_t off[kMaxShards + 1];
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    bool bad = false;
    for (uint32_t p = 0; p < t.S; ++p) {
      off[p] = a;
      const int64_t np = p == t.shard ? 0 : t.xrecv[(size_t)p * t.xcap].t;
      bad |= np < 0 || np >= (int64_t)t.xcap;
      a += (np < 0 || np >= (int64_t)t.xcap) ? 0u : (uint32_t)np;
    }
    off[t.S] = a;
    if (bad && blockIdx.x == 0) atomicOr(&sc->err, ERR_EXCH_HDR);
  }
  __syncthreads();
  const uint32_t base = sc->n_out, tot = off[t.S];
  const uint32_t room = cap > base ? cap - base : 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t.sc->n_in = base + min(tot, room);
    if (tot > room) atomicOr(&sc->err, ERR_CAP_D);
  }
  for (uint32_t j = blockIdx.x * kBlock + threadIdx.x; j < min(tot, room); j += gridDim.x * kBlock) {
    uint32_t p = 0;
    while (p + 1 < t.S && off[p + 1] <= j) ++p;
    const tgsim_record r = t.xrecv[(size_t)p * t.xcap + 1 + (j - off[p])];
    const uint32_t k = base + j;
    o_src[k] = r.src; o_dst[k] = r.dst; o_seq[k] = r.seq; o_t[k] = r.t; o_flags[k] = r.meta;
  }
}

}  // namespace

hipError_t launch_tcp_fwd(Dev& d, TcpDev& t) {
  if (hipMemsetAsync(t.xq, 0, (size_t)t.S * 128, d.stream) != hipSuccess) return hipGetLastError();
  hipLaunchKernelGGL(k_tcp_fwd, dim3(kTcpArriveBlocks), dim3(kBlock), 0, d.stream, d.o_src, d.o_dst, d.o_seq, d.o_t,
                     d.o_flags, d.sc, t);
  hipLaunchKernelGGL(k_tcp_xheaders, dim3(1), dim3(kMaxShards), 0, d.stream, t);
  return hipGetLastError();
}

hipError_t launch_tcp_adopt(Dev& d, TcpDev& t, uint32_t base, uint32_t n, uint32_t wbase, uint32_t sbase) {
  if (!n) return hipSuccess;
  const unsigned g = std::min<unsigned>((n + kBlock - 1) / kBlock, (unsigned)kStreamBlocks);
  hipLaunchKernelGGL(k_tcp_adopt, dim3(g), dim3(kBlock), 0, d.stream, t, base, n, wbase, sbase, d.m_src, d.m_dst,
                     d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

hipError_t launch_tcp_link(Dev& d, TcpDev& t, const uint32_t* links, uint32_t n) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_tcp_link, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, d.stream, t, links, n);
  return hipGetLastError();
}

hipError_t launch_tcp_conn_release(Dev& d, TcpDev& t, uint32_t mode, uint32_t cur, bool base_dev,
                                   uint32_t base_host) {
  if (!t.n_conn) return hipSuccess;
  if (!base_dev) hipLaunchKernelGGL(k_tcp_base, dim3(1), dim3(kBlock), 0, d.stream, d.sc, base_host);
  const unsigned g = std::min<unsigned>((t.n_conn + kBlock - 1) / kBlock, (unsigned)kStreamBlocks);
  hipLaunchKernelGGL(k_tcp_conn_release, dim3(g), dim3(kBlock), 0, d.stream, t, d.sc, mode, cur, d.cap_msgs, d.m_src,
                     d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

#ifndef TG_TCP_COLLECT_BLOCKS
#define TG_TCP_COLLECT_BLOCKS 256  // a thread walks one bitmap word's retransmissions (64 blocks: 18.6 us)
#endif
hipError_t launch_tcp_react(Dev& d, TcpDev& t, uint32_t cur, uint32_t n_host, const uint32_t* n_dev, uint32_t epoch,
                            uint32_t fill) {
  hipLaunchKernelGGL(k_tcp_reset, dim3(1), dim3(kBlock), 0, d.stream, t, cur, d.sc, fill);
  if (t.S > 1)  // after the forward exchange (launch_tcp_fwd + the transport's all-to-all)
    hipLaunchKernelGGL(k_tcp_rx, dim3(kTcpArriveBlocks), dim3(kBlock), 0, d.stream, d.sc, t, (uint32_t)kNSub * d.subcap,
                       d.o_src, d.o_dst, d.o_seq, d.o_t, d.o_flags);
  hipLaunchKernelGGL(k_tcp_status, dim3(kStreamBlocks), dim3(kBlock), 0, d.stream, d.status, d.m_seq, n_host, n_dev, t);
  hipLaunchKernelGGL(k_tcp_arrive, dim3(kTcpArriveBlocks), dim3(kBlock), 0, d.stream, d.o_src, d.o_seq, d.o_t, d.o_flags,
                     d.sc, t);
  hipLaunchKernelGGL(k_tcp_settle, dim3(kTcpArriveBlocks), dim3(kBlock), 0, d.stream, d.o_seq, d.sc, t, epoch, cur);
  hipLaunchKernelGGL(k_tcp_collect, dim3(TG_TCP_COLLECT_BLOCKS), dim3(kBlock), 0, d.stream, d.m_seq, n_host, n_dev, d.o_seq, d.sc, t, cur,
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

hipError_t launch_tcp_release_acks(Dev& d, TcpDev& t, uint32_t cur, bool base_dev, uint32_t base_host, uint32_t head,
                                   bool reg, uint32_t lo, uint32_t hi) {
  if (!base_dev) hipLaunchKernelGGL(k_tcp_base, dim3(1), dim3(kBlock), 0, d.stream, d.sc, base_host);
  hipLaunchKernelGGL(k_tcp_tplan, dim3(1), dim3(kBlock), 0, d.stream, t, d.sc, head, reg ? 1u : 0u, lo, hi, d.cap_msgs);
  hipLaunchKernelGGL(k_tcp_fire, dim3(kStreamBlocks), dim3(kBlock), 0, d.stream, t, d.sc, cur, d.cap_msgs, d.o_src, d.o_dst,
                     d.o_seq, d.o_t, d.m_src, d.m_dst, d.m_seq, d.m_size, d.m_t);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // loss episodes of the connections whose timer fired: their resends' timers join the kept list
  return launch_tcp_conn_release(d, t, kRelLoss, cur ^ 1u, true, 0);
}

}  // namespace tgsim
