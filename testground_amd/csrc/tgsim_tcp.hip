// tgsim_tcp.hip — TCP mode (tgsim_tcp_*): segmentation and loss recovery over the
// per-packet path, for the reference plans that move data over TCP (plans/benchmarks/storm.go:
// 127-180, plans/network/pingpong.go:73-104). Packets are ordinary staged messages with
// seq = segment * 16 + attempt; after every window the reaction reads the window's packet statuses
// and deliveries where the pipeline left them:
//   k_tcp_status   per packet: copies that entered the egress queue (status flags) -> the segment's
//                  outstanding copies; none: refused route (the write fails) or a retransmission at
//                  t_a + rto * 2^a
//   k_tcp_arrive   per delivery: first intact arrival (atomicMin), latest copy (atomicMax), one
//                  outstanding copy fewer
//   k_tcp_settle   per delivery, one thread per segment (epoch claim): a segment that arrived counts
//                  down its write (the last one delivers it); one whose copies all arrived corrupted
//                  is retransmitted at max(t_a + rto * 2^a, its latest copy)
//   k_tcp_release  at the next window start: due retransmissions appended to the staged messages
//                  (device-side count), the rest kept for a later window
// Every decision is order-independent, so the result equals the oracle's
// sequential pass although threads race.
#include "tgsim_dev.h"

namespace tgsim {

namespace {

constexpr uint32_t kArrived = 1u;

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

// attempt s_att[sid] failed, known at t_known: the next one, or the write times out
__device__ __forceinline__ void tcp_schedule(TcpDev& t, uint32_t sid, int64_t t_known, uint32_t cur) {
  const uint32_t a = t.s_att[sid];
  int64_t tn = t.s_tatt[sid] + (t.rto << a);
  tn = tn < t_known ? t_known : tn;
  if (a + 1u >= t.max_att) {
    tcp_fail(t, t.s_w[sid], tn, TGSIM_TCP_TIMEOUT);
    return;
  }
  t.s_att[sid] = a + 1u;
  t.s_tatt[sid] = tn;
  t.s_tlast[sid] = INT64_MIN;
  t.pend[cur][atomicAdd(&t.sc->pend_n[cur], 1u)] = sid;
  atomicAdd(&t.sc->retx, 1ull);
}

__global__ __launch_bounds__(kBlock) void k_tcp_status(const uint8_t* __restrict__ status,
                                                       const uint32_t* __restrict__ seq, uint32_t n_host,
                                                       const uint32_t* n_dev, TcpDev t, uint32_t cur) {
  const uint32_t n = n_dev ? *n_dev : n_host;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sid = seq[i] >> 4;
    const uint8_t st = status[i];
    const uint32_t q = tcp_copies(st);
    if (q) {
      atomicAdd(&t.s_out[sid], q);
      continue;
    }
    const uint32_t code = st & 0x0Fu;
    if (code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) tcp_fail(t, t.s_w[sid], t.s_tatt[sid], TGSIM_TCP_REFUSED);
    else tcp_schedule(t, sid, t.s_tatt[sid], cur);
  }
}

__global__ __launch_bounds__(kBlock) void k_tcp_arrive(const uint32_t* __restrict__ o_seq,
                                                       const int64_t* __restrict__ o_t,
                                                       const uint32_t* __restrict__ o_flags, const DevScalars* sc,
                                                       TcpDev t) {
  const uint32_t n = sc->n_out;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sid = o_seq[i] >> 4;
    const long long ti = (long long)o_t[i];
    if (!(o_flags[i] & TGSIM_F_CORRUPT)) atomicMin(reinterpret_cast<long long*>(&t.s_arr[sid]), ti);
    atomicMax(reinterpret_cast<long long*>(&t.s_tlast[sid]), ti);
    atomicSub(&t.s_out[sid], 1u);
  }
}

__global__ __launch_bounds__(kBlock) void k_tcp_settle(const uint32_t* __restrict__ o_seq, const DevScalars* sc,
                                                       TcpDev t, uint32_t epoch, uint32_t cur) {
  const uint32_t n = sc->n_out;
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    const uint32_t sid = o_seq[i] >> 4;
    if (atomicExch(&t.s_mark[sid], epoch) == epoch) continue;  // one thread per segment
    if (t.s_flags[sid] & kArrived) continue;
    const int64_t arr = t.s_arr[sid];
    if (arr != INT64_MAX) {
      t.s_flags[sid] |= kArrived;
      const uint32_t w = t.s_w[sid];
      atomicMax(reinterpret_cast<long long*>(&t.w_tarr[w]), (long long)arr);
      __threadfence();
      if (atomicSub(&t.w_rem[w], 1u) == 1u &&
          atomicCAS(&t.w_state[w], (uint32_t)TGSIM_TCP_PENDING, (uint32_t)TGSIM_TCP_DELIVERED) == TGSIM_TCP_PENDING) {
        atomicAdd(&t.sc->done, 1u);
        atomicAdd(&t.sc->delivered, 1ull);
      }
    } else if (t.s_out[sid] == 0) {
      tcp_schedule(t, sid, t.s_tlast[sid], cur);
    }
  }
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
    const uint32_t sid = t.pend[cur][i], w = t.s_w[sid];
    if (t.w_state[w] != TGSIM_TCP_PENDING) continue;  // the write has failed: nothing more is sent
    const int64_t ta = t.s_tatt[sid];
    if (ta >= t_end) {
      t.pend[nxt][atomicAdd(&t.sc->pend_n[nxt], 1u)] = sid;
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

}  // namespace

hipError_t launch_tcp_react(Dev& d, TcpDev& t, uint32_t cur, uint32_t n_host, const uint32_t* n_dev, uint32_t epoch) {
  hipLaunchKernelGGL(k_tcp_reset, dim3(1), dim3(kBlock), 0, d.stream, t, cur);
  hipLaunchKernelGGL(k_tcp_status, dim3(kStreamBlocks), dim3(kBlock), 0, d.stream, d.status, d.m_seq, n_host, n_dev, t,
                     cur);
  hipLaunchKernelGGL(k_tcp_arrive, dim3(kStreamBlocks), dim3(kBlock), 0, d.stream, d.o_seq, d.o_t, d.o_flags, d.sc, t);
  hipLaunchKernelGGL(k_tcp_settle, dim3(kStreamBlocks), dim3(kBlock), 0, d.stream, d.o_seq, d.sc, t, epoch, cur);
  return hipGetLastError();
}

hipError_t launch_tcp_release(Dev& d, TcpDev& t, uint32_t cur, uint32_t n_pending, bool base_dev, uint32_t base_host) {
  if (!base_dev) hipLaunchKernelGGL(k_tcp_base, dim3(1), dim3(kBlock), 0, d.stream, d.sc, base_host);
  const unsigned g = std::min<unsigned>((n_pending + kBlock - 1) / kBlock, (unsigned)kStreamBlocks);
  hipLaunchKernelGGL(k_tcp_release, dim3(g ? g : 1), dim3(kBlock), 0, d.stream, t, cur, d.sc, d.cap_msgs, d.m_src,
                     d.m_dst, d.m_seq, d.m_size, d.m_t);
  return hipGetLastError();
}

}  // namespace tgsim
