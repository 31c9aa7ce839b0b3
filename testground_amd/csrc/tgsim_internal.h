// tgsim_internal.h — device-side data layout and helpers shared by the gfx950 kernels and the host
// runtime of libtgsim.so. Semantics: DESIGN.md section 2. Layout rationale: DESIGN.md section 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tgsim.h"

namespace tgsim {

constexpr int kBlock = 256;              // threads per workgroup (4 wave64)
constexpr int kTile = 1024;              // small-segment tile: segments <= kTile sorted in LDS
constexpr int kSpan = 2 * kTile;         // LDS capacity of one small-segment span
constexpr int kThreadSeg = 16;          // segments up to this long: one thread each (k_seg_thread)
constexpr int kListBlocks = 1024;       // grid of k_seg_list (device-side count)
constexpr int kChunk = 2048;             // large-segment chunk (LDS bitonic) and merge tile
constexpr int kRadixBlocks = 256;        // fixed grid of the radix group-by passes (<= 1024: k_radix_rows block)
constexpr int kMaxDigitBits = 11;        // radix digit width <= 11 bits (2048 bins)
constexpr int kMaxBins = 1 << kMaxDigitBits;
constexpr int kNSub = 64;                // append sub-queues per batch (contention sharding)
constexpr int kRankSortMax = 64;         // segments up to this length are rank-sorted in LDS
constexpr int kMaxShards = 64;
// Exchange blocks (sharded runs): peer p's block of xcap records is a header and kXSlices slices of
// x_slice_cap(xcap) records, slice g written only by workgroups of XCD g (blockIdx % 8) through its
// own cursor, so a window's ~1000 token-bucket workgroups no longer serialise on one cursor per peer
// (DESIGN.md 6); the header record's eight 32-bit words are the slices' counts. A block too small to
// split (xcap - 1 < 8 * 64) is one slice: the header's t is its count, as before.
constexpr uint32_t kXSlices = 8;
__host__ __device__ inline uint32_t x_slices(uint32_t xcap) { return xcap - 1u >= kXSlices * 64u ? kXSlices : 1u; }
__host__ __device__ inline uint32_t x_slice_cap(uint32_t xcap) { return (xcap - 1u) / x_slices(xcap); }
// A / D / L sub-queue counters, then the exchange cursors (peer p, slice g) at line 3 kNSub + p kXSlices + g,
// then the deferred-message sub-lists' counters (k_shape: message chunk c appends to sub-list c % kDeferSub)
constexpr int kDeferSub = 16;
constexpr int kQcDefer = 3 * kNSub + kXSlices * kMaxShards;
constexpr int kQcRest = kQcDefer + kDeferSub;  // k_rest_local_hist: role tickets, then rest roles done
constexpr int kQcLines = kQcRest + 2;
// capacity of one deferred-message sub-list: sub-list s takes chunks s, s + kDeferSub, ... of 256
// messages, at most ceil(chunks / kDeferSub) of them
__host__ __device__ inline uint32_t defer_seg_cap(uint32_t cap_msgs) {
  return ((cap_msgs + 255u) / 256u + (uint32_t)kDeferSub - 1u) / (uint32_t)kDeferSub * 256u;
}
constexpr int kMaxRegions = 8192;        // live timing-wheel regions (one per window)
constexpr int kStreamBlocks = 2048;      // grid of grid-stride streaming kernels
constexpr int64_t kNegInf = INT64_MIN / 4;
constexpr int64_t kTbClamp = (int64_t)1 << 61;
constexpr uint64_t kCostClamp = (uint64_t)1 << 52;
constexpr uint32_t kExternalIp = 0x08080808u;
constexpr uint32_t kNetemSalt = 0x4E45544Du;  // "NETM": 4th Philox counter word of netem draws
constexpr uint32_t kStormSalt = 0x53544F52u;  // "STOR": storm generator draws

// device error bits (DevScalars::err)
enum : uint32_t {
  ERR_CAP_A = 1u << 0, ERR_CAP_D = 1u << 1, ERR_CAP_L = 1u << 2, ERR_CAP_X = 1u << 3,
  ERR_ARENA = 1u << 4, ERR_REGIONS = 1u << 5, ERR_CAUSAL = 1u << 6, ERR_SIG_ORDER = 1u << 7,
  ERR_UNRELEASED = 1u << 8, ERR_SIG_CAP = 1u << 9, ERR_TASKS = 1u << 10, ERR_EXCH_HDR = 1u << 11,
  ERR_BAD_MSG = 1u << 12, ERR_STATE_CHUNKS = 1u << 13, ERR_UNSORTED_TARGET = 1u << 14,
  ERR_QUEUE_CAP = 1u << 15,  // a sender's queue bookkeeping outgrew kSeqCap (cannot happen with limit 1000)
  ERR_CAP_M = 1u << 16,      // device-counted staging (flood forwards, appends after them) outgrew cap_msgs
  ERR_TCP_TIMERS = 1u << 17, // TCP acks mode: more live timer batches than the ring holds
  ERR_PROBE_SPAN = 1u << 18  // probe reaction: a request arrival more than 2^40 ns before the window end
  // ERR_TASKS: a large-segment rank task waited past its bound for its chunks (k_rest; never expected)
};

// Per-sender egress state derived from network.LinkShape (48 B; gathered by src).
struct alignas(16) ShapeDev {
  int64_t mu;        // netem latency (ns)
  int64_t tau;       // HTB buffer (ns)
  int32_t sigma;     // netem jitter (ns) as tabledist's s32
  uint32_t loss_t, dup_t, corrupt_t, reorder_t;
  uint32_t mult, shift, flags;    // HTB rate as multiply-shift; flags: kShLimited, kShCorr
};
static_assert(sizeof(ShapeDev) == 48, "ShapeDev layout");

// The token bucket's share of ShapeDev (16 B; gathered by sender in k_tb_bucket / k_rest<TB>, where
// the 48 B entry cost a third of the flood's token-bucket traffic).
struct alignas(16) TbShape {
  int64_t tau;
  uint32_t mult, shift;
};
static_assert(sizeof(TbShape) == 16, "TbShape layout");
constexpr uint32_t kShLimited = 1u;  // Bandwidth != 0
constexpr uint32_t kShCorr = 2u;     // a correlated netem draw is used (messages deferred to k_shape_corr)

struct RuleDev {           // per-sender routing rule, CSR, sorted (plen desc, prefix asc)
  uint32_t prefix;
  uint32_t plen_action;    // plen | action << 8
};

// One live timing-wheel region: the "later" records of one window, bucketed by delivery/ready slot.
struct RegionDev {
  uint64_t arena_off;      // first record in the arena ring
  uint32_t n;              // records
  uint32_t consumed;       // records already extracted (a prefix in slot order)
  int64_t base_slot;       // absolute slot of region slot 0 (= floor(window end / slot_ns))
  uint32_t dir;            // directory index (slot offsets at dirs[dir * (slots + 1)])
  uint32_t pad;
};

// Device-resident scalars of one ctx. Host writes them only through kernels / memsets.
enum { Q_A = 0, Q_D = 1, Q_L = 2, Q_X0 = 3 };  // append queues: TB batch, deliveries, wheel, peers
struct DevScalars {
  int64_t T, t_end;                  // current window
  int64_t H;                         // reaction horizon: earliest admissible t_send
  int64_t base_slot;                 // t_end / slot_ns: timing-wheel slot 0 of this window's insertions
  // ---- per-window block: zeroed by one memset at window start ----
  uint32_t q[Q_X0 + kMaxShards];     // unused (round 4's exchange cursors; now lines of qc, Queues::xctr)
  uint32_t qpre[3][kNSub + 1];       // A, D, L: prefix over sub-queues (after k_qfinal)
  uint32_t qn[3];                    // A, D, L: totals (after k_qfinal)
  uint32_t n_extract;                // records extracted from the wheel this window
  uint32_t plan_tail, plan_n;        // region ring range the extraction plan covers
  uint32_t n_large, max_large, n_chunks;
  uint32_t n_medium;                 // segments for the block-per-segment kernel (k_seg_list)
  uint32_t n_recv, n_out;
  uint32_t n_corr;                   // messages deferred by k_shape (correlated or queue-heavy senders)
  uint32_t n_hrec;                   // due wheel records of queue-heavy senders copied to the H list
  uint32_t seq_left;                 // senders k_shape_seq_wide left to k_shape_seq (0: it has nothing to do)
  uint32_t rest_tb;                  // k_tb_bucket listed long senders for k_rest<TB> (k_rest_local_hist)
  // ---- persistent ----
  uint32_t err;                      // sticky ERR_* bits
  uint32_t reg_head, reg_tail;       // region ring (monotonic counters; slot = counter % kMaxRegions)
  uint32_t sig_n;                    // size of the signal batch being processed
  uint64_t arena_head, arena_tail, arena_used, ins_off;  // arena ring (records)
  uint64_t sig_log_used;             // signal log entries used
  uint32_t pend_max;                 // max over local senders of queued copies (k_pend_max, host gate)
  uint32_t rest_tb_last;             // the last window end's rest_tb (a host hint, read at sync points)
  // device-counted staging: once the flood reaction stages its forwards, the staged
  // count lives here (appends go after it); the window's shape pass reads it, window end moves it
  // to n_msgs_last (the status count of that window) and clears it
  uint32_t n_msgs_dev, n_msgs_last;
  uint32_t fl_total, pad_fl;         // forwards staged by the last flood reaction
  // cumulative statistics (tgsim_stats)
  unsigned long long st[13];
  // cumulative implementation counters (tgsim_kernel_counters; bench.py attributes SURVEY.md 8(d)
  // bytes to the kernels that move them): KC_*
  unsigned long long kc[5];
};
enum { KC_DEFERRED = 0,   // messages decided in the sequential lane (k_shape_seq)
       KC_LONG_TB = 1,    // token-bucket copies of senders with long runs (k_rest<TB>)
       KC_LONG_EMIT = 2,  // deliveries of long inboxes, written by k_rest<Emit> (the wheel-insert launch)
       KC_WIDE = 3,       // deferred messages decided by k_shape_seq_wide (the rest: k_shape_seq)
       KC_WHOLE = 4,      // of KC_LONG_EMIT: inboxes sorted whole by one workgroup (whole_sort, -DTGSIM_WHOLE_SORT)
       KC_COUNT = 5 };
enum { ST_MSGS = 0, ST_COPIES, ST_LOST, ST_DROPPED, ST_REJECTED, ST_UNREACH, ST_EXTERNAL, ST_DESTDOWN,
       ST_LOCAL, ST_DELIVERED, ST_TB_ITEMS, ST_EXTRACTED, ST_INSERTED };
constexpr int ST_OVERLIMIT = 13;  // a row counter only ([kNSub][16] rows; ST_DELIVERED.. live in DevScalars::st)

// Netem's queue limit. A local sender is "queue-heavy" in a window when the copies
// it has queued (pend: its records in the timing wheel at the window start) plus every copy it
// could add in the window may reach the limit; only then are its messages decided sequentially
// (k_shape_seq). m_uniform bounds the messages any sender stages in the window, m_inbox * (its last
// inbox run) the flood forwards; mult = 2 when some shape duplicates.
// A sender with a zero-delay, unshaped link (latency 0, jitter 0, no HTB: every copy departs at its
// enqueue instant, so the next enqueue finds it gone) adds nothing to its own queue: only the copies
// queued at the window start (pend) can count, and it is heavy only when they alone reach the limit
// (zd: bit per local sender, from the shape table). The splitbrain target that receives 10k requests
// in a window then answers them in the parallel netem pass instead of one wave's chunk walk.
// Per-sender queue occupancy (pend): local sender l's count is word l << sh. The deliveries
// decrement the counts with memory-side atomics, which serialise per line: a small shard's counts
// in a few lines (config 2: 1000 senders in 32 lines, ~250k decrements per window) queued every
// delivery workgroup behind the others, so up to kPendSpreadMax senders each count gets a 128-B
// line of its own.
#ifndef TG_PEND_SPREAD_MAX
#define TG_PEND_SPREAD_MAX 16384u
#endif
constexpr uint32_t kPendSpreadMax = TG_PEND_SPREAD_MAX;
__host__ __device__ constexpr uint32_t pend_shift(uint32_t nloc) { return nloc <= kPendSpreadMax ? 5u : 0u; }
struct PendRef {
  uint32_t* p;
  uint32_t sh;
  __host__ __device__ uint32_t& operator[](uint32_t l) const { return p[(size_t)l << sh]; }
  __host__ __device__ explicit operator bool() const { return p != nullptr; }
};

struct Heavy {
  PendRef pend;           // null: the host proved no sender can reach the limit this window
  const uint32_t* inbox;  // [nloc + 1] the last window's inbox offsets (flood forwards), or nullptr
  const uint32_t* retx;   // TCP mode: [nloc] retransmissions pending or released into this window
  const uint32_t* zd;     // [nloc / 32 + 1] zero-delay unshaped senders
  uint32_t m_uniform, m_inbox, mult;
  __host__ __device__ bool of(uint32_t l) const {
    if (!pend) return false;
    if (zd && ((zd[l >> 5] >> (l & 31u)) & 1u)) return pend[l] >= TGSIM_NETEM_LIMIT;
    uint64_t m = m_uniform;
    if (m_inbox) m += (uint64_t)m_inbox * (inbox[l + 1] - inbox[l]);
    if (retx) m += retx[l];
    return (uint64_t)pend[l] + mult * m > TGSIM_NETEM_LIMIT;
  }
};

struct LargeSeg { uint32_t seg, start, len, pad; };
struct SigChunk {  // a run of consecutive sequence numbers of one state
  uint32_t seq_start, len;
  uint64_t log_pos;          // times in seq order at sig_log[log_pos..] (sorted chunks)
  int64_t tmin, tmax;
  uint32_t sorted, pad;
};
constexpr int kMaxChunksPerState = 64;

// Sort element of the segmented sorts: order (seg, k1, k2, k3).
struct SortKey {
  uint32_t seg;
  uint64_t k1, k2;
  uint32_t k3;
};

__host__ __device__ inline bool key_less(uint32_t sa, uint64_t a1, uint64_t a2, uint32_t a3,
                                         uint32_t sb, uint64_t b1, uint64_t b2, uint32_t b3) {
  if (sa != sb) return sa < sb;
  if (a1 != b1) return a1 < b1;
  if (a2 != b2) return a2 < b2;
  return a3 < b3;
}

// Philox4x32-10 (Random123 constants). Counter-based: draws are a pure function of
// (key = run seed, counter = (message id, sender, copy|block, salt)).
__host__ __device__ inline void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Shard k owns [floor(kN/S), floor((k+1)N/S)); the owner of g is floor(((g+1)S - 1)/N).
__host__ __device__ inline uint32_t shard_of(uint32_t g, uint32_t N, uint32_t S) {
  return (uint32_t)((((uint64_t)g + 1) * S - 1) / N);
}
// The same division by a multiply-high: inv = floor(2^64 / N) + 1 makes floor(x * inv / 2^64) =
// floor(x / N) exact for every x with x * N < 2^64 (x = (g + 1) S - 1 < 2^38 here). A 64-bit integer
// division is a ~100-instruction software routine on the GPU; per routed copy it made a sharded
// token bucket slower than the same shard alone (50k instances: 28-30 us -> 26.8 against 20.6; the
// rest was the single exchange cursor per peer, now sliced: kXSlices).
inline uint64_t shard_inv(uint32_t N) { return N ? (uint64_t)(((unsigned __int128)1 << 64) / N) + 1 : 0; }
__device__ __forceinline__ uint32_t shard_of_inv(uint32_t g, uint32_t S, uint64_t inv) {
  return (uint32_t)__umul64hi(((uint64_t)g + 1) * S - 1, inv);
}

// One-sided agent-scope fences: a producer that publishes data through a counter needs only the
// release half (its XCD's L2 written back), a consumer only the acquire half (stale lines dropped);
// __threadfence() does both in every workgroup that runs it.
__device__ inline void fence_release_agent() {
#ifdef TGSIM_FULL_FENCE
  __threadfence();
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
}
__device__ inline void fence_acquire_agent() {
#ifdef TGSIM_FULL_FENCE
  __threadfence();
#else
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
}
// A workgroup publishes its stores through a counter one lane updates (MI355X_MICROARCH.md
// § visibility, valid producer form): every storing wave waits for its stores, the barrier, then ONE
// agent-scope release by the counting lane, then that lane's atomic. One L2 write-back per workgroup
// instead of one per wave, and correct by the model: the release covers the other waves' stores
// because they completed before the barrier. The release lowers to
// `buffer_wbl2 sc1; s_waitcnt vmcnt(0)` on gfx950 (ROCm 7.2): round 5 added a second wait after it
// on the suspicion that the compiler could drop its own; tools/fence_isa.sh checks every write-back
// of the product kernels is followed by its wait (profiles/r06/fence_isa.txt), so that wait is gone.
// Call from every thread; returns true on the counting lane (thread 0).
__device__ inline bool block_release_for_count() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return false;
#ifdef TGSIM_FULL_FENCE
  __threadfence();
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
  return true;
}
// The consumer side: the polling lane (thread 0) has seen the count; ONE agent-scope acquire drops
// this CU's stale lines, its wait holds the barrier until the invalidate is done, then every wave
// loads. Call from every thread.
__device__ inline void block_acquire_after_poll() {
  if (threadIdx.x == 0) {
#ifdef TGSIM_FULL_FENCE
    __threadfence();
#else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}
__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ inline uint32_t mask_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Block-wide exclusive scan (every thread of the block calls it): a wave scan by shuffles, the
// four wave totals through red[0..3], two barriers (the second frees red for reuse).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* red, uint32_t& total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((int)lane >= o) x += y;
  }
  if (lane == 63) red[wave] = x;
  __syncthreads();
  uint32_t pre = 0;
  total = 0;
#pragma unroll
  for (uint32_t w = 0; w < kBlock / 64; ++w) {
    const uint32_t a = red[w];
    pre += w < wave ? a : 0u;
    total += a;
  }
  __syncthreads();
  return pre + x - v;
}

// A reservation of n staged slots behind the device-side count that never leaves the count above
// the capacity: an adder that overshoots pulls it back to cap after its add, so once every adder
// is done the count is <= cap, and every slot below it was reserved by exactly one adder (which
// writes it when p < cap and reports ERR_CAP_M otherwise). The shape pass reads this count.
__device__ __forceinline__ uint32_t reserve_staged(uint32_t* cnt, uint32_t n, uint32_t cap) {
  const uint32_t old = atomicAdd(cnt, n);
  if ((uint64_t)old + n > cap) atomicMin(cnt, cap);
  return old;
}

}  // namespace tgsim
