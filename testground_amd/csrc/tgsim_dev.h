// tgsim_dev.h — raw device view of one simulator context and the window pipeline entry points
// implemented in tgsim_kernels.hip. The host runtime (tgsim_runtime.hip) owns allocation, table
// uploads and the C ABI; everything here is plain pointers.
#pragma once
#include <vector>

#include "tgsim_internal.h"

namespace tgsim {

// Kernel classes timed with HIP events on the ctx stream when profiling is on (tgsim_profile_*).
enum KernelId : int {
  KID_SHAPE = 0, KID_EXTRACT, KID_TB, KID_EMIT, KID_RADIX_HIST, KID_RADIX_ROWS, KID_RADIX_SCATTER,
  KID_KEYS, KID_BOUNDS, KID_REGION_FILL, KID_GEN, KID_SIG, KID_LARGE, KID_BKT_HIST, KID_BKT_SCATTER,
  KID_BKT_SORT, KID_SEG_REST, KID_FLOOD_COUNT, KID_FLOOD_EMIT, KID_SHAPE_SEQ, KID_PROBE, KID_SEG_SMALL, KID_STORM,
  KID_EXCHANGE, KID_ALLREDUCE, KID_SHAPE_WIDE, KID_COPY, KID_COUNT
};
extern const char* const kKernelNames[KID_COUNT];

struct Prof {
  uint32_t mask = 0;  // bit per KernelId
  std::vector<hipEvent_t> pool;
  struct P { int kid; hipEvent_t a, b; };
  std::vector<P> pending;
  double ms[KID_COUNT] = {};
  unsigned long long n[KID_COUNT] = {};
};

// Flood workload state (config 5, tgsim_flood_*): the local rows of the graph, first-receipt bits
// [max_pubs][wpp] and per-item scratch of the reaction (count, first flag, exclusive offsets).
struct Flood {
  uint32_t* off = nullptr;        // [nloc+1] row offsets (local rows, rebased to 0)
  uint32_t* nbr = nullptr;        // neighbours (global ids)
  uint32_t* seen = nullptr;       // [max_pubs * wpp] bit (p, local instance)
  uint32_t D = 0, max_pubs = 0, wpp = 0;
  uint32_t* cnt = nullptr;        // [cap] forwards per delivery (0 unless first receipt)
  uint8_t* first = nullptr;       // [cap] first receipt of (pub, receiver)
  uint32_t* bsum = nullptr;       // [kFloodBlocks] forwards per chunk -> staged offset of the chunk
  uint32_t* mark = nullptr;       // [mark_cap] (local, pub) pairs of a publish batch
  size_t cap = 0, mark_cap = 0;
};

// A topic index for device subscriptions (tgsim_topics.hip): per topic k, runs
// [run_off[k], run_off[k+1]) in position order; run j holds positions pos0[j] .. pos0[j]+len[j]-1 at
// arena entries entry[j] ..; t = the arena's entry times.
struct TopicIndex {
  const uint32_t* run_off = nullptr;
  const uint32_t* pos0 = nullptr;
  const uint32_t* len = nullptr;
  const uint64_t* entry = nullptr;
  const int64_t* t = nullptr;
  uint32_t n_topics = 0;
};

// TCP mode (tgsim_tcp_*): write and segment tables, two lists of segments with a
// retransmission scheduled (the current one is released at the next window start, survivors move
// to the other), and counters.
constexpr int kTcpArriveBlocks = 2048;  // k_tcp_arrive's grid (= TcpDev::part entries)
// the segment word and chains, shared with the storm reactor's writes on connections
constexpr uint32_t kTcpSoleSeg = 0x80000000u;  // s_w: the segment is its write's only one
constexpr uint32_t kTcpWMask = 0x0FFFFFFFu;    // s_w: the write
constexpr uint32_t kTcpNoSeg = 0xFFFFFFFFu;    // end of a connection's segment chain
// k_tcp_conn_release modes: at a write (t0 = the write times), after a window (its ACKs first, t0 =
// the window's end), at a window start for the connections whose timer expired (loss episodes)
constexpr uint32_t kRelAtWrite = 0, kRelAfterWindow = 1, kRelLoss = 2;
constexpr uint32_t kTcpBatches = 1u << 14;  // acks mode: ring of attempt-0 timer batches (one per window)
// acks mode: the segments first sent in one window, [lo, hi), their timers in [t_lo, t_hi)
struct TcpBatch {
  uint32_t lo, hi;
  int64_t t_lo, t_hi;
  uint32_t done, pad;
};
struct TcpScalars {
  uint32_t pend_n[2];             // entries of the two pending lists (acks mode: retransmitted attempts' timers)
  uint32_t done;                  // writes finished by the running reaction
  uint32_t ack_n;                 // acks mode: ACKs of the last reaction (delivery indices in ack_idx)
  uint32_t ack_base;              // ... their first staged slot at the release
  uint32_t tb_tail;               // ... oldest live timer batch
  uint32_t plan_n, plan_total;    // ... batches due at this release and their segments
  uint32_t n_in;                  // the reaction's deliveries: the window's own (n_out) + the copies other
                                  // shards delivered for this shard's writers (sharded: k_tcp_rx)
  unsigned long long retx, delivered, failed, released;
};
struct TcpDev {
  uint32_t *w_src = nullptr, *w_dst = nullptr, *w_rem = nullptr, *w_state = nullptr;
  int64_t* w_tarr = nullptr;      // delivery time (the latest segment's arrival); INT64_MIN until delivered
  int64_t* w_tmax = nullptr;      // latest arrival so far of a multi-segment write (atomicMax)
  int64_t* w_fail = nullptr;      // earliest failure key t * 2 + (timeout ? 1 : 0) (atomicMin)
  uint32_t* s_w = nullptr;        // write (bits 0-27) | copies of the current attempt << 28 | kRetxBit (acks) | kSoleSeg
  uint32_t *s_wire = nullptr, *s_att = nullptr, *s_out = nullptr, *s_mark = nullptr;
  int64_t *s_tatt = nullptr, *s_arr = nullptr, *s_tlast = nullptr;
  // per-window decision bits: retransmissions over the packets (bm_s) and the deliveries (bm_r),
  // duplicated deliveries (bm_d); per-block partial counts of k_tcp_arrive
  uint64_t *bm_s = nullptr, *bm_r = nullptr, *bm_d = nullptr;
  uint32_t* part = nullptr;
  // acks mode (tgsim_tcp_config.acks): ACK bits over the deliveries (intact data), the reaction's ACK
  // list, a segment's settled byte (1 an ACK arrived, 2 gave up), the timer-batch ring and the
  // release's plan over it
  uint32_t acks = 0;
  uint64_t* bm_a = nullptr;
  uint32_t* ack_idx = nullptr;
  uint8_t* s_done = nullptr;
  TcpBatch* tb = nullptr;
  uint32_t *plan_lo = nullptr, *plan_off = nullptr;
  uint32_t* pend[2] = {nullptr, nullptr};
  uint32_t* pend_by = nullptr;    // [N] retransmissions pending (or released into the open window) per sender
  TcpScalars* sc = nullptr;
  // connections (tgsim_tcp_connect): Reno window and the queue of unsent segments
  // (a chain through s_next from c_head); w_conn / s_ack1 exist in acks mode
  uint32_t n_conn = 0;
  uint32_t *c_src = nullptr, *c_dst = nullptr, *c_cwnd = nullptr, *c_ssth = nullptr, *c_cnt = nullptr;
  uint32_t *c_flight = nullptr, *c_queued = nullptr, *c_head = nullptr, *c_acks = nullptr, *c_broken = nullptr;
  unsigned long long* c_acked = nullptr;  // cumulative first ACKs
  int64_t* c_tloss = nullptr;     // the window's earliest expired timer (INT64_MAX: none): a loss episode
  uint32_t* c_una = nullptr;      // no segment before it is outstanding (advanced after ACKs and at a loss episode)
  uint32_t* c_fack = nullptr;     // the window's first ACKs of segments in flight (not marked lost)
  int64_t* c_tack = nullptr;      // the window's latest first-ACK arrival (INT64_MIN: none)
  uint32_t* c_fr = nullptr;       // the segment last fast-retransmitted (kNoSeg: none)
  uint32_t* w_conn = nullptr;     // [W] the write's connection (kNoSeg: tgsim_tcp_send writes)
  uint32_t* s_next = nullptr;     // [S] the connection's next segment
  uint32_t* s_ack1 = nullptr;     // [S] first-ACK claim (a segment frees one flight slot once)
  uint8_t* s_lost = nullptr;      // [S] marked lost by a loss episode: resent under cwnd, no timer meanwhile
  uint8_t* s_tq = nullptr;        // [S] the segment has an entry on the timer lists (pend)
  uint32_t mss = 0, hdr = 0, max_att = 0;
  int64_t rto = 0;
  uint64_t cap_w = 0, cap_s = 0;
  // sharded: instances [lo, lo + nloc) of N on shard `shard` of S; segment ids on the
  // wire are the single run's (generated storm rounds of fanout F: tgsim_tcp.hip tcp_wire / tcp_local);
  // data copies delivered here for another shard's writers go there through the exchange blocks
  uint32_t S = 1, shard = 0, N = 0, lo = 0, nloc = 0, F = 0, xcap = 0;
  uint64_t inv = 0;               // shard_inv(N)
  uint32_t* xq = nullptr;
  tgsim_record *xsend = nullptr, *xrecv = nullptr;
};

// Sequential probes (tgsim_probe_*): per local prober its position in order,
// state, flags and times; outcome bytes [nloc][n_order]; per-reaction scalars.
struct ProbeScalars {
  int64_t next_end;               // the proposed end of the next window
  int64_t min_dl;                 // running min over waiting probers of their deadline (k_probe_step)
  uint32_t active;                // probers still waiting (k_probe_step -> snapshot n_active)
  uint32_t n_active;
  uint32_t done, n_ans;           // k_probe_step workgroups finished (the last one proposes the window end);
                                  // probers whose requests the local peers answer in this reaction (sharded)
  int64_t prop[3];                // this shard's proposal inputs: busy, waiting probers, earliest deadline
};
struct ProbeDev {
  uint32_t* order = nullptr;      // [n_order]
  uint32_t* pos = nullptr;        // [nloc] the current probe's position
  uint8_t* state = nullptr;       // [nloc] idle / waiting / done
  uint8_t* refused = nullptr;     // [nloc] the current request was refused by the prober's route
  uint8_t* replied = nullptr;     // [nloc] the peer has answered the current request (2: in this reaction,
                                  // its reply sent at t_rep)
  int64_t *t_req = nullptr, *t_rep = nullptr, *t_reparr = nullptr, *t_done = nullptr;  // [nloc]
  uint8_t* out = nullptr;         // [nloc * n_order] TGSIM_PROBE_*
  ProbeScalars* sc = nullptr;
  uint32_t n_order = 0, req_bytes = 0, rep_bytes = 0;
  int64_t timeout = 0, window = 0;
  // the answering side, per prober g [N] (the requests that peers on this shard received): the last
  // position answered + 1, the position answered in this reaction + 1 (the highest new one), its
  // first arrival of that position's request (only the highest position's), packed as
  // (position + 1) << 40 | (t_end - 1 - arrival) so one 64-bit atomicMax keeps both
  // (0 = none); the probers to answer (sharded: k_probe_answer)
  uint32_t *ans = nullptr, *cur = nullptr, *alist = nullptr;
  uint64_t* rqa = nullptr;
  // sharding (as StormDev): notices to a prober's shard go into the exchange blocks
  uint32_t lo = 0, nloc = 0, N = 0, S = 1, shard = 0, xcap = 0;
  uint32_t* xq = nullptr;
  tgsim_record *xsend = nullptr, *xrecv = nullptr;
  int64_t* prop_all = nullptr;
};

// Storm plan reactor (tgsim_storm_*): per connection h (instance * O + k) its dial
// and write state, per local instance its dial FIFO position, semaphore slots and writesem queue.
struct StormScalars {
  int64_t next_end;               // the proposed end of the next window
  int64_t min_dl;                 // running min of waiting dials' deadlines (k_storm_step)
  int64_t next_start;             // running min of the start times of admitted dials not yet due
  uint32_t active, n_active;      // connections dialling / writing (k_storm_step -> snapshot)
  uint32_t done, waiting;         // k_storm_step workgroups finished (the last proposes the window end);
                                  // dials holding a semaphore slot
  unsigned long long written, delivered, failed, bytes;  // chunks (cumulative)
  uint32_t n_ans, pad_ans;        // connections whose SYN the local listeners answer in this reaction
  int64_t prop[3];                // this shard's proposal inputs: busy, active connections, earliest deadline
                                  // + 1 / dial start (sharded: gathered, then reduced by k_storm_prop)
};
struct StormDev {
  uint32_t O = 0, C = 0, Hc = 0;  // connections per instance, semaphore width, holder capacity min(C, O)
  uint32_t nchunks = 0, chunk = 0, hdr = 0, syn = 0, win = 0;
  uint64_t data = 0;
  int64_t timeout = 0, window = 0;
  uint32_t n_conn = 0, phase = 0;  // phase 0: dials, 1: writes
  // TCP mode: connection h is TCP connection h; its SYN write and chunk writes have
  // ids reserved at setup - write W0 + h * (nchunks + 1) + j (j = 0 the SYN), segments from
  // S0 + h * spcon (the SYN's, then spc per full chunk)
  uint32_t tcp = 0, W0 = 0, S0 = 0, spcon = 0, spc = 0, mss = 0;
  uint32_t* settled = nullptr;    // [n_conn] chunk writes settled (delivered or failed), in order
  uint32_t* wsegs = nullptr;      // [n_conn] segments written (the SYN's included)
  // [n_conn]
  uint32_t* dst = nullptr;
  int64_t* t_ready = nullptr;
  uint8_t* state = nullptr;       // sleeping / waiting / done (dial) - kept through the write phase
  uint8_t* flags = nullptr;       // bit 0 refused, bit 1 the peer answered the SYN, bit 3 it did in this
                                  // reaction (the listener's notice: t_rep is the SYN-ACK's send time)
  uint8_t* res = nullptr;         // TGSIM_PROBE_* dial outcome
  uint32_t* slot = nullptr;       // the dial semaphore slot a waiting dial holds
  int64_t *t_start = nullptr, *t_synarr = nullptr, *t_ackarr = nullptr, *t_done = nullptr, *t_rep = nullptr;
  uint32_t* emit = nullptr;       // this reaction's staging per connection (dial: bits; writes: chunks)
  uint32_t* rem = nullptr;        // chunks not yet written
  uint32_t* infl = nullptr;       // chunks in the send buffer (neither arrived nor failed)
  uint32_t* order = nullptr;      // per instance its connections k in dial FIFO order (t_ready, k)
  uint32_t* ring = nullptr;       // per instance the writesem FIFO (O entries, a ring)
  uint32_t* claim = nullptr;      // bit per chunk (h * nchunks + j): first arrival seen (dialer's shard)
  // the listener's side of connection h (on dst[h]'s shard): t_synarr = the SYN's first arrival;
  // ans[h] 0 / 2 (first arrival in this reaction, listed in alist) / 1 (answered)
  uint32_t* ans = nullptr;
  uint32_t* alist = nullptr;
  // sharding: local instances [lo, lo + nloc) of N on shard `shard` of S; notices to a
  // dialer's shard go into the exchange blocks (cursor of peer p at xq[p << 5])
  uint32_t lo = 0, N = 0, S = 1, shard = 0, xcap = 0;
  uint32_t* xq = nullptr;
  tgsim_record *xsend = nullptr, *xrecv = nullptr;
  int64_t* prop_all = nullptr;    // [S * 3] the shards' proposal inputs (all-gathered)
  // [nloc]
  uint32_t *dq = nullptr, *qh = nullptr, *ql = nullptr, *nh = nullptr;
  int64_t* slot_t = nullptr;      // [nloc * C] time each semaphore slot fell free (kBusy: held)
  uint32_t* hold = nullptr;       // [nloc * Hc] goroutines holding writesem, blocked in conn.Write
  uint8_t* failed = nullptr;      // an instance's chunk failed
  int64_t* t_last = nullptr;      // its last conn.Write return
  StormScalars* sc = nullptr;
};

struct Dev {
  Prof prof;
  Flood fl;
  ProbeDev pr;
  StormDev sm;
  hipStream_t stream = nullptr;
  uint32_t N = 0, S = 1, shard = 0, lo = 0, nloc = 0;
  uint32_t data_net = 0, data_mask = 0, data_len = 0;
  uint32_t key0 = 0, key1 = 0;
  int64_t slot_ns = 1000000;
  uint32_t slots = 1024;
  uint32_t cap_msgs = 0, cap_rec = 0;
  uint32_t subcap = 0;            // per sub-queue capacity of the A/D/L batches (kNSub sub-queues)
  uint64_t cap_arena = 0;
  uint32_t xcap = 0;
  DevScalars* sc = nullptr;       // device
  DevScalars* h_sc = nullptr;     // pinned host mirror (read at sync points)

  // tables
  ShapeDev* shape = nullptr;
  TbShape* tbs = nullptr;  // [nloc] the token bucket's fields of shape (uploaded with it)
  uint32_t* zd = nullptr;  // [nloc / 32 + 1] zero-delay unshaped senders (Heavy::zd, uploaded with shape)
  int64_t* X = nullptr;
  // [N] ip | flags << 32 per instance (flags bit0 link enabled, bit1 external routing allowed): one
  // 8-B gather gives a destination's address and link state
  uint64_t* ipf = nullptr;
  uint32_t* en_bits = nullptr;    // [N / 32 + 1] link enabled (flags bit 0), the destination test
  uint32_t* rule_off = nullptr;   // [nloc+1]
  RuleDev* rules = nullptr;

  // netem correlations: per local sender (dup, corrupt, reorder, -) rho and crandom state
  uint32_t* cor_rho = nullptr;    // [4 * nloc]
  uint32_t* cor_last = nullptr;   // [4 * nloc]
  uint32_t* corr_idx = nullptr;   // [kDeferSub][defer_seg_cap(cap_msgs)] deferred message indices (k_shape)
  uint32_t* corr_sorted = nullptr;  // [cap_msgs] the same, grouped by sender in (t_send, seq) order
  bool any_corr = false;          // some local shape has kShCorr
  // some local sender has ever been bandwidth-limited (kShLimited): only then can a copy reach the
  // token-bucket batch A (copies of an unlimited sender carry TGSIM_F_STAGE_D from the netem pass,
  // wheel included), so the window skips the A partition, k_tb_bucket and k_rest<TB> until then
  bool ever_limited = false;
  // single-shard contexts: this window's k_rest<TB> rides in the window end's first launch
  // (k_rest_local_hist) instead of a launch of its own
  bool tb_rest_owed = false;
  uint32_t* moff = nullptr;       // [segK] per local sender: its deferred messages in corr_sorted

  // netem queue limit: pend[l] = local sender l's records in the timing wheel
  // (maintained by k_wheel_scatter +, k_tb_bucket / k_emit_bucket / k_recv -); heavy = this window's
  // test (heavy.pend == nullptr: the host proved no sender can reach the limit); H = due wheel
  // records of heavy senders (copies, grouped by sender for k_shape_seq)
  uint32_t* pend = nullptr;        // [nloc << pend_shift(nloc)]: use pend_ref
  uint32_t* pend_part = nullptr;   // [kRadixBlocks] k_pend_max's per-block maxima
  // the window's wheel insert on a side stream (contexts with a flood graph): side_ev marks its end,
  // main_ev the point of the context stream it starts from; side_pending until the context stream
  // has been made to wait for it (join_side)
  hipStream_t side = nullptr;
  hipEvent_t side_ev = nullptr, main_ev = nullptr;
  bool side_pending = false;
  Heavy heavy{};
  tgsim_record* H = nullptr;
  uint32_t *hkeys = nullptr, *hvals = nullptr;
  uint32_t h_cap = 0;
  // the H list's own group-by (it shares its launches with the deferred messages' one): output
  // (hkeys1, hvals1), per-sender offsets hoff [nloc + 1], partition tables as hist / histx / tot / bstart
  uint32_t *hkeys1 = nullptr, *hvals1 = nullptr, *hoff = nullptr;
  uint32_t *hhist = nullptr, *hhistx = nullptr, *htot = nullptr, *hbstart = nullptr;
  uint8_t* seq_done = nullptr;     // [nloc] k_shape_seq_wide decided the sender's deferred messages

  // staged messages (SoA) + per-message status
  uint32_t *m_src = nullptr, *m_dst = nullptr, *m_seq = nullptr, *m_size = nullptr;
  int64_t* m_t = nullptr;
  uint8_t* status = nullptr;

  // record batches and the wheel
  tgsim_record *A = nullptr, *D = nullptr, *L = nullptr, *arena = nullptr;
  uint32_t *KA = nullptr, *KD = nullptr, *KL = nullptr;  // group-by keys written by the producers
  tgsim_record *xsend = nullptr, *xrecv = nullptr;
  RegionDev* regions = nullptr;
  uint32_t* dirs = nullptr;
  uint32_t* plan_start = nullptr;
  uint32_t* plan_off = nullptr;

  // sort scratch
  uint32_t *keys0 = nullptr, *keys1 = nullptr, *vals0 = nullptr, *vals1 = nullptr;
  uint32_t* hist = nullptr;       // [kRadixBlocks * kMaxBins] per-partition-block histogram rows
  uint32_t* histx = nullptr;      // [kMaxBins * kRadixBlocks] per bin the blocks' exclusive offsets
  uint2* kv1 = nullptr;           // k_bkt_local output: (key, physical index) per item
  uint32_t* poff = nullptr;       // [kRadixBlocks * (kMaxBins + 1)] per-block bucket offsets (k_bkt_local)
  uint32_t* keys2 = nullptr;      // oversized fused buckets: contiguous copy for the global path
  uint32_t* vals2 = nullptr;
  uint32_t* tot = nullptr;        // [kMaxBins]
  int n_cu = 256;                 // compute units of the device (bucket widths)
#ifndef TG_BKT_LOAD
#define TG_BKT_LOAD 1u
#endif
  uint32_t bkt_load = TG_BKT_LOAD;  // copies per key relative to one packet per message (TCP acks: 2)
  int grid_shape = 2048;          // k_shape / k_gen_storm grids (init_launch_geometry)
  int grid_gen = 2048;
  uint32_t* bstart = nullptr;     // [kMaxBins + 1] bucket starts of the last partition pass
  uint32_t* qc = nullptr;         // [kQcLines][32] append counters (128 B apart): A / D / L, exchange
  uint32_t* seg_off = nullptr;    // [max(nloc, slots, max_states) + 1]
  LargeSeg* large = nullptr;
  uint32_t* medium = nullptr;     // [segK] ids of segments kThreadSeg < len <= kTile
  uint32_t* chunk_off = nullptr;
  uint64_t *K1a = nullptr, *K1b = nullptr, *K2a = nullptr, *K2b = nullptr;
  uint32_t *K3a = nullptr, *K3b = nullptr;

  // outputs of the last window
  int64_t* o_t = nullptr;
  uint32_t *o_src = nullptr, *o_dst = nullptr, *o_seq = nullptr, *o_size = nullptr,
           *o_flags = nullptr, *o_coff = nullptr;
  uint32_t* inbox = nullptr;      // [nloc+1]

  // sync service
  uint32_t max_states = 0, max_waiters = 0;
  uint64_t max_signals = 0;
  uint32_t *s_state = nullptr, *s_inst = nullptr, *s_seq = nullptr;  // batch (device)
  int64_t* s_t = nullptr;
  uint32_t s_cap = 0;
  uint32_t* st_count = nullptr;
  int64_t* st_last = nullptr;
  uint32_t* st_nchunks = nullptr;
  SigChunk* st_chunks = nullptr;
  int64_t* sig_log = nullptr;
  uint32_t* w_state = nullptr;
  uint32_t* w_target = nullptr;
  int64_t* w_twait = nullptr;
  int64_t* w_release = nullptr;
  int64_t* sig_part = nullptr;    // [2 * 4096] per-block (min, max) of a signal batch
  int64_t* sig_red = nullptr;     // [4] count-only batch: last tmin, running tmin, running tmax, last tmax
  unsigned long long* stats = nullptr;  // [kNSub][16] sharded k_shape counters (ST_MSGS..ST_LOCAL)
};

// Times the launches issued while it is alive with a HIP event pair on d.stream (if enabled).
struct ProfScope {
  Dev& d;
  int kid;
  hipEvent_t a = nullptr;
  hipStream_t st;
  ProfScope(Dev& dd, int k, hipStream_t s = nullptr) : d(dd), kid(k), st(s ? s : dd.stream) {
    if (!(d.prof.mask & (1u << kid))) return;
    a = take();
    (void)hipEventRecord(a, st);
  }
  ~ProfScope() {
    if (!a) return;
    hipEvent_t b = take();
    (void)hipEventRecord(b, st);
    d.prof.pending.push_back({kid, a, b});
  }
  hipEvent_t take() {
    if (!d.prof.pool.empty()) {
      hipEvent_t e = d.prof.pool.back();
      d.prof.pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    return e;
  }
};

// Every function returns hipSuccess or the first HIP error; device-side capacity/ordering problems
// are reported through DevScalars::err and surfaced by the host at the next sync.
// Window start: the new window begins at the previous window's end (read on the device); its end is
// explicit, a barrier waiter's release + offset, or a device value + offset.
hipError_t launch_set_window(Dev& d, int64_t t_end);
hipError_t launch_set_window_barrier(Dev& d, uint32_t waiter, int64_t offset_ns);
hipError_t launch_set_window_dev(Dev& d, const int64_t* t_end_dev, int64_t offset_ns);
// The storm's deferred count-only commit (+ the barrier registered after it) fused with the window
// start that waits on waiter `waiter` (launch_sig_commit's arguments).
hipError_t launch_set_window_barrier_commit(Dev& d, uint32_t waiter, int64_t offset_ns, uint32_t nparts, uint32_t n,
                                            uint32_t st, uint32_t nw, bool add, uint32_t add_state,
                                            uint32_t add_target, int64_t add_twait);
hipError_t launch_reset_tb(Dev& d, const uint32_t* locals_dev, uint32_t n);
// sc->pend_max = max over local senders of their queued copies (the host's exact occupancy bound)
// retx: TCP pending per sender; inbox_mult: acks mode, packets per delivery of the sender's last inbox
// per-block maxima into d.pend_part, then copied to host[kRadixBlocks] (pinned) on the stream
hipError_t join_side(Dev& d);
inline PendRef pend_ref(const Dev& d) { return PendRef{d.pend, pend_shift(d.nloc)}; }
hipError_t launch_pend_max(Dev& d, const uint32_t* retx, uint32_t inbox_mult, uint32_t mult, uint32_t* host);
// sharded storm batch: generator partials -> red2 = {last, -first} (for a MAX all-reduce) -> the
// batch's single partial in sig_part
hipError_t launch_storm_red(Dev& d, uint32_t nparts, int64_t* red2);
hipError_t launch_storm_unpack(Dev& d, const int64_t* red2);
// init_crandom on a Shape call: the state of local sender pairs[2i] re-seeded for epoch pairs[2i+1]
hipError_t launch_reset_corr(Dev& d, const uint32_t* pairs_dev, uint32_t n);
// wheel extract, shape, token bucket, pack; n_dev non-null: the staged count is read on the device
hipError_t window_begin(Dev& d, uint32_t n_staged, const uint32_t* n_dev = nullptr);
hipError_t window_end(Dev& d);                       // receive, deliveries, wheel insert
// window_end with the storm round `round` (fanout 8, t0 = this window's end, staged at 0, spread,
// size) generated inside the wheel-insert launch; *nparts = its signal partials
hipError_t window_end_storm(Dev& d, uint32_t round, uint32_t size, int64_t spread_ns, uint32_t* nparts);
hipError_t sync_scalars(Dev& d);                     // copy DevScalars to d.h_sc (blocking)
// Signal batch already in d.s_state/s_inst/s_t. States lie in [kmin, kmax]. count_only: the
// batch has one state and no sequence numbers are materialised.
hipError_t signal_batch(Dev& d, uint32_t n, uint32_t kmin, uint32_t kmax, uint64_t log_base, uint32_t n_waiters,
                        bool count_only);
hipError_t add_waiter(Dev& d, uint32_t idx, uint32_t state, uint32_t target, int64_t t_wait);
hipError_t resolve_waiters(Dev& d, uint32_t n_waiters);
void init_launch_geometry(Dev& d);
hipError_t launch_gen_storm(Dev& d, uint32_t staged_base, uint32_t round, int64_t t0, uint32_t fanout,
                            uint32_t size, int64_t spread_ns, uint32_t* nparts);
// Finish a count-only batch from its per-block partials: (tmin, tmax) -> sig_red[0], [3]; with
// commit, count it into state st and resolve waiters [0, n_waiters); add: register waiter
// n_waiters (state, target, t_wait) in the same launch and resolve it.
hipError_t launch_sig_commit(Dev& d, uint32_t nparts, bool commit, uint32_t n, uint32_t st, uint32_t n_waiters,
                             bool add, uint32_t add_state, uint32_t add_target, int64_t add_twait);

// Flood reaction over the last window's deliveries (sc->n_out of them, inbox order), with no host
// read: count pass (first receipt of (pub, receiver) against the seen bits and the receiver's
// earlier deliveries) over kFloodBlocks chunks, a one-block scan of the chunk totals, then the
// forwards of every first receipt (seen bit set, t_send = max(t_deliver, horizon), seq = pub * D +
// neighbour slot) staged after the staged messages: at base_host, or at sc->n_msgs_dev when
// base_dev; sc->n_msgs_dev = the new staged count.
hipError_t launch_flood_react(Dev& d, bool base_dev, uint32_t base_host, uint32_t size, int64_t horizon);
// Staging behind a device-side count: n messages (SoA at the given device pointers) appended at
// sc->n_msgs_dev, which then grows by n.
hipError_t launch_append(Dev& d, const uint32_t* src, const uint32_t* dst, const uint32_t* seq, const uint32_t* size,
                         const int64_t* t, uint32_t n);
// The same copy at a host-known staged offset `base` (tgsim_enqueue_device): one launch, five arrays.
hipError_t launch_stage(Dev& d, const uint32_t* src, const uint32_t* dst, const uint32_t* seq, const uint32_t* size,
                        const int64_t* t, uint32_t n, uint32_t base);
// A publish batch: set the seen bits of (local, pub) pairs already in d.fl.mark.
hipError_t launch_flood_mark(Dev& d, uint32_t n);
// TCP mode: the last window's packets (status, seq; count n_host or *n_dev) and deliveries ->
// queued copies, first intact arrivals, finished writes, retransmissions onto pend[cur]
hipError_t launch_tcp_react(Dev& d, TcpDev& t, uint32_t cur, uint32_t n_host, const uint32_t* n_dev, uint32_t epoch,
                            uint32_t fill);  // fill: acks mode, the batch registered for this window (or ~0u)
// window start: pend[cur] entries due before the window's end staged behind sc->n_msgs_dev (which
// the caller has set), the others moved to pend[cur ^ 1]
hipError_t launch_tcp_release(Dev& d, TcpDev& t, uint32_t cur, bool base_dev, uint32_t base_host);
// acks mode, at the window start: the last reaction's ACKs staged, due timers fired (attempt-0 batches
// [tail, head) and the retransmitted attempts on pend[cur]), survivors to pend[cur ^ 1]; batch `head`
// registered for the segments [lo, hi) this window sends (reg)
hipError_t launch_tcp_release_acks(Dev& d, TcpDev& t, uint32_t cur, bool base_dev, uint32_t base_host, uint32_t head,
                                   bool reg, uint32_t lo, uint32_t hi);
// TCP mode: the staged storm round [base, base + n) adopted as writes wbase.. / segments sbase..
hipError_t launch_tcp_adopt(Dev& d, TcpDev& t, uint32_t base, uint32_t n, uint32_t wbase, uint32_t sbase);
// sharded: the window's data copies for other shards' writers into the exchange blocks (+ headers)
hipError_t launch_tcp_fwd(Dev& d, TcpDev& t);
// connections: new segments linked to their queues (links: n quads conn, old tail, first, count),
// then every connection sends what its window has room for, at max(written, t0) (t0 = INT64_MIN:
// at the write times; after_window: first apply the window's ACKs and resets, t0 = the window's
// end), staged behind sc->n_msgs_dev (set from base_host unless base_dev), timers on pend[cur]
hipError_t launch_tcp_link(Dev& d, TcpDev& t, const uint32_t* links, uint32_t n);
hipError_t launch_tcp_conn_release(Dev& d, TcpDev& t, uint32_t mode, uint32_t cur, bool base_dev,
                                   uint32_t base_host);
constexpr uint32_t kFloodBlocks = 4096;  // chunks of the flood reaction (>= 16 waves per CU)

// Sequential probes: every local prober without a probe sends its first at t0 (device staging
// behind sc->n_msgs_dev, set from base_host unless base_dev).
hipError_t launch_probe_start(Dev& d, bool base_dev, uint32_t base_host, int64_t t0);
// After a window: the window's refused requests (status over the staged packets, n_host or
// *n_dev), first arrivals of requests and replies (deliveries), then per prober the reply it owes,
// the end of its probe and the next request (staged behind sc->n_msgs_dev), and the next window's
// proposed end (ProbeScalars::next_end)
// sharded (S > 1), around the runtime's notice exchange and proposal all-gather
hipError_t launch_probe_react_pre(Dev& d, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                                  const uint32_t* n_status_dev);
hipError_t launch_probe_react_post(Dev& d);
hipError_t launch_probe_prop(Dev& d);
hipError_t launch_probe_react(Dev& d, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                              const uint32_t* n_status_dev);

// Storm plan reactor. start: the first dials (frame H = t_end = t_now); react: the window's statuses
// and deliveries, then per instance its dials / writes (staged behind sc->n_msgs_dev, set from
// base_host unless base_dev) and the next window's proposed end (StormScalars::next_end).
hipError_t launch_storm_start(Dev& d, const TcpDev& td, bool base_dev, uint32_t base_host, int64_t t_now);
// Message mode, in three parts around the collectives of a sharded run: _pre (packets, deliveries, the
// listeners' answers, notices into the exchange blocks), the notice exchange (runtime, S > 1), _post
// (notices applied, the step); then, S > 1, the proposal all-gather (runtime) and launch_storm_prop.
hipError_t launch_storm_react_pre(Dev& d, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                                  const uint32_t* n_status_dev);
hipError_t launch_storm_react_post(Dev& d, const TcpDev& td);
hipError_t launch_storm_prop(Dev& d);
hipError_t launch_storm_react(Dev& d, const TcpDev& td, bool base_dev, uint32_t base_host, uint32_t n_status_host,
                              const uint32_t* n_status_dev);
// the write phase: every connection queued on its instance's writesem, first round at t0
hipError_t launch_storm_write_start(Dev& d, const TcpDev& td, bool base_dev, uint32_t base_host, int64_t t0);
// TCP mode: the reserved writes' and segments' static fields (sources, sizes, chains inside a write)
hipError_t launch_storm_tcp_init(Dev& d, const TcpDev& td);

// Batched Subscribe (tgsim_sync_subscribe_device): per-subscriber counts into cnt[0..n] (u64 scratch),
// exclusive scan into offsets[0..n], then (entries != nullptr) the entry ids, at most entries_cap.
hipError_t launch_subscribe(Dev& d, const TopicIndex& ti, uint32_t n, const uint32_t* topics, const uint32_t* from,
                            const int64_t* until, uint32_t cap_each, uint64_t* cnt, void* scan_tmp, size_t scan_bytes,
                            uint64_t* offsets, uint32_t* entries, uint64_t entries_cap);
size_t subscribe_scan_bytes(uint32_t n);

// Wave-collective: a reactor's notice to shard p's exchange block (one reservation per wave and
// peer on the peer's cursor xq[p << 5]); p == kNoPeer: none. The record carries t = v, src = a,
// dst = b, seq = kind. Overflow sets ERR_CAP_X (ECAPACITY at the next check).
constexpr uint32_t kNoPeer = 0xFFFFFFFFu;
__device__ __forceinline__ void notice_push(uint32_t* xq, tgsim_record* xsend, uint32_t xcap, DevScalars* sc,
                                            uint32_t p, uint32_t a, uint32_t b, uint32_t kind, int64_t v) {
  bool pending = p != kNoPeer;
  for (;;) {
    const uint64_t m = __ballot(pending);
    if (m == 0) break;
    const int leader = __ffsll((unsigned long long)m) - 1;
    const uint32_t lp = __shfl(p, leader);
    const bool mine = pending && p == lp;
    const uint64_t mm = __ballot(mine);
    uint32_t base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(xq + (lp << 5), (uint32_t)__popcll(mm));
    base = __shfl(base, leader);
    if (mine) {
      const uint32_t pos = base + mask_rank(mm);
      if (pos < xcap - 1) {
        tgsim_record* r = xsend + (size_t)p * xcap + 1 + pos;
        r->t = v; r->src = a; r->dst = b; r->seq = kind; r->size = 0; r->meta = 0; r->corrupt_off = 0;
      } else {
        atomicOr(&sc->err, ERR_CAP_X);
      }
      pending = false;
    }
  }
}

}  // namespace tgsim
