// tgsim_runtime.hip — host runtime of libtgsim.so: context, table compilation (LinkShape -> netem/HTB
// state, LinkRule -> per-sender LPM tables), uploads, and the C ABI declared in include/tgsim.h.
//
// The table compilation restates the reference's configuration path:
//   pkg/sidecar/link.go:143-217 (toMicroseconds, Shape, AddRules), pkg/sidecar/route.go:102-117
//   (routing policy), pkg/sidecar/docker_network.go:51-148 (apply order), plus the recalled
//   vishvananda/netlink v1.1.0 and Linux sch_htb/sch_netem conversions marked [EXT] in DESIGN.md.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <exception>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include <rccl/rccl.h>

#include "tgsim_dev.h"

using namespace tgsim;

#define TGSIM_VERSION_STRING "tgsim-mi355x 0.1.0 (gfx950)"

struct tgsim_ctx {
  tgsim_config cfg{};
  Dev d;
  std::string err;
  bool own_stream = false;
  uint32_t N = 0, S = 1, shard = 0, lo = 0, hi = 0, nloc = 0;
  uint32_t data_net = 0, data_mask = 0, data_len = 0;
  std::vector<ShapeDev> shape_h;
  std::vector<TbShape> tbs_h;       // source of the last d.tbs upload (kept alive for the async copy)
  std::vector<uint32_t> zd_h;       // source of the last d.zd upload
  bool all_zd = false;              // every local sender is zero-delay and unshaped (Heavy::zd)
  std::vector<uint8_t> flags_h;
  std::vector<uint32_t> ip_h;
  uint64_t space = 0;               // addresses in the data subnet
  // ip - data_net -> instance for addresses that are not their owner's initial one (data_net + 2 + id):
  // the reverse map stays O(moved instances), whatever the prefix length
  std::unordered_map<uint32_t, uint32_t> moved;
  std::vector<std::vector<RuleDev>> rules_h;
  std::vector<uint32_t> tb_reset;
  std::vector<uint32_t> rho_h;       // [4 * nloc] netem correlations per local sender
  std::vector<uint32_t> corr_epoch;  // [nloc] Shape calls so far
  std::vector<uint32_t> corr_reset;  // (local, epoch) pairs to re-seed at the next upload
  uint32_t* corr_reset_dev = nullptr;
  uint32_t corr_reset_cap = 0;
  bool shape_dirty = true, flags_dirty = true, ip_dirty = true, rules_dirty = true;
  size_t rules_cap_dev = 0;
  uint32_t* tb_reset_dev = nullptr;
  uint32_t tb_reset_cap = 0;
  int64_t now = 0;
  int64_t horizon = 0;   // start of the last completed window: earliest admissible t_send
  uint32_t n_staged = 0, n_status_last = 0;
  // tgsim_enqueue_device's batch when it was the first staging of the window: it occupies [0, n) of
  // the staged messages and is read in place by the window when nothing else was staged after it
  // (else copied in front at the window start: begin_common). VERDICT r5 item 6: config 2 copied 48 MB
  // of caller-resident messages into the staged arrays every round.
  struct ExtBatch {
    const uint32_t *src = nullptr, *dst = nullptr, *seq = nullptr, *size = nullptr;
    const int64_t* t = nullptr;
    uint32_t n = 0;
  } ext;
  bool in_window = false;
  bool now_from_device = false;
  bool end_known = false;             // the open window's end was given by the host (explicit t_end)
  int64_t end_h = 0;
  uint64_t sig_log_used = 0;
  uint32_t n_waiters = 0;
  // a storm batch whose count-only commit is deferred to the next sync-service call (a barrier
  // rides in the same launch): partials in d.sig_part
  bool storm_pending = false;
  uint32_t storm_parts = 0, storm_state = 0;
  uint32_t storm_n = 0;  // signals in the pending batch (the shard's instances, or all with a transport)
  // ... and a barrier registered after it, not yet launched (waiter storm_nw; the window start that
  // waits on it carries the commit too)
  bool storm_add = false;
  uint32_t storm_nw = 0, add_state = 0, add_target = 0;
  int64_t add_twait = 0;
  std::vector<void*> allocs;
  // speculative storm generation: after a storm round staged at the device clock, the
  // window's last launch also generates the next round (round + 1, state + 1, same shape); the
  // next tgsim_gen_storm_round that asks for exactly it only does the host bookkeeping. Any call that
  // writes the staged arrays or the signal partials first drops it.
  struct StormSpec { bool hint = false, valid = false; uint32_t round = 0, size = 0, state = 0, parts = 0; int64_t spread = 0; };
  StormSpec spec;
  // netem queue limit: the host's proof that no sender can reach the limit in a
  // window (then the kernels skip the test). pend_bound >= every local sender's queued copies at the
  // next window start: the exact maximum when last refreshed (k_pend_max, only when the bound is
  // inconclusive), plus what one window can add (mult * its per-sender message bound) for each since.
  uint64_t pend_bound = 0;
  bool pend_exact = true;
  std::vector<uint32_t> hcnt;        // host-staged messages per local sender this window
  std::vector<uint32_t> hcnt_touched;
  uint32_t win_m_host = 0;           // max of hcnt
  uint64_t win_m_extra = 0;          // device-staged messages (storm fanout, enqueue_device n): any sender
  uint32_t win_m_inbox = 0;          // flood forwards staged: (D - 1) per delivery of the sender's last inbox
  uint64_t win_inbox_max = 0;        // a bound on any sender's last inbox run (probes: N; floods use fl_npubs)
  // flood: a sender forwards each publication once (first receipt), so (D - 1) * (publications so
  // far) bounds its forwards in any window without reading the device
  uint32_t fl_npubs = 0;
  std::vector<uint8_t> fl_pub_seen;
  // A lifetime bound on any sender's queued + staged copies while the flood is the only reactor: every
  // message it ever staged from the host (life_host: the per-window maxima summed) plus at most D per
  // publication (a node publishes or forwards a publication once), times the largest duplication
  // multiplier seen. While that stays within the queue limit no window needs the exact refresh (a
  // host sync every few windows of config 5). life_ok clears for good when probes, a storm reactor
  // or TCP mode stage traffic the bound does not count.
  uint64_t life_host = 0;
  uint64_t life_mult = 1;
  bool life_ok = true;
  uint32_t* pend_host = nullptr;     // [kRadixBlocks] pinned: k_pend_max's per-block maxima
  // device-counted staging: after an asynchronous flood reaction the staged count is
  // sc->n_msgs_dev; host / device enqueues then append behind it on the device
  bool staged_dev = false;
  uint8_t* app = nullptr;  // [app_cap * 24] t | src | dst | seq | size, the pinned layout (one copy)
  size_t app_cap = 0;
  // pinned staging of host uploads (messages, publish marks): the copies are asynchronous, a buffer
  // is reused once its event has passed
  struct Pinned { uint8_t* p = nullptr; size_t cap = 0; hipEvent_t ev = nullptr; bool busy = false; };
  Pinned pin_msgs, pin_marks, pin_tcp;
  // TCP mode (tgsim_tcp_*)
  bool tcp_on = false, tcp_need_react = false;
  tgsim_tcp_config tcp{};
  TcpDev td;
  uint64_t tw_n = 0, tsg_n = 0;       // writes / segments so far
  uint32_t tcp_cur = 0, tcp_epoch = 0;
  // acks mode: timer batches registered (one per window with new segments), the first segment not
  // yet in one, and the batch the open window registered (its timer range is filled at the reaction)
  uint32_t tcp_nb = 0, tcp_fill = ~0u;
  uint64_t tcp_seg_batched = 0;
  // connections: host copies of their ends and queue tails; link scratch
  std::vector<uint32_t> conn_src, conn_dst, conn_tail;
  uint32_t conn_cap = 0;
  uint32_t* link_dev = nullptr;
  size_t link_cap = 0;
  // the reactions' counters land in two pinned snapshots (read once their event has completed);
  // nothing on the window path reads them (the queue-limit bound folds the pending retransmissions
  // into the occupancy: tgsim_tcp.hip)
  TcpScalars* tcp_snap = nullptr;
  hipEvent_t tcp_ev[2] = {nullptr, nullptr};
  uint32_t tcp_snap_cur[2] = {0, 0};
  bool tcp_snap_live[2] = {false, false};
  uint32_t tcp_snap_slot = 0;         // the next snapshot's slot (the other one holds the latest)
  tgsim_tcp_stats tstats{};
  bool any_dup = false;
  // cross-shard transport: the exchange, the storm batch's MAX all-reduce and the
  // signal all-gather run inside the library - natively over RCCL (comm), or through caller callbacks
  bool has_tr = false, tr_aborted = false;
  tgsim_transport tr{};
  ncclComm_t comm = nullptr;
  int64_t* d_red2 = nullptr;   // [2] storm batch: {last time, -first time} for the MAX all-reduce
  uint64_t* d_gather = nullptr;  // all-gather scratch (signal batch sizes and records)
  size_t gather_cap = 0;          // in uint64 units
  bool replicated_batch = false;  // publish: topic batches are replicated, never gathered
  int64_t max_tsend_h = INT64_MIN;   // latest host-staged send time (checked against t_end before launch)
  // topics (tgsim_sync_publish / _subscribe): entries live in device arenas, sorted by (topic,
  // position) per batch; the host keeps each topic's runs of consecutive positions
  // latest time of the host-submitted signals per state: a batch that goes back in time is
  // refused before anything changes (the device check stays for device-generated storm batches)
  std::vector<int64_t> st_last_h;
  struct TopicRun { uint32_t pos0, len; uint64_t entry; };
  std::vector<std::vector<TopicRun>> topic_runs;
  uint32_t* tp_inst = nullptr;
  int64_t* tp_t = nullptr;
  uint64_t* tp_off = nullptr;
  uint32_t* tp_len = nullptr;
  uint8_t* tp_bytes = nullptr;
  uint64_t tp_n = 0, tp_cap = 0, tp_nbytes = 0, tp_bytes_cap = 0;
  // device topic index for tgsim_sync_subscribe_device (CSR of topic_runs; rebuilt after a publish)
  bool tp_index_dirty = true;
  uint32_t *ti_off = nullptr, *ti_pos0 = nullptr, *ti_len = nullptr;
  uint64_t* ti_entry = nullptr;
  size_t ti_cap = 0;
  uint64_t* sub_cnt = nullptr;   // [sub_cap + 1] per-subscriber counts (scan input)
  void* sub_scan = nullptr;
  size_t sub_cap = 0, sub_scan_bytes = 0;
  // flood workload (tgsim_flood_*): host copy of the local rows (publish builds its messages here)
  std::vector<uint32_t> fl_off, fl_nbr;
  // fingerprints of the flood graph (rows, max_pubs) and of the probe setup (order, configuration):
  // a snapshot taken with either restores only into a context set up the same way
  uint64_t fl_hash = 0, probe_hash = 0, storm_hash = 0, tcp_hash = 0;
  uint32_t snap_staged = 0;  // the staged messages a snapshot image holds (sizes snap_regions)
  uint32_t snap_acks = 0;    // TCP acks mode: the last reaction's ACKs (ack_idx entries) it holds
  uint32_t fail_alloc = 0;  // tgsim_debug_fail_alloc: the n-th allocation point throws std::bad_alloc
  bool probes = false;      // tgsim_probe_setup done
  // a window ended with probes set up: tgsim_probe_react must run before anything stages messages or
  // opens the next window (it reads the window's staged rows and deliveries)
  bool probe_need_react = false;
  bool storm_on = false;    // tgsim_storm_setup done, not ended
  // a TCP storm's connections [lo, hi): host writes are refused on them, also after tgsim_storm_end
  // (their queues end at the last chunk the reactor linked, which the host does not track)
  uint64_t storm_conn_lo = 0, storm_conn_hi = 0;
  bool storm_need_react = false;
};

// Calls that stage messages or open a window refuse while a reaction is owed for the last one.
static int fail(tgsim_ctx* c, int code, const char* fmt, ...);
static int react_owed(tgsim_ctx* c) {
  if (c->probe_need_react) return fail(c, TGSIM_ESTATE, "probes: tgsim_probe_react after every window");
  if (c->storm_need_react) return fail(c, TGSIM_ESTATE, "storm: tgsim_storm_react after every window");
  return 0;
}

// FNV-1a over bytes, for the setup fingerprints the snapshot header carries
static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
  return h;
}

// An allocation point of a host-side table (tgsim_debug_fail_alloc makes the chosen one throw, so
// the tests can drive the ABI's bad_alloc path without exhausting memory).
static void alloc_point(tgsim_ctx* c) {
  if (c && c->fail_alloc && --c->fail_alloc == 0) throw std::bad_alloc();
}

// Commit a deferred storm batch before anything reads or reuses the sync state.
static hipError_t flush_storm(tgsim_ctx* c) {
  if (!c->storm_pending) return hipSuccess;
  c->storm_pending = false;
  const bool add = c->storm_add;
  c->storm_add = false;
  return launch_sig_commit(c->d, c->storm_parts, true, c->storm_n, c->storm_state, add ? c->storm_nw : c->n_waiters,
                           add, c->add_state, c->add_target, c->add_twait);
}

static int fail(tgsim_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    try {
      c->err = buf;
    } catch (...) {  // no memory for the message: the code still reports the error
      c->err.clear();
    }
  }
  return code;
}

// Every int-returning entry point runs its body through this guard: nothing thrown by the host
// side (std::vector / std::string growth, std::unordered_map) crosses extern "C" into a Go or
// Python caller. An allocation failure is TGSIM_ENOMEM and leaves the context usable: the tables
// are rebuilt into temporaries and swapped in only once complete.
// It also makes the context stream wait for a wheel insert still running on the side stream
// (Dev::side) - join = false only for the calls that may run beside it (the flood's reaction and
// publications touch neither the wheel nor the insert's inputs).
template <class F>
static int abi_guard(tgsim_ctx* c, F&& body, bool join = true) noexcept {
  try {
    if (join && c && c->d.side_pending) {
      const hipError_t e = join_side(c->d);
      if (e != hipSuccess) return fail(c, TGSIM_EHIP, "side stream: %s", hipGetErrorString(e));
    }
    return body();
  } catch (const std::bad_alloc&) {
    return fail(c, TGSIM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(c, TGSIM_EINVAL, "internal error: %s", e.what());
  } catch (...) {
    return fail(c, TGSIM_EINVAL, "internal error");
  }
}

static int hipfail(tgsim_ctx* c, hipError_t e, const char* what) {
  return fail(c, TGSIM_EHIP, "%s: %s", what, hipGetErrorString(e));
}

#define HIPCK(c, x, what)                          \
  do {                                             \
    hipError_t e__ = (x);                          \
    if (e__ != hipSuccess) return hipfail(c, e__, what); \
  } while (0)

constexpr uint32_t kStatusOnDevice = 0xFFFFFFFFu;  // n_status_last: the count is sc->n_msgs_last

// A pinned upload buffer of at least `bytes` in *out, once the copies that last used it have completed.
static int pin_acquire(tgsim_ctx* c, tgsim_ctx::Pinned& b, size_t bytes, uint8_t** out) {
  if (b.busy) {
    HIPCK(c, hipEventSynchronize(b.ev), "pinned staging event");
    b.busy = false;
  }
  if (!b.ev) HIPCK(c, hipEventCreateWithFlags(&b.ev, hipEventDisableTiming), "event");
  if (bytes > b.cap) {
    const size_t cap = std::max<size_t>({bytes, 2 * b.cap, (size_t)1 << 16});
    if (b.p) (void)hipHostFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    if (hipHostMalloc((void**)&b.p, cap, hipHostMallocDefault) != hipSuccess)
      return fail(c, TGSIM_ENOMEM, "pinned staging (%zu bytes)", cap);
    b.cap = cap;
  }
  *out = b.p;
  return TGSIM_OK;
}
// The copies out of b have been issued on the ctx stream.
static int pin_issued(tgsim_ctx* c, tgsim_ctx::Pinned& b) {
  HIPCK(c, hipEventRecord(b.ev, c->d.stream), "event");
  b.busy = true;
  return TGSIM_OK;
}

static void dfree(tgsim_ctx* c, void* p) {
  if (!p) return;
  auto it = std::find(c->allocs.begin(), c->allocs.end(), p);
  if (it != c->allocs.end()) c->allocs.erase(it);
  (void)hipFree(p);
}

template <typename T>
static int dalloc(tgsim_ctx* c, T** p, size_t n) {
  void* q = nullptr;
  size_t bytes = n * sizeof(T);
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess) return fail(c, TGSIM_ENOMEM, "hipMalloc(%zu bytes): %s", bytes, hipGetErrorString(e));
  c->allocs.push_back(q);
  *p = static_cast<T*>(q);
  return 0;
}

// ============================== LinkShape -> device shape ====================================

static uint32_t go_u32_of_double(double v) {  // Go uint32(float) on amd64: via int64, low 32 bits
  if (!(v > -9.2233720368547758e18 && v < 9.2233720368547758e18)) return 0u;
  return (uint32_t)(uint64_t)(int64_t)v;
}
static uint32_t pct2u32(float pct) {  // netlink Percentage2u32 [EXT]
  if (pct == 100.0f) return 0xFFFFFFFFu;
  volatile float q = pct / 100.0f;
  volatile float v = 4294967296.0f * q;
  return go_u32_of_double((double)v);
}
static uint32_t time2tick(uint32_t us) { return (uint32_t)(((uint64_t)us * 125u) >> 3); }  // us * 15.625
static uint32_t to_us(int64_t ns) {  // link.go:143-151
  int64_t us = ns / 1000;
  if (us > (int64_t)0xFFFFFFFFu) us = 0xFFFFFFFFu;
  return (uint32_t)(uint64_t)us;
}

// rho (optional): netem correlations (dup, corrupt, reorder, 0) via netlink Percentage2u32
static int compile_shape(const tgsim_link_shape& s, ShapeDev& o, std::string* err, uint32_t* rho = nullptr) {
  memset(&o, 0, sizeof(o));
  const uint64_t bw = s.bandwidth_bps == 0 ? UINT64_MAX : s.bandwidth_bps;  // link.go:156-159
  const uint64_t rate = bw / 8;                                               // netlink NewHtbClass
  if (rate == 0) {
    if (err) *err = "invalid htb rate";
    return TGSIM_EINVAL;
  }
  o.flags = s.bandwidth_bps != 0 ? kShLimited : 0u;
  // psched_ratecfg_precompute [EXT]
  uint64_t factor = 1000000000ull;
  uint32_t mult = 1, shift = 0;
  for (;;) {
    mult = (uint32_t)(factor / rate);
    if ((mult & (1u << 31)) || (factor & (1ull << 63))) break;
    factor <<= 1;
    ++shift;
  }
  o.mult = mult;
  o.shift = shift;
  const uint32_t buf_bytes = go_u32_of_double((double)rate / 1e9 + 1600.0);
  const uint32_t buf_us = go_u32_of_double(1000000.0 * ((double)buf_bytes / (double)rate));
  o.tau = (int64_t)time2tick(buf_us) << 6;
  const uint32_t lat_ticks = time2tick(to_us(s.latency_ns));
  const uint32_t jit_us = to_us(s.jitter_ns);
  const uint32_t jit_ticks = lat_ticks > 0 ? time2tick(jit_us) : jit_us;  // netlink NewNetem quirk [EXT]
  o.mu = (int64_t)lat_ticks << 6;
  o.sigma = (int32_t)(uint32_t)((uint64_t)jit_ticks << 6);
  o.loss_t = pct2u32(s.loss);
  o.dup_t = pct2u32(s.duplicate);
  o.corrupt_t = pct2u32(s.corrupt);
  o.reorder_t = pct2u32(s.reorder);
  // correlations (link.go:173-178): get_crandom is only reached when the probability is non-zero
  const uint32_t dr = s.duplicate_corr != 0.0f ? pct2u32(s.duplicate_corr) : 0u;
  const uint32_t cr = s.corrupt_corr != 0.0f ? pct2u32(s.corrupt_corr) : 0u;
  const uint32_t rr = s.reorder_corr != 0.0f ? pct2u32(s.reorder_corr) : 0u;
  if ((dr && o.dup_t) || (cr && o.corrupt_t) || (rr && o.reorder_t)) o.flags |= kShCorr;
  if (rho) { rho[0] = dr; rho[1] = cr; rho[2] = rr; rho[3] = 0; }
  return TGSIM_OK;
}

static ShapeDev default_shape() {
  tgsim_link_shape z;
  memset(&z, 0, sizeof(z));
  ShapeDev o;
  compile_shape(z, o, nullptr);
  return o;
}

// ============================== lifecycle ====================================================

extern "C" const char* tgsim_version(void) { return TGSIM_VERSION_STRING; }
extern "C" int tgsim_abi_version(void) { return TGSIM_ABI_VERSION; }

extern "C" void tgsim_destroy(tgsim_ctx* c) {
  if (!c) return;
  if (c->d.side) (void)hipStreamSynchronize(c->d.side);
  if (c->d.stream) (void)hipStreamSynchronize(c->d.stream);
  for (tgsim_ctx::Pinned* b : {&c->pin_msgs, &c->pin_marks, &c->pin_tcp}) {
    if (b->p) (void)hipHostFree(b->p);
    if (b->ev) (void)hipEventDestroy(b->ev);
  }
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->d.h_sc) (void)hipHostFree(c->d.h_sc);
  if (c->tcp_snap) (void)hipHostFree(c->tcp_snap);
  if (c->pend_host) (void)hipHostFree(c->pend_host);
  for (hipEvent_t e : c->tcp_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->own_stream && c->d.stream) (void)hipStreamDestroy(c->d.stream);
  if (c->d.side) (void)hipStreamDestroy(c->d.side);
  for (hipEvent_t e : {c->d.side_ev, c->d.main_ev})
    if (e) (void)hipEventDestroy(e);
  delete c;
}

static int create_impl(const tgsim_config* cfg, tgsim_ctx** out);

// Every allocation failure inside the C ABI is an error code, never an exception across extern "C".
extern "C" int tgsim_create(const tgsim_config* cfg, tgsim_ctx** out) {
  try {
    return create_impl(cfg, out);
  } catch (const std::bad_alloc&) {
    if (out) *out = nullptr;
    return TGSIM_ENOMEM;
  }
}

static int create_impl(const tgsim_config* cfg, tgsim_ctx** out) {
  if (!out) return TGSIM_EINVAL;
  *out = nullptr;
  if (!cfg || cfg->n_instances == 0 || cfg->n_shards == 0 || cfg->n_shards > (uint32_t)kMaxShards ||
      cfg->shard_id >= cfg->n_shards || cfg->data_prefix_len < 1 || cfg->data_prefix_len > 30)
    return TGSIM_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return TGSIM_ENODEV;
  if ((int)cfg->device >= ndev) return TGSIM_ENODEV;
  if (hipSetDevice((int)cfg->device) != hipSuccess) return TGSIM_ENODEV;

  tgsim_ctx* c = new tgsim_ctx();
  struct Guard {  // a bad_alloc below frees the half-built context
    tgsim_ctx*& c;
    ~Guard() { if (c) tgsim_destroy(c); }
  } guard{c};
  c->cfg = *cfg;
  c->N = cfg->n_instances;
  c->S = cfg->n_shards;
  c->shard = cfg->shard_id;
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, (int)cfg->device) == hipSuccess && ncu > 0)
      c->d.n_cu = ncu;
  }
  c->lo = (uint32_t)(((uint64_t)c->shard * c->N) / c->S);
  c->hi = (uint32_t)(((uint64_t)(c->shard + 1) * c->N) / c->S);
  c->nloc = c->hi - c->lo;
  c->data_len = cfg->data_prefix_len;
  c->data_mask = 0xFFFFFFFFu << (32 - c->data_len);
  c->data_net = cfg->data_subnet & c->data_mask;
  const uint64_t space = 1ull << (32 - c->data_len);
  if ((uint64_t)c->N + 3 > space || (kExternalIp & c->data_mask) == c->data_net) {
    return TGSIM_EINVAL;
  }
  Dev& d = c->d;
  d.N = c->N; d.S = c->S; d.shard = c->shard; d.lo = c->lo; d.nloc = c->nloc;
  d.data_net = c->data_net; d.data_mask = c->data_mask; d.data_len = c->data_len;
  d.key0 = (uint32_t)cfg->seed; d.key1 = (uint32_t)(cfg->seed >> 32);
  d.slot_ns = cfg->wheel_slot_ns > 0 ? cfg->wheel_slot_ns : 1000000;
  d.slots = cfg->wheel_slots ? cfg->wheel_slots : 1024;
  const uint64_t cap_msgs = cfg->max_msgs_per_window ? cfg->max_msgs_per_window : (1u << 20);
  const uint64_t cap_rec = cfg->max_records ? cfg->max_records : (1u << 22);
  // group-by limits: <= 2^20 instances per shard, <= 2^24 sync states, <= 2048 wheel slots
  if (cap_msgs > 0x7FFFFFFFull || cap_rec > 0x7FFFFFFFull || d.slots < 2 || d.slots > (uint32_t)kMaxBins ||
      c->nloc > (1u << 20) || (cfg->max_states && cfg->max_states > (1u << 24))) {
    return TGSIM_EINVAL;
  }
  d.cap_msgs = (uint32_t)cap_msgs;
  d.cap_rec = (uint32_t)cap_rec;
  d.subcap = (uint32_t)(cap_rec / kNSub + 4096);  // per sub-queue, with headroom for imbalance
  const size_t phys_rec = (size_t)kNSub * d.subcap;
  d.cap_arena = 2 * cap_rec;
  const uint64_t xcap = c->S > 1 ? (cfg->exchange_cap ? cfg->exchange_cap : 65536) : 1;
  // a header and a record per peer block; slot offsets in 32 bits (Queues::xslot)
  if ((c->S > 1 && xcap < 2) || (uint64_t)c->S * xcap >= (1ull << 32)) return TGSIM_EINVAL;
  d.xcap = (uint32_t)xcap;
  d.max_states = cfg->max_states ? cfg->max_states : 4096;
  d.max_waiters = cfg->max_waiters ? cfg->max_waiters : 65536;
  d.max_signals = cfg->max_signals ? cfg->max_signals : (1ull << 24);
  d.s_cap = std::max<uint32_t>(c->nloc, 1u << 16);

  hipError_t e = hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking);
  if (e != hipSuccess) return TGSIM_EHIP;
  c->own_stream = true;
  if (hipHostMalloc((void**)&d.h_sc, sizeof(DevScalars), hipHostMallocDefault) != hipSuccess) return TGSIM_ENOMEM;
  memset(d.h_sc, 0, sizeof(DevScalars));

  const size_t nl1 = (size_t)c->nloc + 1;
  const size_t segK = std::max<size_t>(std::max<size_t>(c->nloc, d.slots), d.max_states) + 1;
  int rc = 0;
  rc |= dalloc(c, &d.sc, 1);
  rc |= dalloc(c, &d.shape, std::max<size_t>(c->nloc, 1));
  rc |= dalloc(c, &d.tbs, std::max<size_t>(c->nloc, 1));
  rc |= dalloc(c, &d.zd, (size_t)c->nloc / 32 + 1);
  rc |= dalloc(c, &d.X, std::max<size_t>(c->nloc, 1));
  rc |= dalloc(c, &d.pend, std::max<size_t>(c->nloc, 1) << pend_shift(c->nloc));
  rc |= dalloc(c, &d.seq_done, std::max<size_t>(c->nloc, 1));
  rc |= dalloc(c, &c->d_red2, 2);
  rc |= dalloc(c, &d.moff, segK);
  rc |= dalloc(c, &d.ipf, c->N);
  rc |= dalloc(c, &d.en_bits, (size_t)c->N / 32 + 1);
  rc |= dalloc(c, &d.rule_off, nl1);
  rc |= dalloc(c, &d.rules, 1);
  rc |= dalloc(c, &d.m_src, d.cap_msgs);
  rc |= dalloc(c, &d.m_dst, d.cap_msgs);
  rc |= dalloc(c, &d.m_seq, d.cap_msgs);
  rc |= dalloc(c, &d.m_size, d.cap_msgs);
  rc |= dalloc(c, &d.m_t, d.cap_msgs);
  rc |= dalloc(c, &d.status, d.cap_msgs);
  rc |= dalloc(c, &d.corr_idx, (size_t)kDeferSub * defer_seg_cap(d.cap_msgs));
  rc |= dalloc(c, &d.corr_sorted, d.cap_msgs);
  rc |= dalloc(c, &d.cor_rho, 4 * (size_t)std::max<uint32_t>(c->nloc, 1));
  rc |= dalloc(c, &d.cor_last, 4 * (size_t)std::max<uint32_t>(c->nloc, 1));
  rc |= dalloc(c, &d.A, phys_rec);
  rc |= dalloc(c, &d.D, phys_rec);
  rc |= dalloc(c, &d.L, phys_rec);
  rc |= dalloc(c, &d.KA, phys_rec);
  rc |= dalloc(c, &d.KD, phys_rec);
  rc |= dalloc(c, &d.KL, phys_rec);
  rc |= dalloc(c, &d.arena, d.cap_arena);
  rc |= dalloc(c, &d.xsend, (size_t)c->S * d.xcap);
  rc |= dalloc(c, &d.xrecv, (size_t)c->S * d.xcap);
  rc |= dalloc(c, &d.regions, kMaxRegions);
  rc |= dalloc(c, &d.dirs, (size_t)kMaxRegions * (d.slots + 1));
  rc |= dalloc(c, &d.plan_start, kMaxRegions + 1);
  rc |= dalloc(c, &d.plan_off, kMaxRegions + 1);
  // every per-window item array holds the physical queue space (kNSub sub-queues of subcap): a
  // window can carry up to kNSub * subcap > cap_rec items before the overflow bits stop it
  rc |= dalloc(c, &d.keys0, phys_rec);
  rc |= dalloc(c, &d.keys1, phys_rec);
  rc |= dalloc(c, &d.keys2, phys_rec);
  rc |= dalloc(c, &d.kv1, phys_rec);
  rc |= dalloc(c, &d.vals0, phys_rec);
  rc |= dalloc(c, &d.vals1, phys_rec);
  rc |= dalloc(c, &d.vals2, phys_rec);
  rc |= dalloc(c, &d.poff, (size_t)kRadixBlocks * (kMaxBins + 1));
  rc |= dalloc(c, &d.hist, (size_t)kMaxBins * kRadixBlocks);
  rc |= dalloc(c, &d.histx, (size_t)kMaxBins * kRadixBlocks);
  rc |= dalloc(c, &d.tot, kMaxBins);
  rc |= dalloc(c, &d.bstart, kMaxBins + 1);
  rc |= dalloc(c, &d.qc, (size_t)kQcLines * 32);
  rc |= dalloc(c, &d.pend_part, kRadixBlocks);
  rc |= dalloc(c, &d.sig_red, 4);
  rc |= dalloc(c, &d.sig_part, 2 * 4096);
  rc |= dalloc(c, &d.stats, (size_t)kNSub * 16);
  rc |= dalloc(c, &d.seg_off, segK);
  rc |= dalloc(c, &d.large, phys_rec / kTile + 16);
  rc |= dalloc(c, &d.medium, segK);
  rc |= dalloc(c, &d.chunk_off, phys_rec / kTile + 17);
  rc |= dalloc(c, &d.K1a, phys_rec);
  rc |= dalloc(c, &d.K1b, phys_rec);
  rc |= dalloc(c, &d.K2a, phys_rec);
  rc |= dalloc(c, &d.K2b, phys_rec);
  rc |= dalloc(c, &d.K3a, phys_rec);
  rc |= dalloc(c, &d.K3b, phys_rec);
  rc |= dalloc(c, &d.o_t, phys_rec);
  rc |= dalloc(c, &d.o_src, phys_rec);
  rc |= dalloc(c, &d.o_dst, phys_rec);
  rc |= dalloc(c, &d.o_seq, phys_rec);
  rc |= dalloc(c, &d.o_size, phys_rec);
  rc |= dalloc(c, &d.o_flags, phys_rec);
  rc |= dalloc(c, &d.o_coff, phys_rec);
  rc |= dalloc(c, &d.inbox, nl1);
  rc |= dalloc(c, &d.s_state, d.s_cap);
  rc |= dalloc(c, &d.s_inst, d.s_cap);
  rc |= dalloc(c, &d.s_seq, d.s_cap);
  rc |= dalloc(c, &d.s_t, d.s_cap);
  rc |= dalloc(c, &d.st_count, d.max_states);
  rc |= dalloc(c, &d.st_last, d.max_states);
  rc |= dalloc(c, &d.st_nchunks, d.max_states);
  rc |= dalloc(c, &d.st_chunks, (size_t)d.max_states * kMaxChunksPerState);
  rc |= dalloc(c, &d.sig_log, d.max_signals);
  rc |= dalloc(c, &d.w_state, d.max_waiters);
  rc |= dalloc(c, &d.w_target, d.max_waiters);
  rc |= dalloc(c, &d.w_twait, d.max_waiters);
  rc |= dalloc(c, &d.w_release, d.max_waiters);
  if (rc) return TGSIM_ENOMEM;
  c->rules_cap_dev = 1;
  init_launch_geometry(d);

  hipStream_t s = d.stream;
  bool ok = hipMemsetAsync(d.sc, 0, sizeof(DevScalars), s) == hipSuccess &&
            hipMemsetAsync(d.st_count, 0, d.max_states * sizeof(uint32_t), s) == hipSuccess &&
            hipMemsetAsync(d.stats, 0, (size_t)kNSub * 16 * sizeof(unsigned long long), s) == hipSuccess &&
            hipMemsetAsync(d.st_nchunks, 0, d.max_states * sizeof(uint32_t), s) == hipSuccess &&
            hipMemsetAsync(d.st_last, 0, d.max_states * sizeof(int64_t), s) == hipSuccess &&
            hipMemsetAsync(d.rule_off, 0, nl1 * sizeof(uint32_t), s) == hipSuccess &&
            hipMemsetAsync(d.inbox, 0, nl1 * sizeof(uint32_t), s) == hipSuccess &&
            hipMemsetAsync(d.pend, 0, (std::max<size_t>(c->nloc, 1) << pend_shift(c->nloc)) * sizeof(uint32_t), s) == hipSuccess;
  if (!ok) return TGSIM_EHIP;

  // initial state = after the sidecar's Config{Network:"default", Enable:true} (sidecar_handler.go:26-29)
  c->shape_h.assign(c->nloc, default_shape());
  c->rho_h.assign(4 * (size_t)c->nloc, 0u);
  c->corr_epoch.assign(c->nloc, 0u);
  c->flags_h.assign(c->N, 1u);  // enabled, external routing off (zero RoutingPolicy -> disable)
  c->ip_h.resize(c->N);
  c->space = space;
  c->hcnt.assign(c->nloc, 0u);
  for (uint32_t g = 0; g < c->N; ++g) c->ip_h[g] = c->data_net + 2u + g;
  c->rules_h.assign(c->nloc, {});
  std::vector<int64_t> xs(std::max<uint32_t>(c->nloc, 1), kNegInf);
  if (hipMemcpy(d.X, xs.data(), xs.size() * sizeof(int64_t), hipMemcpyHostToDevice) != hipSuccess) {
    return TGSIM_EHIP;
  }
  *out = c;
  c = nullptr;  // owned by the caller now
  return TGSIM_OK;
}

extern "C" const char* tgsim_last_error(const tgsim_ctx* c) { return c ? c->err.c_str() : "null context"; }

static int tgsim_set_stream_body(tgsim_ctx* c, void* stream);
extern "C" int tgsim_set_stream(tgsim_ctx* c, void* stream) {
  return abi_guard(c, [&] { return tgsim_set_stream_body(c, stream); });
}
static int tgsim_set_stream_body(tgsim_ctx* c, void* stream) {
  if (!c) return TGSIM_EINVAL;
  HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
  if (c->own_stream) (void)hipStreamDestroy(c->d.stream);
  if (stream) {
    c->d.stream = (hipStream_t)stream;
    c->own_stream = false;
  } else {
    HIPCK(c, hipStreamCreateWithFlags(&c->d.stream, hipStreamNonBlocking), "stream");
    c->own_stream = true;
  }
  return TGSIM_OK;
}

static int tgsim_shard_range_body(const tgsim_ctx* c, uint32_t* lo, uint32_t* hi);
extern "C" int tgsim_shard_range(const tgsim_ctx* c, uint32_t* lo, uint32_t* hi) {
  return abi_guard(const_cast<tgsim_ctx*>(c), [&] { return tgsim_shard_range_body(c, lo, hi); });
}
static int tgsim_shard_range_body(const tgsim_ctx* c, uint32_t* lo, uint32_t* hi) {
  if (!c) return TGSIM_EINVAL;
  *lo = c->lo;
  *hi = c->hi;
  return TGSIM_OK;
}

static int check_device_errors(tgsim_ctx* c) {
  const uint32_t e = c->d.h_sc->err;
  if (!e) return TGSIM_OK;
  if (e & (ERR_CAP_A | ERR_CAP_D | ERR_CAP_L | ERR_CAP_X | ERR_ARENA | ERR_REGIONS | ERR_SIG_CAP | ERR_STATE_CHUNKS |
           ERR_QUEUE_CAP | ERR_CAP_M | ERR_TCP_TIMERS))
    return fail(c, TGSIM_ECAPACITY, "device capacity exceeded (err bits 0x%x)", e);
  if (e & (ERR_CAUSAL | ERR_SIG_ORDER)) return fail(c, TGSIM_ECAUSALITY, "causality violation on device (err 0x%x)", e);
  if (e & ERR_UNSORTED_TARGET)
    return fail(c, TGSIM_ENOTSUP, "barrier target falls inside a count-only signal batch (only its first/last member is known)");
  if (e & ERR_UNRELEASED) return fail(c, TGSIM_ESTATE, "advance_to_barrier: barrier not released");
  if (e & ERR_PROBE_SPAN)
    return fail(c, TGSIM_ENOTSUP, "probe reaction: a request arrived more than 2^40 ns before its window's end");
  return fail(c, TGSIM_EINVAL, "device error bits 0x%x", e);
}

static int sync_and_check(tgsim_ctx* c) {
  HIPCK(c, flush_storm(c), "storm commit");
  HIPCK(c, sync_scalars(c->d), "sync");
  if (c->now_from_device && !c->in_window) {
    c->horizon = c->d.h_sc->T;
    c->now = c->d.h_sc->t_end;
    c->now_from_device = false;
  }
  return check_device_errors(c);
}

static int tgsim_sync_body(tgsim_ctx* c);
extern "C" int tgsim_sync(tgsim_ctx* c) {
  return abi_guard(c, [&] { return tgsim_sync_body(c); });
}
static int tgsim_sync_body(tgsim_ctx* c) {
  if (!c) return TGSIM_EINVAL;
  return sync_and_check(c);
}

static int tgsim_get_stats_body(tgsim_ctx* c, tgsim_stats* o);
extern "C" int tgsim_get_stats(tgsim_ctx* c, tgsim_stats* o) {
  return abi_guard(c, [&] { return tgsim_get_stats_body(c, o); });
}
static int tgsim_get_stats_body(tgsim_ctx* c, tgsim_stats* o) {
  if (!c || !o) return TGSIM_EINVAL;
  int rc = sync_and_check(c);
  const DevScalars& h = *c->d.h_sc;
  std::vector<unsigned long long> rows((size_t)kNSub * 16);
  HIPCK(c, hipMemcpy(rows.data(), c->d.stats, rows.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost), "stats");
  unsigned long long st[16] = {};
  for (int r = 0; r < kNSub; ++r)
    for (int k = 0; k < 16; ++k) st[k] += rows[(size_t)r * 16 + k];
  o->msgs_in = st[ST_MSGS]; o->copies = st[ST_COPIES]; o->lost = st[ST_LOST];
  o->dropped = st[ST_DROPPED]; o->rejected = st[ST_REJECTED]; o->unreachable = st[ST_UNREACH];
  o->external = st[ST_EXTERNAL]; o->dest_down = st[ST_DESTDOWN]; o->local = st[ST_LOCAL];
  o->delivered = h.st[ST_DELIVERED];
  o->windows = 0;
  o->inflight = h.arena_used;
  o->tb_items = h.st[ST_TB_ITEMS];
  o->extracted = h.st[ST_EXTRACTED];
  o->inserted = h.st[ST_INSERTED];
  o->overlimit = st[ST_OVERLIMIT];
  return rc;
}

static int tgsim_profile_set_body(tgsim_ctx* c, uint32_t mask);
extern "C" int tgsim_profile_set(tgsim_ctx* c, uint32_t mask) {
  return abi_guard(c, [&] { return tgsim_profile_set_body(c, mask); });
}
static int tgsim_profile_set_body(tgsim_ctx* c, uint32_t mask) {
  if (!c) return TGSIM_EINVAL;
  c->d.prof.mask = mask;
  return TGSIM_OK;
}

// Test hook: the n-th host allocation point from now (add_rules, flood_set_graph) throws
// std::bad_alloc, which the entry point must turn into TGSIM_ENOMEM with the context usable.
static int tgsim_debug_fail_alloc_body(tgsim_ctx* c, uint32_t nth);
extern "C" int tgsim_debug_fail_alloc(tgsim_ctx* c, uint32_t nth) {
  return abi_guard(c, [&] { return tgsim_debug_fail_alloc_body(c, nth); });
}
static int tgsim_debug_fail_alloc_body(tgsim_ctx* c, uint32_t nth) {
  if (!c) return TGSIM_EINVAL;
  c->fail_alloc = nth;
  return TGSIM_OK;
}

static int tgsim_profile_read_body(tgsim_ctx* c, double* ms, uint64_t* launches, size_t cap, size_t* n);
extern "C" int tgsim_profile_read(tgsim_ctx* c, double* ms, uint64_t* launches, size_t cap, size_t* n) {
  return abi_guard(c, [&] { return tgsim_profile_read_body(c, ms, launches, cap, n); });
}
static int tgsim_profile_read_body(tgsim_ctx* c, double* ms, uint64_t* launches, size_t cap, size_t* n) {
  if (!c || !n) return TGSIM_EINVAL;
  int rc = sync_and_check(c);
  *n = KID_COUNT;
  if (cap < (size_t)KID_COUNT) return fail(c, TGSIM_ECAPACITY, "profile capacity");
  for (int k = 0; k < KID_COUNT; ++k) {
    if (ms) ms[k] = c->d.prof.ms[k];
    if (launches) launches[k] = c->d.prof.n[k];
  }
  return rc;
}

static int tgsim_kernel_counters_body(tgsim_ctx* c, uint64_t* out, size_t cap, size_t* n);
extern "C" int tgsim_kernel_counters(tgsim_ctx* c, uint64_t* out, size_t cap, size_t* n) {
  return abi_guard(c, [&] { return tgsim_kernel_counters_body(c, out, cap, n); });
}
static int tgsim_kernel_counters_body(tgsim_ctx* c, uint64_t* out, size_t cap, size_t* n) {
  if (!c || !n) return TGSIM_EINVAL;
  *n = KC_COUNT;
  if (!out) return TGSIM_OK;
  if (cap < (size_t)KC_COUNT) return fail(c, TGSIM_ECAPACITY, "counter capacity");
  const int rc = sync_and_check(c);
  if (rc) return rc;
  for (int k = 0; k < KC_COUNT; ++k) out[k] = c->d.h_sc->kc[k];
  return TGSIM_OK;
}

extern "C" int tgsim_kernel_classes(void) { return KID_COUNT; }
extern "C" const char* tgsim_kernel_name(int k) { return (k >= 0 && k < KID_COUNT) ? kKernelNames[k] : "?"; }

// The host view of the clock lags behind device-ended windows until the next synchronisation.
static void refresh_clock(const tgsim_ctx* cc) {
  tgsim_ctx* c = const_cast<tgsim_ctx*>(cc);
  if (c->now_from_device && !c->in_window) (void)sync_and_check(c);
}
extern "C" int64_t tgsim_now(const tgsim_ctx* c) {
  if (!c) return -1;
  refresh_clock(c);
  return c->now;
}
extern "C" int64_t tgsim_horizon(const tgsim_ctx* c) {
  if (!c) return -1;
  refresh_clock(c);
  return c->horizon;
}

// ============================== network configuration ========================================

static bool is_local(const tgsim_ctx* c, uint32_t g) { return g >= c->lo && g < c->hi; }

static int tgsim_set_shape_body(tgsim_ctx* c, uint32_t g, const tgsim_link_shape* s);
extern "C" int tgsim_set_shape(tgsim_ctx* c, uint32_t g, const tgsim_link_shape* s) {
  return abi_guard(c, [&] { return tgsim_set_shape_body(c, g, s); });
}
static int tgsim_set_shape_body(tgsim_ctx* c, uint32_t g, const tgsim_link_shape* s) {
  if (!c || !s || g >= c->N) return fail(c, TGSIM_EINVAL, "bad instance");
  ShapeDev o;
  std::string e;
  uint32_t rho[4];
  int rc = compile_shape(*s, o, &e, rho);
  if (rc) return fail(c, rc, "%s", e.c_str());
  if (is_local(c, g)) {
    const uint32_t l = g - c->lo;
    c->shape_h[l] = o;
    memcpy(&c->rho_h[4 * (size_t)l], rho, sizeof(rho));
    c->shape_dirty = true;
    // netem_change -> init_crandom: every Shape re-seeds the correlation state [EXT]
    c->corr_reset.push_back(l);
    c->corr_reset.push_back(++c->corr_epoch[l]);
  }
  return TGSIM_OK;
}

static int tgsim_set_shapes_body(tgsim_ctx* c, const uint32_t* inst, const tgsim_link_shape* shapes, size_t n);
extern "C" int tgsim_set_shapes(tgsim_ctx* c, const uint32_t* inst, const tgsim_link_shape* shapes, size_t n) {
  return abi_guard(c, [&] { return tgsim_set_shapes_body(c, inst, shapes, n); });
}
static int tgsim_set_shapes_body(tgsim_ctx* c, const uint32_t* inst, const tgsim_link_shape* shapes, size_t n) {
  if (!c || (n && (!inst || !shapes))) return fail(c, TGSIM_EINVAL, "bad arguments");
  for (size_t i = 0; i < n; ++i) {
    int rc = tgsim_set_shape(c, inst[i], &shapes[i]);
    if (rc) return rc;
  }
  return TGSIM_OK;
}

static bool rule_before(const RuleDev& a, uint32_t prefix, uint32_t plen) {
  const uint32_t la = a.plen_action & 0xFFu;
  if (la != plen) return la > plen;
  return a.prefix < prefix;
}

// NetlinkLink.AddRules (link.go:187-217): the rules in order, each a RouteReplace (Drop, Reject) or
// a RouteDel of both routes for exactly that prefix (Accept, errors ignored); the first invalid rule
// returns its error with the earlier ones applied, as the reference's loop does. A batch is applied
// as one sort + merge (the last rule per prefix wins): O(R log R + table), not O(R) per rule.
static int tgsim_add_rules_body(tgsim_ctx* c, uint32_t g, const tgsim_link_rule* rules, size_t n);
extern "C" int tgsim_add_rules(tgsim_ctx* c, uint32_t g, const tgsim_link_rule* rules, size_t n) {
  return abi_guard(c, [&] { return tgsim_add_rules_body(c, g, rules, n); });
}
static int tgsim_add_rules_body(tgsim_ctx* c, uint32_t g, const tgsim_link_rule* rules, size_t n) {
  if (!c || g >= c->N || (n && !rules)) return fail(c, TGSIM_EINVAL, "bad arguments");
  struct Op { uint32_t prefix, plen, action, idx; };
  std::vector<Op> ops;
  int rc = TGSIM_OK;
  const bool local = is_local(c, g);
  if (local) ops.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t plen = rules[i].prefix_len;
    if (plen > 32) { rc = fail(c, TGSIM_EINVAL, "invalid prefix length %u", plen); break; }
    const uint32_t mask = plen ? 0xFFFFFFFFu << (32 - plen) : 0u;
    const uint32_t prefix = rules[i].subnet_ip;
    const int action = rules[i].shape.filter;
    if (action != TGSIM_FILTER_ACCEPT && action != TGSIM_FILTER_REJECT && action != TGSIM_FILTER_DROP) {
      rc = fail(c, TGSIM_EINVAL, "unknown filter action %d", action);
      break;
    }
    if (action != TGSIM_FILTER_ACCEPT && (prefix & ~mask)) {
      rc = fail(c, TGSIM_EINVAL, "invalid prefix for given prefix length");
      break;
    }
    if (!local) continue;
    if (action == TGSIM_FILTER_ACCEPT && (prefix & ~mask)) continue;  // RouteDel finds nothing
    ops.push_back(Op{prefix, plen, (uint32_t)action, (uint32_t)i});
  }
  if (ops.empty()) return rc;
  alloc_point(c);
  // table order (plen desc, prefix asc); within a key the batch order, so the last op is the one kept
  std::sort(ops.begin(), ops.end(), [](const Op& a, const Op& b) {
    if (a.plen != b.plen) return a.plen > b.plen;
    if (a.prefix != b.prefix) return a.prefix < b.prefix;
    return a.idx < b.idx;
  });
  auto& v = c->rules_h[g - c->lo];
  std::vector<RuleDev> out;
  out.reserve(v.size() + ops.size());
  size_t j = 0;
  bool changed = false;
  for (size_t i = 0; i < ops.size();) {
    size_t k = i;
    while (k + 1 < ops.size() && ops[k + 1].plen == ops[i].plen && ops[k + 1].prefix == ops[i].prefix) ++k;
    const Op& o = ops[k];  // the last rule for this prefix
    while (j < v.size() && rule_before(v[j], o.prefix, o.plen)) out.push_back(v[j++]);
    const bool present = j < v.size() && v[j].prefix == o.prefix && (v[j].plen_action & 0xFFu) == o.plen;
    if (o.action == TGSIM_FILTER_ACCEPT) {
      if (present) { ++j; changed = true; }
    } else {
      const uint32_t pa = o.plen | (o.action << 8);
      if (present) ++j;
      out.push_back(RuleDev{o.prefix, pa});
      changed = true;
    }
    i = k + 1;
  }
  while (j < v.size()) out.push_back(v[j++]);
  if (changed) {
    v.swap(out);
    c->rules_dirty = true;
  }
  return rc;
}

static int tgsim_set_policy_body(tgsim_ctx* c, uint32_t g, int32_t policy);
extern "C" int tgsim_set_policy(tgsim_ctx* c, uint32_t g, int32_t policy) {
  return abi_guard(c, [&] { return tgsim_set_policy_body(c, g, policy); });
}
static int tgsim_set_policy_body(tgsim_ctx* c, uint32_t g, int32_t policy) {  // route.go:102-117
  if (!c || g >= c->N) return fail(c, TGSIM_EINVAL, "bad instance");
  const uint8_t f = (uint8_t)((c->flags_h[g] & 1u) | (policy == TGSIM_POLICY_ALLOW_ALL ? 2u : 0u));
  if (f != c->flags_h[g]) { c->flags_h[g] = f; c->flags_dirty = true; }
  return TGSIM_OK;
}

// The instance holding data-subnet address offset off, or UINT32_MAX.
static uint32_t holder_of(const tgsim_ctx* c, uint32_t off) {
  const auto it = c->moved.find(off);
  if (it != c->moved.end()) return it->second;
  if (off >= 2 && off - 2 < c->N && c->ip_h[off - 2] == c->data_net + off) return off - 2;
  return UINT32_MAX;
}

static int set_ip(tgsim_ctx* c, uint32_t g, uint32_t ip) {
  if ((ip & c->data_mask) != c->data_net) return fail(c, TGSIM_EINVAL, "ip outside the data subnet");
  const uint32_t off = ip - c->data_net;
  if (off <= 1 || off == (uint32_t)(c->space - 1)) return fail(c, TGSIM_EINVAL, "reserved address");
  const uint32_t h = holder_of(c, off);
  if (h != UINT32_MAX && h != g) return fail(c, TGSIM_EINVAL, "address already in use");
  c->moved.erase(c->ip_h[g] - c->data_net);
  c->ip_h[g] = ip;
  if (off != g + 2u) c->moved[off] = g;
  c->ip_dirty = true;
  return TGSIM_OK;
}

// docker_network.go:65-133: disconnect / (re)connect; a new link is a fresh HTB class + netem qdisc.
static int tgsim_set_enabled_body(tgsim_ctx* c, uint32_t g, int32_t enabled, int32_t has_ip, uint32_t ip);
extern "C" int tgsim_set_enabled(tgsim_ctx* c, uint32_t g, int32_t enabled, int32_t has_ip, uint32_t ip) {
  return abi_guard(c, [&] { return tgsim_set_enabled_body(c, g, enabled, has_ip, ip); });
}
static int tgsim_set_enabled_body(tgsim_ctx* c, uint32_t g, int32_t enabled, int32_t has_ip, uint32_t ip) {
  if (!c || g >= c->N) return fail(c, TGSIM_EINVAL, "bad instance");
  uint8_t& f = c->flags_h[g];
  if (!enabled) {
    if (f & 1u) { f &= ~1u; c->flags_dirty = true; }
    return TGSIM_OK;
  }
  if ((f & 1u) && has_ip && ip != c->ip_h[g]) { f &= ~1u; c->flags_dirty = true; }
  if (!(f & 1u)) {
    if (has_ip) {
      int rc = set_ip(c, g, ip);
      if (rc) return rc;
    }
    f |= 1u;
    c->flags_dirty = true;
    if (is_local(c, g)) {
      c->shape_h[g - c->lo] = default_shape();
      c->shape_dirty = true;
      c->tb_reset.push_back(g - c->lo);
    }
  }
  return TGSIM_OK;
}

static int tgsim_configure_network_body(tgsim_ctx* c, uint32_t g, const tgsim_network_config* cfg);
extern "C" int tgsim_configure_network(tgsim_ctx* c, uint32_t g, const tgsim_network_config* cfg) {
  return abi_guard(c, [&] { return tgsim_configure_network_body(c, g, cfg); });
}
static int tgsim_configure_network_body(tgsim_ctx* c, uint32_t g, const tgsim_network_config* cfg) {
  if (!c || !cfg || g >= c->N) return fail(c, TGSIM_EINVAL, "bad arguments");
  const char* net = cfg->network ? cfg->network : "";
  if (strcmp(net, "default") != 0) return fail(c, TGSIM_EUNSUPPORTED_NETWORK, "unsupported network: %s", net);
  int rc = tgsim_set_policy(c, g, cfg->routing_policy);
  if (rc) return rc;
  if (!cfg->enable) return tgsim_set_enabled(c, g, 0, 0, 0);
  rc = tgsim_set_enabled(c, g, 1, cfg->has_ipv4, cfg->ipv4);
  if (rc) return rc;
  rc = tgsim_set_shape(c, g, &cfg->default_shape);
  if (rc) return rc;
  return tgsim_add_rules(c, g, cfg->rules, cfg->n_rules);
}

// K8sNetwork.ConfigureNetwork, k8s_network.go:43-176: policy last, untouched by a disconnect.
static int tgsim_configure_network_order_body(tgsim_ctx* c, uint32_t g, const tgsim_network_config* cfg, int32_t order);
extern "C" int tgsim_configure_network_order(tgsim_ctx* c, uint32_t g, const tgsim_network_config* cfg, int32_t order) {
  return abi_guard(c, [&] { return tgsim_configure_network_order_body(c, g, cfg, order); });
}
static int tgsim_configure_network_order_body(tgsim_ctx* c, uint32_t g, const tgsim_network_config* cfg, int32_t order) {
  if (order == TGSIM_APPLY_DOCKER) return tgsim_configure_network(c, g, cfg);
  if (!c || !cfg || g >= c->N || order != TGSIM_APPLY_K8S) return fail(c, TGSIM_EINVAL, "bad arguments");
  const char* net = cfg->network ? cfg->network : "";
  if (strcmp(net, "default") != 0) return fail(c, TGSIM_EUNSUPPORTED_NETWORK, "unsupported network: %s", net);
  if (!cfg->enable) return tgsim_set_enabled(c, g, 0, 0, 0);
  int rc = tgsim_set_enabled(c, g, 1, cfg->has_ipv4, cfg->ipv4);
  if (rc) return rc;
  rc = tgsim_set_shape(c, g, &cfg->default_shape);
  if (rc) return rc;
  rc = tgsim_add_rules(c, g, cfg->rules, cfg->n_rules);
  if (rc) return rc;
  return tgsim_set_policy(c, g, cfg->routing_policy);
}

static int tgsim_get_ip_body(const tgsim_ctx* c, uint32_t g, uint32_t* ip);
extern "C" int tgsim_get_ip(const tgsim_ctx* c, uint32_t g, uint32_t* ip) {
  return abi_guard(const_cast<tgsim_ctx*>(c), [&] { return tgsim_get_ip_body(c, g, ip); });
}
static int tgsim_get_ip_body(const tgsim_ctx* c, uint32_t g, uint32_t* ip) {
  if (!c || !ip || g >= c->N) return TGSIM_EINVAL;
  *ip = c->ip_h[g];
  return TGSIM_OK;
}

static int upload_tables(tgsim_ctx* c) {
  Dev& d = c->d;
  bool copied = false;
  if (c->shape_dirty && c->nloc) {
    HIPCK(c, hipMemcpyAsync(d.shape, c->shape_h.data(), c->nloc * sizeof(ShapeDev), hipMemcpyHostToDevice, d.stream), "upload shapes");
    HIPCK(c, hipMemcpyAsync(d.cor_rho, c->rho_h.data(), c->rho_h.size() * 4, hipMemcpyHostToDevice, d.stream), "upload shapes");
    d.any_corr = false;
    c->any_dup = false;
    c->tbs_h.resize(c->nloc);
    c->zd_h.assign((size_t)c->nloc / 32 + 1, 0u);
    c->all_zd = true;
    for (uint32_t l = 0; l < c->nloc; ++l) {
      const ShapeDev& sh = c->shape_h[l];
      d.any_corr |= (sh.flags & kShCorr) != 0;
      d.ever_limited |= (sh.flags & kShLimited) != 0;  // sticky: its copies may still be in flight
      c->any_dup |= sh.dup_t != 0;
      c->tbs_h[l] = TbShape{sh.tau, sh.mult, sh.shift};
      if (sh.mu == 0 && sh.sigma == 0 && !(sh.flags & kShLimited)) c->zd_h[l >> 5] |= 1u << (l & 31u);
      else c->all_zd = false;
    }
    HIPCK(c, hipMemcpyAsync(d.tbs, c->tbs_h.data(), c->nloc * sizeof(TbShape), hipMemcpyHostToDevice, d.stream), "upload shapes");
    HIPCK(c, hipMemcpyAsync(d.zd, c->zd_h.data(), c->zd_h.size() * 4, hipMemcpyHostToDevice, d.stream), "upload shapes");
    copied = true;
  }
  if (!c->corr_reset.empty()) {
    const uint32_t n = (uint32_t)(c->corr_reset.size() / 2);
    if (n > c->corr_reset_cap) {
      HIPCK(c, hipStreamSynchronize(d.stream), "sync");
      dfree(c, c->corr_reset_dev);
      c->corr_reset_dev = nullptr;
      if (dalloc(c, &c->corr_reset_dev, 2 * (size_t)n)) return TGSIM_ENOMEM;
      c->corr_reset_cap = n;
    }
    HIPCK(c, hipMemcpyAsync(c->corr_reset_dev, c->corr_reset.data(), 2 * (size_t)n * 4, hipMemcpyHostToDevice, d.stream), "upload resets");
    HIPCK(c, launch_reset_corr(d, c->corr_reset_dev, n), "reset corr");
    copied = true;
  }
  std::vector<uint64_t> ipf;
  std::vector<uint32_t> en;
  if (c->flags_dirty || c->ip_dirty) {
    ipf.resize(c->N);
    en.assign((size_t)c->N / 32 + 1, 0u);
    for (uint32_t g = 0; g < c->N; ++g) {
      ipf[g] = (uint64_t)c->ip_h[g] | ((uint64_t)c->flags_h[g] << 32);
      en[g >> 5] |= (uint32_t)(c->flags_h[g] & 1u) << (g & 31u);
    }
    HIPCK(c, hipMemcpyAsync(d.ipf, ipf.data(), c->N * sizeof(uint64_t), hipMemcpyHostToDevice, d.stream), "upload ip/flags");
    HIPCK(c, hipMemcpyAsync(d.en_bits, en.data(), en.size() * 4, hipMemcpyHostToDevice, d.stream), "upload ip/flags");
    copied = true;
  }
  std::vector<uint32_t> off;
  std::vector<RuleDev> flat;
  if (c->rules_dirty) {
    off.resize((size_t)c->nloc + 1);
    size_t total = 0;
    for (uint32_t i = 0; i < c->nloc; ++i) { off[i] = (uint32_t)total; total += c->rules_h[i].size(); }
    off[c->nloc] = (uint32_t)total;
    if (total > 0xFFFFFFF0ull) return fail(c, TGSIM_ECAPACITY, "too many rules");
    flat.reserve(total);
    for (uint32_t i = 0; i < c->nloc; ++i) flat.insert(flat.end(), c->rules_h[i].begin(), c->rules_h[i].end());
    if (total > c->rules_cap_dev) {
      HIPCK(c, hipStreamSynchronize(d.stream), "sync");
      auto it = std::find(c->allocs.begin(), c->allocs.end(), (void*)d.rules);
      if (it != c->allocs.end()) { (void)hipFree(d.rules); c->allocs.erase(it); }
      size_t cap = std::max<size_t>(total, 2 * c->rules_cap_dev);
      if (dalloc(c, &d.rules, cap)) return TGSIM_ENOMEM;
      c->rules_cap_dev = cap;
    }
    HIPCK(c, hipMemcpyAsync(d.rule_off, off.data(), off.size() * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream), "upload rules");
    if (total)
      HIPCK(c, hipMemcpyAsync(d.rules, flat.data(), total * sizeof(RuleDev), hipMemcpyHostToDevice, d.stream), "upload rules");
    copied = true;
  }
  if (!c->tb_reset.empty()) {
    const uint32_t n = (uint32_t)c->tb_reset.size();
    if (n > c->tb_reset_cap) {
      HIPCK(c, hipStreamSynchronize(d.stream), "sync");
      if (dalloc(c, &c->tb_reset_dev, n)) return TGSIM_ENOMEM;
      c->tb_reset_cap = n;
    }
    HIPCK(c, hipMemcpyAsync(c->tb_reset_dev, c->tb_reset.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, d.stream), "upload resets");
    HIPCK(c, launch_reset_tb(d, c->tb_reset_dev, n), "reset tb");
    copied = true;
  }
  // host sources are pageable vectors that later calls may modify: wait for the copies
  if (copied) HIPCK(c, hipStreamSynchronize(d.stream), "sync uploads");
  c->tb_reset.clear();
  c->corr_reset.clear();
  c->shape_dirty = c->flags_dirty = c->ip_dirty = c->rules_dirty = false;
  return TGSIM_OK;
}

// ============================== data path ====================================================

static int validate_msgs(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    if (m->src[i] >= c->N || (m->dst[i] >= c->N && m->dst[i] != TGSIM_DST_EXTERNAL))
      return fail(c, TGSIM_EINVAL, "message %zu: bad instance id", i);
    if (!is_local(c, m->src[i])) return fail(c, TGSIM_EINVAL, "message %zu: sender not in this shard", i);
    if (m->t_send[i] < c->horizon) return fail(c, TGSIM_ECAUSALITY, "message %zu: t_send before the reaction horizon", i);
    if (m->size[i] >= 0x80000000u) return fail(c, TGSIM_EINVAL, "message %zu: size too large", i);
  }
  return TGSIM_OK;
}

static int enqueue_host(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n);
static int tgsim_enqueue_body(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n);
extern "C" int tgsim_enqueue(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  return abi_guard(c, [&] { return tgsim_enqueue_body(c, m, n); });
}
static int tgsim_enqueue_body(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (c && c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode: traffic goes through tgsim_tcp_send");
  return enqueue_host(c, m, n);
}
static int enqueue_host(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (!c || !m) return TGSIM_EINVAL;
  c->spec.valid = false;  // staged arrays change: no speculative storm round
  if (c->in_window) return fail(c, TGSIM_ESTATE, "enqueue inside a window");
  if (int rc = react_owed(c)) return rc;
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  if (!c->staged_dev && (uint64_t)c->n_staged + n > c->d.cap_msgs)
    return fail(c, TGSIM_ECAPACITY, "staged-message capacity");
  if (n > c->d.cap_msgs) return fail(c, TGSIM_ECAPACITY, "staged-message capacity");
  int rc = validate_msgs(c, m, n);
  if (rc) return rc;
  if (!n) return TGSIM_OK;
  for (size_t i = 0; i < n; ++i) {  // per-sender counts for the queue-limit test, latest send time
    const uint32_t l = m->src[i] - c->lo;
    if (c->hcnt[l]++ == 0) c->hcnt_touched.push_back(l);
    c->win_m_host = std::max(c->win_m_host, c->hcnt[l]);
    c->max_tsend_h = std::max(c->max_tsend_h, m->t_send[i]);
  }
  Dev& d = c->d;
  uint8_t* pin = nullptr;  // t | src | dst | seq | size
  rc = pin_acquire(c, c->pin_msgs, n * 24, &pin);
  if (rc) return rc;
  memcpy(pin, m->t_send, n * 8);
  memcpy(pin + n * 8, m->src, n * 4);
  memcpy(pin + n * 12, m->dst, n * 4);
  memcpy(pin + n * 16, m->seq, n * 4);
  memcpy(pin + n * 20, m->size, n * 4);
  if (c->staged_dev) {  // behind the device-side count: via scratch, then appended on the device
    if (n > c->app_cap) {
      HIPCK(c, hipStreamSynchronize(d.stream), "sync");
      dfree(c, c->app);
      c->app = nullptr;
      const size_t cap = std::max<size_t>(n, 2 * c->app_cap);
      if (dalloc(c, &c->app, cap * 24)) return TGSIM_ENOMEM;
      c->app_cap = cap;
    }
    HIPCK(c, hipMemcpyAsync(c->app, pin, n * 24, hipMemcpyHostToDevice, d.stream), "enqueue");
    const uint32_t* a32 = reinterpret_cast<const uint32_t*>(c->app + n * 8);
    HIPCK(c, launch_append(d, a32, a32 + n, a32 + 2 * n, a32 + 3 * n, reinterpret_cast<const int64_t*>(c->app),
                           (uint32_t)n), "append");
    return pin_issued(c, c->pin_msgs);
  }
  const size_t o = c->n_staged;
  HIPCK(c, hipMemcpyAsync(d.m_t + o, pin, n * 8, hipMemcpyHostToDevice, d.stream), "enqueue");
  HIPCK(c, hipMemcpyAsync(d.m_src + o, pin + n * 8, n * 4, hipMemcpyHostToDevice, d.stream), "enqueue");
  HIPCK(c, hipMemcpyAsync(d.m_dst + o, pin + n * 12, n * 4, hipMemcpyHostToDevice, d.stream), "enqueue");
  HIPCK(c, hipMemcpyAsync(d.m_seq + o, pin + n * 16, n * 4, hipMemcpyHostToDevice, d.stream), "enqueue");
  HIPCK(c, hipMemcpyAsync(d.m_size + o, pin + n * 20, n * 4, hipMemcpyHostToDevice, d.stream), "enqueue");
  c->n_staged += (uint32_t)n;
  return pin_issued(c, c->pin_msgs);
}

static int tgsim_enqueue_device_body(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n);
extern "C" int tgsim_enqueue_device(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  return abi_guard(c, [&] { return tgsim_enqueue_device_body(c, m, n); });
}
static int tgsim_enqueue_device_body(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (!c || !m) return TGSIM_EINVAL;
  c->spec.valid = false;  // staged arrays change: no speculative storm round
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode: traffic goes through tgsim_tcp_send");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "enqueue inside a window");
  if (int rc = react_owed(c)) return rc;
  if ((c->staged_dev ? 0 : (uint64_t)c->n_staged) + n > c->d.cap_msgs)
    return fail(c, TGSIM_ECAPACITY, "staged-message capacity");
  if (!n) return TGSIM_OK;
  c->win_m_extra += n;  // any one sender may hold all of them (queue-limit test)
  Dev& d = c->d;
  if (c->staged_dev) {
    HIPCK(c, launch_append(d, m->src, m->dst, m->seq, m->size, m->t_send, (uint32_t)n), "append");
    return TGSIM_OK;
  }
  // the window's first staging, with no reactor that reads the staged arrays after the window (the
  // probes' and the storm plan's reactions do; TCP mode refused above): no copy (begin_common)
  if (c->n_staged == 0 && !c->probes && !c->storm_on) {
    c->ext.src = m->src; c->ext.dst = m->dst; c->ext.seq = m->seq; c->ext.size = m->size; c->ext.t = m->t_send;
    c->ext.n = (uint32_t)n;
    c->n_staged = (uint32_t)n;
    return TGSIM_OK;
  }
  // one copy kernel for the five arrays (five hipMemcpyAsync cost ~5 us of launch each: config 2's
  // million-message rounds spent 28 us per round staging)
  HIPCK(c, launch_stage(d, m->src, m->dst, m->seq, m->size, m->t_send, (uint32_t)n, c->n_staged), "enqueue");
  c->n_staged += (uint32_t)n;
  return TGSIM_OK;
}

// acks mode: packets a sender can stage per delivery it got last window - one ACK per data copy,
// and with connections up to two segments more per ACK (slow start: a flight slot and a cwnd step)
static uint32_t tcp_inbox_mult(const tgsim_ctx* c) { return c->td.n_conn ? 3u : 1u; }

// The lifetime bound (life_host, fl_npubs) counts host and device enqueues (win_m_host / win_m_extra,
// every window) and flood forwards (at most D per publication). Every other device reactor stages
// traffic it does not count; this is the one list of them, checked every window, that turns the
// bound off for good (a new reactor must be added here, or the queue-limit test would be
// skipped for its traffic - test_flood_queue_limit_reopens_* pins the flood side)
static bool uncounted_staging(const tgsim_ctx* c) {
  return c->tcp_on || c->probes || c->storm_on || c->win_inbox_max != 0;
}

// The window's queue-limit test. The kernels test every sender only when the host
// cannot prove that none can reach the limit: pend_bound (queued copies of any sender at this
// window's start) + mult * (the most messages one sender can have staged) <= TGSIM_NETEM_LIMIT.
static int plan_queue_limit(tgsim_ctx* c) {
  Dev& d = c->d;
  const uint64_t mult = c->any_dup ? 2 : 1;
  const uint64_t m_uniform = std::min<uint64_t>((uint64_t)c->win_m_host + c->win_m_extra, 0x7FFFFFFFull);
  const uint64_t m_max = m_uniform + (uint64_t)c->win_m_inbox * std::max<uint64_t>(c->fl_npubs, c->win_inbox_max);
  // zero-delay unshaped senders only: the window's own copies never count, and none of them stays
  // queued past its enqueue instant, so the bound does not grow either (Heavy::zd)
  const bool zd_only = c->all_zd && !c->tcp_on;
  bool gate = zd_only ? c->pend_bound >= TGSIM_NETEM_LIMIT : c->pend_bound + mult * m_max > TGSIM_NETEM_LIMIT;
  // inconclusive: refresh the bound with the exact maximum (one sync) - unless the window's own
  // staging bound already reaches the limit, when no refresh can close the gate
  c->life_host = std::min<uint64_t>(c->life_host + m_uniform, 1ull << 40);
  c->life_mult = std::max<uint64_t>(c->life_mult, mult);
  if (uncounted_staging(c)) c->life_ok = false;
  if (gate && c->life_ok && !zd_only &&
      c->life_mult * ((uint64_t)c->d.fl.D * c->fl_npubs + c->life_host) <= TGSIM_NETEM_LIMIT)
    gate = false;  // no sender can ever have queued and staged more than the limit
  if (gate && !c->pend_exact && (zd_only || mult * m_max <= TGSIM_NETEM_LIMIT)) {
    if (!c->pend_host &&
        hipHostMalloc((void**)&c->pend_host, kRadixBlocks * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
      return fail(c, TGSIM_ENOMEM, "pinned pend maxima");
    HIPCK(c, launch_pend_max(d, c->tcp_on ? c->td.pend_by + c->lo : nullptr, c->tcp_on && c->tcp.acks ? tcp_inbox_mult(c) : 0u,
                             (uint32_t)mult, c->pend_host), "pend max");
    HIPCK(c, sync_scalars(d), "sync");
    uint32_t mx = 0;
    for (int b = 0; b < kRadixBlocks; ++b) mx = std::max(mx, c->pend_host[b]);
    c->pend_bound = mx;
    c->pend_exact = true;
    gate = zd_only ? c->pend_bound >= TGSIM_NETEM_LIMIT : c->pend_bound + mult * m_max > TGSIM_NETEM_LIMIT;
  }
  d.heavy = Heavy{};
  if (gate) {
    if (!d.H) {  // first window that needs the H list: room for every due record of a window
      HIPCK(c, hipStreamSynchronize(d.stream), "sync");
      const size_t cap = (size_t)kNSub * d.subcap;
      if (dalloc(c, &d.H, cap) || dalloc(c, &d.hkeys, cap) || dalloc(c, &d.hvals, cap) || dalloc(c, &d.hkeys1, cap) ||
          dalloc(c, &d.hvals1, cap) || dalloc(c, &d.hoff, (size_t)d.nloc + 2) ||
          dalloc(c, &d.hhist, (size_t)kMaxBins * kRadixBlocks) || dalloc(c, &d.hhistx, (size_t)kMaxBins * kRadixBlocks) ||
          dalloc(c, &d.htot, kMaxBins) || dalloc(c, &d.hbstart, kMaxBins + 1))
        return TGSIM_ENOMEM;
      d.h_cap = (uint32_t)cap;
    }
    d.heavy.pend = pend_ref(d);
    d.heavy.zd = d.zd;
    d.heavy.inbox = c->win_m_inbox ? d.inbox : nullptr;
    d.heavy.retx = c->tcp_on ? c->td.pend_by + c->lo : nullptr;  // [N] by instance: the local senders' part
    d.heavy.m_uniform = (uint32_t)m_uniform;
    d.heavy.m_inbox = c->win_m_inbox;
    if (c->tcp_on && c->tcp.acks) {  // ACKs: at most one per delivery the sender got last window
      d.heavy.inbox = d.inbox;
      d.heavy.m_inbox = tcp_inbox_mult(c);
    }
    d.heavy.mult = (uint32_t)mult;
  }
  if (!zd_only) {
    c->pend_bound = std::min<uint64_t>(c->pend_bound + mult * m_max, 1ull << 62);
    c->pend_exact = m_max == 0;
  }
  for (uint32_t l : c->hcnt_touched) c->hcnt[l] = 0;
  c->hcnt_touched.clear();
  c->win_m_host = 0;
  c->win_m_extra = 0;
  c->win_m_inbox = 0;
  c->win_inbox_max = 0;
  c->max_tsend_h = INT64_MIN;
  return TGSIM_OK;
}

static int begin_common(tgsim_ctx* c) {
  c->spec.valid = false;  // a window runs before any storm round: the speculative one is stale
  int rc = upload_tables(c);
  if (rc) return rc;
  if (c->tcp_on) {
    if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tgsim_tcp_react after every window");
    if (c->tcp.acks) {
      // the last reaction's ACKs and the due timers join the staged packets behind the device-side
      // count; the window's new segments (all staged now) register one timer batch
      if (c->td.n_conn) c->tcp_seg_batched = c->tsg_n;  // connection segments' timers ride the pend lists
      const bool reg = c->tsg_n > c->tcp_seg_batched;
      HIPCK(c, launch_tcp_release_acks(c->d, c->td, c->tcp_cur, c->staged_dev, c->n_staged, c->tcp_nb, reg,
                                       (uint32_t)c->tcp_seg_batched, (uint32_t)c->tsg_n), "tcp release");
      c->tcp_fill = reg ? c->tcp_nb : ~0u;
      if (reg) c->tcp_nb++;
      c->tcp_seg_batched = c->tsg_n;
      // a timer can re-queue a segment that sits in no count (delivered, ACK outstanding): the
      // queue-limit bound is refreshed exactly every window
      c->pend_bound = 1ull << 62;
      c->pend_exact = false;
    } else {
      // due retransmissions join the staged packets behind the device-side count (the pending count
      // is device-side too, and the queue-limit test reads the per-sender counts on the device)
      HIPCK(c, launch_tcp_release(c->d, c->td, c->tcp_cur, c->staged_dev, c->n_staged), "tcp release");
    }
    c->staged_dev = true;
    c->tcp_cur ^= 1u;
  }
  rc = plan_queue_limit(c);
  if (rc) return rc;
  Dev& d = c->d;
  // tgsim_enqueue_device's batch: the window reads the caller's arrays when the batch is all it
  // stages (the launches take the pointers now; the staged arrays are the library's again after
  // them), else the batch goes in front of what was staged after it
  const bool in_place = c->ext.n && c->n_staged == c->ext.n && !c->staged_dev;
  if (c->ext.n && !in_place)
    HIPCK(c, launch_stage(d, c->ext.src, c->ext.dst, c->ext.seq, c->ext.size, c->ext.t, c->ext.n, 0), "enqueue");
  uint32_t *own_src = d.m_src, *own_dst = d.m_dst, *own_seq = d.m_seq, *own_size = d.m_size;
  int64_t* own_t = d.m_t;
  if (in_place) {  // read only by the window's netem pass and its sequential lane
    d.m_src = const_cast<uint32_t*>(c->ext.src); d.m_dst = const_cast<uint32_t*>(c->ext.dst);
    d.m_seq = const_cast<uint32_t*>(c->ext.seq); d.m_size = const_cast<uint32_t*>(c->ext.size);
    d.m_t = const_cast<int64_t*>(c->ext.t);
  }
  const hipError_t we = window_begin(d, c->n_staged, c->staged_dev ? &c->d.sc->n_msgs_dev : nullptr);
  d.m_src = own_src; d.m_dst = own_dst; d.m_seq = own_seq; d.m_size = own_size; d.m_t = own_t;
  c->ext.n = 0;
  HIPCK(c, we, "window_begin");
  c->n_status_last = c->staged_dev ? kStatusOnDevice : c->n_staged;
  c->n_staged = 0;
  c->staged_dev = false;
  c->end_known = false;  // device-ended windows (barrier / device t_end); explicit ones set it after
  c->in_window = true;
  c->tcp_need_react = c->tcp_on;
  c->probe_need_react = c->probes;
  c->storm_need_react = c->storm_on;
  return TGSIM_OK;  // device-side errors surface at the next synchronisation
}

static int tgsim_advance_begin_body(tgsim_ctx* c, int64_t t_end);
extern "C" int tgsim_advance_begin(tgsim_ctx* c, int64_t t_end) {
  return abi_guard(c, [&] { return tgsim_advance_begin_body(c, t_end); });
}
static int tgsim_advance_begin_body(tgsim_ctx* c, int64_t t_end) {
  if (!c) return TGSIM_EINVAL;
  if (c->in_window) return fail(c, TGSIM_ESTATE, "window already open");
  if (int rc = react_owed(c)) return rc;
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  if (t_end < c->now) return fail(c, TGSIM_ECAUSALITY, "t_end before window start");
  // a host-staged message sent at or after t_end is refused before anything changes (the context
  // stays usable, as in the oracle); device-staged batches are checked on the device
  if (c->max_tsend_h >= t_end) return fail(c, TGSIM_ECAUSALITY, "a staged message is sent at/after t_end");
  HIPCK(c, flush_storm(c), "storm commit");
  HIPCK(c, launch_set_window(c->d, t_end), "set window");
  const int rc = begin_common(c);
  if (rc) return rc;
  c->end_known = true;  // begin_common cleared it
  c->end_h = t_end;
  return TGSIM_OK;
}

static int tgsim_exchange_buffers_body(tgsim_ctx* c, void** send, void** recv, size_t* bytes);
extern "C" int tgsim_exchange_buffers(tgsim_ctx* c, void** send, void** recv, size_t* bytes) {
  return abi_guard(c, [&] { return tgsim_exchange_buffers_body(c, send, recv, bytes); });
}
static int tgsim_exchange_buffers_body(tgsim_ctx* c, void** send, void** recv, size_t* bytes) {
  if (!c || !send || !recv || !bytes) return TGSIM_EINVAL;
  *send = c->d.xsend;
  *recv = c->d.xrecv;
  *bytes = (size_t)c->S * c->d.xcap * sizeof(tgsim_record);
  return TGSIM_OK;
}

static int tgsim_set_exchange_buffers_body(tgsim_ctx* c, void* send, void* recv, size_t bytes);
extern "C" int tgsim_set_exchange_buffers(tgsim_ctx* c, void* send, void* recv, size_t bytes) {
  return abi_guard(c, [&] { return tgsim_set_exchange_buffers_body(c, send, recv, bytes); });
}
static int tgsim_set_exchange_buffers_body(tgsim_ctx* c, void* send, void* recv, size_t bytes) {
  if (!c || !send || !recv) return TGSIM_EINVAL;
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  const size_t need = (size_t)c->S * c->d.xcap * sizeof(tgsim_record);
  if (bytes < need) return fail(c, TGSIM_ECAPACITY, "exchange buffers need %zu bytes", need);
  if ((uintptr_t)send % 16 || (uintptr_t)recv % 16) return fail(c, TGSIM_EINVAL, "exchange buffers must be 16-B aligned");
  c->d.xsend = static_cast<tgsim_record*>(send);
  c->d.xrecv = static_cast<tgsim_record*>(recv);
  return TGSIM_OK;
}

static int tgsim_advance_begin_device_body(tgsim_ctx* c, const int64_t* t_end_dev, int64_t offset_ns);
extern "C" int tgsim_advance_begin_device(tgsim_ctx* c, const int64_t* t_end_dev, int64_t offset_ns) {
  return abi_guard(c, [&] { return tgsim_advance_begin_device_body(c, t_end_dev, offset_ns); });
}
static int tgsim_advance_begin_device_body(tgsim_ctx* c, const int64_t* t_end_dev, int64_t offset_ns) {
  if (!c || !t_end_dev) return TGSIM_EINVAL;
  if (c->in_window) return fail(c, TGSIM_ESTATE, "window already open");
  if (int rc = react_owed(c)) return rc;
  HIPCK(c, flush_storm(c), "storm commit");
  HIPCK(c, launch_set_window_dev(c->d, t_end_dev, offset_ns), "set window");
  return begin_common(c);
}

static int tgsim_advance_end_body(tgsim_ctx* c);
extern "C" int tgsim_advance_end(tgsim_ctx* c) {
  return abi_guard(c, [&] { return tgsim_advance_end_body(c); });
}
static int tgsim_advance_end_body(tgsim_ctx* c) {
  if (!c) return TGSIM_EINVAL;
  if (!c->in_window) return fail(c, TGSIM_ESTATE, "no open window");
  {
    tgsim_ctx::StormSpec& sp = c->spec;
    sp.valid = false;
    // the next round is generated here only when nothing can read the staged arrays or the
    // signal partials in between: no deferred storm commit, no TCP / flood staging
    const bool spec = sp.hint && !c->storm_pending && !c->tcp_on && !c->staged_dev && c->n_staged == 0 &&
                      (uint64_t)c->nloc * 8 <= c->d.cap_msgs && c->nloc <= c->d.s_cap && sp.state < c->d.max_states &&
                      c->fl_off.empty();
    sp.hint = false;
    if (spec) {
      HIPCK(c, window_end_storm(c->d, sp.round, sp.size, sp.spread, &sp.parts), "window_end");
      sp.valid = true;
    } else {
      HIPCK(c, window_end(c->d), "window_end");
    }
  }
  c->in_window = false;
  // No host round trip: a host-given end is the new clock; a device-ended window's end (and any
  // device-side error) is read at the next sync.
  if (c->end_known) {
    c->horizon = c->now;
    c->now = c->end_h;
  } else {
    c->now_from_device = true;
  }
  return TGSIM_OK;
}

// ============================== cross-shard transport =======================================
// one exchange per window (the peer blocks travel whole: their capacity is the
// device-known bound, no count goes to the host), one MAX all-reduce per storm batch, an all-gather
// per host signal batch. RCCL is one implementation of the three operations (ncclSend / ncclRecv
// grouped, ncclAllReduce, ncclAllGather on the ctx stream); a caller's callbacks are another.

static int rccl_alltoall(void* user, const void* send, void* recv, size_t block, void* stream) {
  tgsim_ctx* c = static_cast<tgsim_ctx*>(user);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (ncclGroupStart() != ncclSuccess) return -1;
  for (uint32_t p = 0; p < c->S; ++p) {
    if (p == c->shard) continue;
    if (ncclSend(static_cast<const uint8_t*>(send) + p * block, block, ncclUint8, (int)p, c->comm, s) != ncclSuccess ||
        ncclRecv(static_cast<uint8_t*>(recv) + p * block, block, ncclUint8, (int)p, c->comm, s) != ncclSuccess) {
      (void)ncclGroupEnd();
      return -1;
    }
  }
  return ncclGroupEnd() == ncclSuccess ? 0 : -1;
}
static int rccl_allreduce_max(void* user, int64_t* buf, size_t n, void* stream) {
  tgsim_ctx* c = static_cast<tgsim_ctx*>(user);
  return ncclAllReduce(buf, buf, n, ncclInt64, ncclMax, c->comm, static_cast<hipStream_t>(stream)) == ncclSuccess ? 0 : -1;
}
static int rccl_allgather(void* user, const void* send, void* recv, size_t bytes, void* stream) {
  tgsim_ctx* c = static_cast<tgsim_ctx*>(user);
  return ncclAllGather(send, recv, bytes, ncclUint8, c->comm, static_cast<hipStream_t>(stream)) == ncclSuccess ? 0 : -1;
}

static int tgsim_comm_unique_id_body(uint8_t out[TGSIM_COMM_ID_BYTES]);
extern "C" int tgsim_comm_unique_id(uint8_t out[TGSIM_COMM_ID_BYTES]) {
  return abi_guard(nullptr, [&] { return tgsim_comm_unique_id_body(out); });
}
static int tgsim_comm_unique_id_body(uint8_t out[TGSIM_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == TGSIM_COMM_ID_BYTES, "RCCL unique id size");
  if (!out) return TGSIM_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return TGSIM_EHIP;
  memcpy(out, &id, sizeof(id));
  return TGSIM_OK;
}

static int tgsim_comm_init_body(tgsim_ctx* c, const uint8_t id[TGSIM_COMM_ID_BYTES], uint32_t nranks, uint32_t rank);
extern "C" int tgsim_comm_init(tgsim_ctx* c, const uint8_t id[TGSIM_COMM_ID_BYTES], uint32_t nranks, uint32_t rank) {
  return abi_guard(c, [&] { return tgsim_comm_init_body(c, id, nranks, rank); });
}
static int tgsim_comm_init_body(tgsim_ctx* c, const uint8_t id[TGSIM_COMM_ID_BYTES], uint32_t nranks, uint32_t rank) {
  if (!c || !id) return TGSIM_EINVAL;
  if (nranks != c->S || rank != c->shard) return fail(c, TGSIM_EINVAL, "communicator rank %u/%u != shard %u/%u", rank, nranks, c->shard, c->S);
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  HIPCK(c, hipSetDevice((int)c->cfg.device), "device");
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
  const ncclResult_t r = ncclCommInitRank(&c->comm, (int)nranks, uid, (int)rank);
  if (r != ncclSuccess) { c->comm = nullptr; return fail(c, TGSIM_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r)); }
  c->tr.user = c;
  c->tr.alltoall = rccl_alltoall;
  c->tr.allreduce_max_i64 = rccl_allreduce_max;
  c->tr.allgather = rccl_allgather;
  c->tr.abort = nullptr;  // shard_failed aborts the communicator itself
  c->has_tr = true;
  c->tr_aborted = false;
  return TGSIM_OK;
}

static int tgsim_set_transport_body(tgsim_ctx* c, const tgsim_transport* t);
extern "C" int tgsim_set_transport(tgsim_ctx* c, const tgsim_transport* t) {
  return abi_guard(c, [&] { return tgsim_set_transport_body(c, t); });
}
static int tgsim_set_transport_body(tgsim_ctx* c, const tgsim_transport* t) {
  if (!c) return TGSIM_EINVAL;
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (t && (!t->alltoall || !t->allreduce_max_i64 || !t->allgather)) return fail(c, TGSIM_EINVAL, "incomplete transport");
  if (c->comm) { (void)ncclCommDestroy(c->comm); c->comm = nullptr; }
  c->has_tr = t != nullptr;
  c->tr = t ? *t : tgsim_transport{};
  c->tr_aborted = false;
  return TGSIM_OK;
}

// The window's exchange (between begin and end): the peer blocks, whole.
static int exchange_window(tgsim_ctx* c) {
  const size_t block = (size_t)c->d.xcap * sizeof(tgsim_record);
  ProfScope ps_(c->d, KID_EXCHANGE);  // the window's peer blocks (HIP events on the ctx stream)
  if (c->tr.alltoall(c->tr.user, c->d.xsend, c->d.xrecv, block, c->d.stream) != 0)
    return fail(c, TGSIM_EHIP, "transport all-to-all failed");
  return TGSIM_OK;
}

static int need_transport(tgsim_ctx* c) {
  if (c->S != 1 && !c->has_tr)
    return fail(c, TGSIM_ESTATE, c->tr_aborted ? "the transport was aborted (a shard failed)"
                                               : "a sharded context needs a transport (tgsim_comm_init / tgsim_set_transport) or begin/end");
  return TGSIM_OK;
}

// A shard whose sharded call fails must not leave the others waiting in a collective it will never
// join: the caller's transport is told (tgsim_transport.abort) and the native
// communicator aborted, so the peers' pending and later collectives fail; sharded calls are then
// refused here.
static int shard_failed(tgsim_ctx* c, int rc) {
  if (rc == TGSIM_OK || c == nullptr || c->S == 1 || !c->has_tr) return rc;
  if (c->comm) {
    (void)ncclCommAbort(c->comm);
    c->comm = nullptr;
  } else if (c->tr.abort) {
    c->tr.abort(c->tr.user);
  }
  c->has_tr = false;
  c->tr_aborted = true;
  c->in_window = false;
  return rc;
}

static int tgsim_comm_abort_body(tgsim_ctx* c);
extern "C" int tgsim_comm_abort(tgsim_ctx* c) {
  return abi_guard(c, [&] { return tgsim_comm_abort_body(c); });
}
static int tgsim_comm_abort_body(tgsim_ctx* c) {
  if (!c) return TGSIM_EINVAL;
  (void)shard_failed(c, TGSIM_ESTATE);
  return TGSIM_OK;
}


static int tgsim_advance_body(tgsim_ctx* c, int64_t t_end);
extern "C" int tgsim_advance(tgsim_ctx* c, int64_t t_end) {
  return abi_guard(c, [&] { return shard_failed(c, tgsim_advance_body(c, t_end)); });
}
static int tgsim_advance_body(tgsim_ctx* c, int64_t t_end) {
  if (!c) return TGSIM_EINVAL;
  int rc = need_transport(c);
  if (rc) return rc;
  rc = tgsim_advance_begin(c, t_end);
  if (rc) return rc;
  if (c->S != 1) {
    rc = exchange_window(c);
    if (rc) return rc;
  }
  rc = tgsim_advance_end(c);
  if (rc) return rc;
  return sync_and_check(c);  // the host-driven API reports the window's errors here
}

static int tgsim_advance_async_body(tgsim_ctx* c, int64_t t_end);
extern "C" int tgsim_advance_async(tgsim_ctx* c, int64_t t_end) {
  return abi_guard(c, [&] { return shard_failed(c, tgsim_advance_async_body(c, t_end)); });
}
static int tgsim_advance_async_body(tgsim_ctx* c, int64_t t_end) {
  if (!c) return TGSIM_EINVAL;
  int rc = need_transport(c);
  if (rc) return rc;
  rc = tgsim_advance_begin(c, t_end);
  if (rc) return rc;
  if (c->S != 1) {
    rc = exchange_window(c);
    if (rc) return rc;
  }
  return tgsim_advance_end(c);
}

static int tgsim_advance_to_barrier_body(tgsim_ctx* c, uint32_t waiter, int64_t offset_ns);
extern "C" int tgsim_advance_to_barrier(tgsim_ctx* c, uint32_t waiter, int64_t offset_ns) {
  return abi_guard(c, [&] { return shard_failed(c, tgsim_advance_to_barrier_body(c, waiter, offset_ns)); });
}
static int tgsim_advance_to_barrier_body(tgsim_ctx* c, uint32_t waiter, int64_t offset_ns) {
  if (!c) return TGSIM_EINVAL;
  int rc0 = need_transport(c);
  if (rc0) return rc0;
  if (c->in_window) return fail(c, TGSIM_ESTATE, "window already open");
  if (waiter >= c->n_waiters) return fail(c, TGSIM_EINVAL, "bad waiter");
  if (int rc = react_owed(c)) return rc;
  if (c->storm_pending) {  // commit + barrier registration + window start: one launch
    c->storm_pending = false;
    const bool add = c->storm_add;
    c->storm_add = false;
    HIPCK(c, launch_set_window_barrier_commit(c->d, waiter, offset_ns, c->storm_parts, c->storm_n, c->storm_state,
                                              add ? c->storm_nw : c->n_waiters, add, c->add_state, c->add_target,
                                              c->add_twait), "set window");
  } else {
    HIPCK(c, launch_set_window_barrier(c->d, waiter, offset_ns), "set window");
  }
  int rc = begin_common(c);
  if (rc) return rc;
  if (c->S != 1) {
    rc = exchange_window(c);
    if (rc) return rc;
  }
  return tgsim_advance_end(c);
}

static int tgsim_delivery_count_body(tgsim_ctx* c, size_t* n);
extern "C" int tgsim_delivery_count(tgsim_ctx* c, size_t* n) {
  return abi_guard(c, [&] { return tgsim_delivery_count_body(c, n); });
}
static int tgsim_delivery_count_body(tgsim_ctx* c, size_t* n) {
  if (!c || !n) return TGSIM_EINVAL;
  int rc = sync_and_check(c);
  *n = c->d.h_sc->n_out;
  return rc;
}

static int tgsim_copy_deliveries_body(tgsim_ctx* c, tgsim_delivery_soa* o, size_t cap, size_t* n);
extern "C" int tgsim_copy_deliveries(tgsim_ctx* c, tgsim_delivery_soa* o, size_t cap, size_t* n) {
  return abi_guard(c, [&] { return tgsim_copy_deliveries_body(c, o, cap, n); });
}
static int tgsim_copy_deliveries_body(tgsim_ctx* c, tgsim_delivery_soa* o, size_t cap, size_t* n) {
  if (!c || !o || !n) return TGSIM_EINVAL;
  int rc = sync_and_check(c);
  if (rc) return rc;
  const size_t k = c->d.h_sc->n_out;
  *n = k;
  if (k > cap) return fail(c, TGSIM_ECAPACITY, "output capacity %zu < %zu deliveries", cap, k);
  if (!k) return TGSIM_OK;
  Dev& d = c->d;
  HIPCK(c, hipMemcpy(o->t_deliver, d.o_t, k * 8, hipMemcpyDeviceToHost), "copy");
  HIPCK(c, hipMemcpy(o->src, d.o_src, k * 4, hipMemcpyDeviceToHost), "copy");
  HIPCK(c, hipMemcpy(o->dst, d.o_dst, k * 4, hipMemcpyDeviceToHost), "copy");
  HIPCK(c, hipMemcpy(o->seq, d.o_seq, k * 4, hipMemcpyDeviceToHost), "copy");
  HIPCK(c, hipMemcpy(o->size, d.o_size, k * 4, hipMemcpyDeviceToHost), "copy");
  HIPCK(c, hipMemcpy(o->flags, d.o_flags, k * 4, hipMemcpyDeviceToHost), "copy");
  HIPCK(c, hipMemcpy(o->corrupt_off, d.o_coff, k * 4, hipMemcpyDeviceToHost), "copy");
  return TGSIM_OK;
}

static int tgsim_copy_inbox_offsets_body(tgsim_ctx* c, uint32_t* out, size_t cap);
extern "C" int tgsim_copy_inbox_offsets(tgsim_ctx* c, uint32_t* out, size_t cap) {
  return abi_guard(c, [&] { return tgsim_copy_inbox_offsets_body(c, out, cap); });
}
static int tgsim_copy_inbox_offsets_body(tgsim_ctx* c, uint32_t* out, size_t cap) {
  if (!c || !out) return TGSIM_EINVAL;
  if (cap < (size_t)c->nloc + 1) return fail(c, TGSIM_ECAPACITY, "inbox capacity");
  int rc = sync_and_check(c);
  if (rc) return rc;
  HIPCK(c, hipMemcpy(out, c->d.inbox, ((size_t)c->nloc + 1) * 4, hipMemcpyDeviceToHost), "copy");
  return TGSIM_OK;
}

static int tgsim_copy_status_body(tgsim_ctx* c, uint8_t* out, size_t cap, size_t* n);
extern "C" int tgsim_copy_status(tgsim_ctx* c, uint8_t* out, size_t cap, size_t* n) {
  return abi_guard(c, [&] { return tgsim_copy_status_body(c, out, cap, n); });
}
static int tgsim_copy_status_body(tgsim_ctx* c, uint8_t* out, size_t cap, size_t* n) {
  if (!c || !n) return TGSIM_EINVAL;
  int rc = sync_and_check(c);
  if (rc) return rc;
  const uint32_t k = c->n_status_last == kStatusOnDevice ? c->d.h_sc->n_msgs_last : c->n_status_last;
  *n = k;
  if (k > cap) return fail(c, TGSIM_ECAPACITY, "status capacity");
  if (k) HIPCK(c, hipMemcpy(out, c->d.status, k, hipMemcpyDeviceToHost), "copy");
  return TGSIM_OK;
}

static int tgsim_deliveries_device_body(tgsim_ctx* c, tgsim_delivery_soa* o);
extern "C" int tgsim_deliveries_device(tgsim_ctx* c, tgsim_delivery_soa* o) {
  return abi_guard(c, [&] { return tgsim_deliveries_device_body(c, o); });
}
static int tgsim_deliveries_device_body(tgsim_ctx* c, tgsim_delivery_soa* o) {
  if (!c || !o) return TGSIM_EINVAL;
  Dev& d = c->d;
  o->t_deliver = d.o_t; o->src = d.o_src; o->dst = d.o_dst; o->seq = d.o_seq; o->size = d.o_size;
  o->flags = d.o_flags; o->corrupt_off = d.o_coff;
  return TGSIM_OK;
}

// ============================== sync service =================================================

static int signal_local(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t, size_t n,
                        uint32_t* seq_out);

// A sharded batch over a transport: every shard's signals, gathered in shard order (sizes first,
// then the records padded to the largest batch), processed whole on every shard; seq_out gets the
// sequence numbers of this shard's own signals. Every decision below depends on gathered data
// only, so the shards agree on it (a refusal is collective too).
static int signal_gathered(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t, size_t n,
                           uint32_t* seq_out) {
  struct Rec { uint32_t state, inst; int64_t t; };
  static_assert(sizeof(Rec) == 16, "gather record");
  Dev& d = c->d;
  const uint32_t S = c->S;
  auto room = [&](size_t words) -> int {
    if (words <= c->gather_cap) return TGSIM_OK;
    HIPCK(c, hipStreamSynchronize(d.stream), "sync");
    dfree(c, c->d_gather);
    c->d_gather = nullptr;
    const size_t cap = std::max(words, 2 * c->gather_cap);
    if (dalloc(c, &c->d_gather, cap)) return TGSIM_ENOMEM;
    c->gather_cap = cap;
    return TGSIM_OK;
  };
  int rc = room(1 + S);
  if (rc) return rc;
  const uint64_t n64 = n;
  HIPCK(c, hipMemcpyAsync(c->d_gather, &n64, 8, hipMemcpyHostToDevice, d.stream), "gather");
  if (c->tr.allgather(c->tr.user, c->d_gather, c->d_gather + 1, 8, d.stream) != 0)
    return fail(c, TGSIM_EHIP, "transport all-gather failed");
  std::vector<uint64_t> sizes(S);
  HIPCK(c, hipMemcpyAsync(sizes.data(), c->d_gather + 1, 8 * (size_t)S, hipMemcpyDeviceToHost, d.stream), "gather");
  HIPCK(c, hipStreamSynchronize(d.stream), "gather");
  uint64_t maxn = 0, total = 0, mine = 0;
  for (uint32_t k = 0; k < S; ++k) {
    if (k == c->shard) mine = total;
    maxn = std::max(maxn, sizes[k]);
    total += sizes[k];
  }
  if (sizes[c->shard] != n64) return fail(c, TGSIM_EHIP, "transport all-gather returned a wrong size");
  if (total > c->d.s_cap) return fail(c, TGSIM_ECAPACITY, "gathered signal batch larger than %u", c->d.s_cap);
  if (total == 0) return signal_local(c, nullptr, nullptr, nullptr, 0, nullptr);
  rc = room(2 * maxn * (1 + (size_t)S));
  if (rc) return rc;
  std::vector<Rec> loc(maxn, Rec{0, 0, 0});
  for (size_t i = 0; i < n; ++i) loc[i] = Rec{states[i], inst[i], t[i]};
  uint64_t* send = c->d_gather;
  uint64_t* recv = c->d_gather + 2 * maxn;
  HIPCK(c, hipMemcpyAsync(send, loc.data(), maxn * sizeof(Rec), hipMemcpyHostToDevice, d.stream), "gather");
  if (c->tr.allgather(c->tr.user, send, recv, maxn * sizeof(Rec), d.stream) != 0)
    return fail(c, TGSIM_EHIP, "transport all-gather failed");
  std::vector<Rec> all(maxn * S);
  HIPCK(c, hipMemcpyAsync(all.data(), recv, all.size() * sizeof(Rec), hipMemcpyDeviceToHost, d.stream), "gather");
  HIPCK(c, hipStreamSynchronize(d.stream), "gather");
  std::vector<uint32_t> gs(total), gi(total), gq(total);
  std::vector<int64_t> gt(total);
  size_t j = 0;
  for (uint32_t k = 0; k < S; ++k)
    for (uint64_t i = 0; i < sizes[k]; ++i, ++j) {
      const Rec& r = all[(size_t)k * maxn + i];
      gs[j] = r.state; gi[j] = r.inst; gt[j] = r.t;
    }
  rc = signal_local(c, gs.data(), gi.data(), gt.data(), total, gq.data());
  if (rc) return rc;
  if (seq_out && n) memcpy(seq_out, gq.data() + mine, n * sizeof(uint32_t));
  return TGSIM_OK;
}

static int tgsim_sync_signal_body(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                                 size_t n, uint32_t* seq_out);
extern "C" int tgsim_sync_signal(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                                 size_t n, uint32_t* seq_out) {
  return abi_guard(c, [&] { return shard_failed(c, tgsim_sync_signal_body(c, states, inst, t, n, seq_out)); });
}
static int tgsim_sync_signal_body(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                                 size_t n, uint32_t* seq_out) {
  if (!c || (n && (!states || !inst || !t))) return TGSIM_EINVAL;
  c->spec.valid = false;  // signal partials change: no speculative storm round
  if (c->in_window) return fail(c, TGSIM_ESTATE, "signal inside a window");
  if (c->S != 1 && c->has_tr && !c->replicated_batch) return signal_gathered(c, states, inst, t, n, seq_out);
  return signal_local(c, states, inst, t, n, seq_out);
}

static int signal_submit(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t, size_t n,
                         uint32_t* seq_out);
static int signal_local(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t, size_t n,
                        uint32_t* seq_out) {
  if (c->in_window) return fail(c, TGSIM_ESTATE, "signal inside a window");
  if (c->sig_log_used + n > c->d.max_signals) return fail(c, TGSIM_ECAPACITY, "signal log full");
  if (c->st_last_h.size() < c->d.max_states) c->st_last_h.resize(c->d.max_states, INT64_MIN);
  for (size_t i = 0; i < n; ++i) {
    if (states[i] >= c->d.max_states) return fail(c, TGSIM_EINVAL, "state id %u >= max_states", states[i]);
    if (t[i] < 0) return fail(c, TGSIM_ECAUSALITY, "negative signal time");
    if (t[i] < c->st_last_h[states[i]]) return fail(c, TGSIM_ECAUSALITY, "signal %zu goes back in time", i);
  }
  for (size_t i = 0; i < n; ++i) c->st_last_h[states[i]] = std::max(c->st_last_h[states[i]], t[i]);
  if (n <= c->d.s_cap) return signal_submit(c, states, inst, t, n, seq_out);
  // A batch larger than the device batch (the storm's N * outgoing dial signals): in (t, instance)
  // order - the order sequence numbers follow inside a batch - cut into consecutive device batches,
  // so every state's signals get the numbers one batch would give them, and no cut goes back in time.
  alloc_point(c);
  std::vector<uint32_t> ord(n);
  for (size_t i = 0; i < n; ++i) ord[i] = (uint32_t)i;
  std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
    return t[a] != t[b] ? t[a] < t[b] : inst[a] < inst[b];
  });
  const size_t cap = c->d.s_cap;
  std::vector<uint32_t> bs(cap), bi(cap), bq(cap);
  std::vector<int64_t> bt(cap);
  for (size_t a = 0; a < n; a += cap) {
    const size_t m = std::min(cap, n - a);
    for (size_t j = 0; j < m; ++j) {
      const uint32_t i = ord[a + j];
      bs[j] = states[i]; bi[j] = inst[i]; bt[j] = t[i];
    }
    const int rc = signal_submit(c, bs.data(), bi.data(), bt.data(), m, bq.data());
    if (rc) return rc;
    if (seq_out)
      for (size_t j = 0; j < m; ++j) seq_out[ord[a + j]] = bq[j];
  }
  return TGSIM_OK;
}

// One device batch (n <= s_cap), validated by signal_local.
static int signal_submit(tgsim_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t, size_t n,
                         uint32_t* seq_out) {
  Dev& d = c->d;
  HIPCK(c, flush_storm(c), "storm commit");
  uint32_t kmin = UINT32_MAX, kmax = 0;
  for (size_t i = 0; i < n; ++i) { kmin = std::min(kmin, states[i]); kmax = std::max(kmax, states[i]); }
  if (n) {
    HIPCK(c, hipMemcpyAsync(d.s_state, states, n * 4, hipMemcpyHostToDevice, d.stream), "signal");
    HIPCK(c, hipMemcpyAsync(d.s_inst, inst, n * 4, hipMemcpyHostToDevice, d.stream), "signal");
    HIPCK(c, hipMemcpyAsync(d.s_t, t, n * 8, hipMemcpyHostToDevice, d.stream), "signal");
  }
  const uint64_t base = c->sig_log_used;
  HIPCK(c, signal_batch(d, (uint32_t)n, n ? kmin : 0, n ? kmax : 0, base, c->n_waiters, false), "signal batch");
  c->sig_log_used += n;
  if (seq_out && n) HIPCK(c, hipMemcpyAsync(seq_out, d.s_seq, n * 4, hipMemcpyDeviceToHost, d.stream), "seq");
  return sync_and_check(c);
}

static int tgsim_sync_barrier_body(tgsim_ctx* c, uint32_t state, uint32_t target, int64_t t_wait, uint32_t* w);
extern "C" int tgsim_sync_barrier(tgsim_ctx* c, uint32_t state, uint32_t target, int64_t t_wait, uint32_t* w) {
  return abi_guard(c, [&] { return tgsim_sync_barrier_body(c, state, target, t_wait, w); });
}
static int tgsim_sync_barrier_body(tgsim_ctx* c, uint32_t state, uint32_t target, int64_t t_wait, uint32_t* w) {
  if (!c || !w) return TGSIM_EINVAL;
  if (state >= c->d.max_states) return fail(c, TGSIM_EINVAL, "state id %u >= max_states", state);
  if (c->n_waiters >= c->d.max_waiters) return fail(c, TGSIM_ECAPACITY, "too many barrier waiters");
  Dev& d = c->d;
  const uint32_t i = c->n_waiters;
  if (c->storm_pending && !c->storm_add) {
    // the storm batch's commit and this registration wait for the next launch (normally the window
    // start that waits on this barrier: tgsim_advance_to_barrier)
    c->storm_add = true;
    c->storm_nw = i;
    c->add_state = state;
    c->add_target = target;
    c->add_twait = t_wait;
  } else {
    HIPCK(c, flush_storm(c), "storm commit");
    HIPCK(c, add_waiter(d, i, state, target, t_wait), "barrier");
  }
  c->n_waiters++;
  *w = i;  // the new waiter is resolved now; the others can only move when signals arrive
  return TGSIM_OK;
}

static int tgsim_sync_poll_body(tgsim_ctx* c, uint32_t w, int64_t* rel);
extern "C" int tgsim_sync_poll(tgsim_ctx* c, uint32_t w, int64_t* rel) {
  return abi_guard(c, [&] { return tgsim_sync_poll_body(c, w, rel); });
}
static int tgsim_sync_poll_body(tgsim_ctx* c, uint32_t w, int64_t* rel) {
  if (!c || !rel) return TGSIM_EINVAL;
  if (w >= c->n_waiters) return fail(c, TGSIM_EINVAL, "bad waiter");
  HIPCK(c, flush_storm(c), "storm commit");
  HIPCK(c, hipMemcpyAsync(rel, c->d.w_release + w, 8, hipMemcpyDeviceToHost, c->d.stream), "poll");
  return sync_and_check(c);
}

static int tgsim_sync_count_body(tgsim_ctx* c, uint32_t state, uint32_t* count);
extern "C" int tgsim_sync_count(tgsim_ctx* c, uint32_t state, uint32_t* count) {
  return abi_guard(c, [&] { return tgsim_sync_count_body(c, state, count); });
}
static int tgsim_sync_count_body(tgsim_ctx* c, uint32_t state, uint32_t* count) {
  if (!c || !count) return TGSIM_EINVAL;
  if (state >= c->d.max_states) return fail(c, TGSIM_EINVAL, "bad state");
  HIPCK(c, flush_storm(c), "storm commit");
  HIPCK(c, hipMemcpyAsync(count, c->d.st_count + state, 4, hipMemcpyDeviceToHost, c->d.stream), "count");
  return sync_and_check(c);
}

// ============================== workloads ====================================================

static int gen_storm_impl(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size, int64_t spread_ns,
                          uint32_t state);
static int tgsim_gen_storm_round_body(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                                     int64_t spread_ns, uint32_t state);
extern "C" int tgsim_gen_storm_round(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                                     int64_t spread_ns, uint32_t state) {
  return abi_guard(c, [&] { return shard_failed(c, tgsim_gen_storm_round_body(c, round, t0, fanout, size, spread_ns, state)); });
}
static int tgsim_gen_storm_round_body(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                                     int64_t spread_ns, uint32_t state) {
  if (c && c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode: tgsim_tcp_gen_storm_round");
  if (c) if (int rc = react_owed(c)) return rc;
  return gen_storm_impl(c, round, t0, fanout, size, spread_ns, state);
}

static int gen_storm_impl(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size, int64_t spread_ns,
                          uint32_t state) {
  if (!c) return TGSIM_EINVAL;
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (fanout == 0 || fanout >= c->N || fanout > 32) return fail(c, TGSIM_EINVAL, "bad fanout");
  if (size >= 0x80000000u || spread_ns < 0) return fail(c, TGSIM_EINVAL, "bad size/spread");
  if (state >= c->d.max_states) return fail(c, TGSIM_EINVAL, "bad state");
  if (c->staged_dev) return fail(c, TGSIM_ENOTSUP, "a storm round after a flood reaction in the same window");
  if (t0 != TGSIM_T_NOW) {
    if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
    if (t0 < c->now) return fail(c, TGSIM_ECAUSALITY, "t0 before window start");
  }
  const uint64_t n = (uint64_t)c->nloc * fanout;
  if (c->n_staged + n > c->d.cap_msgs) return fail(c, TGSIM_ECAPACITY, "staged-message capacity");
  if (c->nloc > c->d.s_cap) return fail(c, TGSIM_ECAPACITY, "signal batch capacity");
  HIPCK(c, flush_storm(c), "storm commit");
  uint32_t parts = 0;
  tgsim_ctx::StormSpec& sp = c->spec;
  if (sp.valid && c->n_staged == 0 && t0 == TGSIM_T_NOW && fanout == 8 && round == sp.round && size == sp.size &&
      spread_ns == sp.spread && state == sp.state) {
    parts = sp.parts;  // generated by the last window's final launch
  } else {
    HIPCK(c, launch_gen_storm(c->d, c->n_staged, round, t0, fanout, size, spread_ns, &parts), "gen storm");
  }
  sp.valid = false;
  // arm the next round's speculation (plain storm rounds at the device clock only; the TCP variant
  // rewrites the staged records after generation)
  sp.hint = !c->tcp_on && t0 == TGSIM_T_NOW && fanout == 8 && c->n_staged == 0 && round + 1u != 0u;
  sp.round = round + 1u; sp.size = size; sp.spread = spread_ns; sp.state = state + 1u;
  c->n_staged += (uint32_t)n;
  c->win_m_extra += fanout;
  if (c->S == 1) {
    // SignalAndWait(state, N) by every instance: the return values are unused by the plan, so the
    // batch is committed count-only (count, first/last time) - deferred to the next
    // sync-service call, so that the plan's barrier rides in the same launch
    c->storm_pending = true;
    c->storm_parts = parts;
    c->storm_state = state;
    c->storm_n = c->nloc;
  } else if (c->has_tr) {
    // every shard commits the whole batch: its first / last time MAX-reduced over the shards (the
    // count is n_instances: every instance signals), replicated sync state
    HIPCK(c, launch_storm_red(c->d, parts, c->d_red2), "storm reduce");
    {
      ProfScope ps_(c->d, KID_ALLREDUCE);  // the storm batch's SignalAndWait: one MAX all-reduce
      if (c->tr.allreduce_max_i64(c->tr.user, c->d_red2, 2, c->d.stream) != 0)
        return fail(c, TGSIM_EHIP, "transport all-reduce failed");
    }
    HIPCK(c, launch_storm_unpack(c->d, c->d_red2), "storm reduce");
    c->storm_pending = true;
    c->storm_parts = 1;
    c->storm_state = state;
    c->storm_n = c->N;
  } else {
    // sharded: the release time is the MAX over shards of the local latest signal (sig_red[3])
    HIPCK(c, launch_sig_commit(c->d, parts, false, c->nloc, state, 0, false, 0, 0, 0), "storm release");
  }
  return TGSIM_OK;
}

static int tgsim_storm_release_device_body(tgsim_ctx* c, int64_t* out);
extern "C" int tgsim_storm_release_device(tgsim_ctx* c, int64_t* out) {
  return abi_guard(c, [&] { return tgsim_storm_release_device_body(c, out); });
}
static int tgsim_storm_release_device_body(tgsim_ctx* c, int64_t* out) {
  if (!c || !out) return TGSIM_EINVAL;
  if (c->S == 1) return fail(c, TGSIM_ESTATE, "single-shard storms commit their signals: use a barrier");
  HIPCK(c, hipMemcpyAsync(out, c->d.sig_red + 3, sizeof(int64_t), hipMemcpyDeviceToDevice, c->d.stream), "release");
  return TGSIM_OK;
}

// ============================== flood workload (config 5) ===================================
// publications flood a fixed graph with first-receipt dedup. The oracle
// twin is oracle/tgsim_oracle.c tgo_flood_*; kernels in tgsim_flood.hip.

static int tgsim_flood_set_graph_body(tgsim_ctx* c, const uint32_t* off, const uint32_t* nbr, uint32_t max_pubs);
extern "C" int tgsim_flood_set_graph(tgsim_ctx* c, const uint32_t* off, const uint32_t* nbr, uint32_t max_pubs) {
  return abi_guard(c, [&] { return tgsim_flood_set_graph_body(c, off, nbr, max_pubs); });
}
static int tgsim_flood_set_graph_body(tgsim_ctx* c, const uint32_t* off, const uint32_t* nbr, uint32_t max_pubs) {
  if (!c || !off || (off[c->N] && !nbr) || max_pubs == 0) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  // a flood reaction reads deliveries as publications (seq / D): TCP packets (seq = segment << 4 |
  // attempt) would be forwarded as floods and corrupt the TCP state
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is on: flood workloads need message mode");
  if (c->probes) return fail(c, TGSIM_ESTATE, "probes are set up: floods need the deliveries to themselves");
  if (c->storm_on) return fail(c, TGSIM_ESTATE, "a storm reactor is set up: floods need the deliveries to themselves");
  uint32_t D = 1;
  for (uint32_t g = 0; g < c->N; ++g) {
    if (off[g + 1] < off[g]) return fail(c, TGSIM_EINVAL, "offsets not monotonic");
    const uint32_t len = off[g + 1] - off[g];
    if (len > 64) return fail(c, TGSIM_EINVAL, "degree %u > 64", len);
    D = std::max(D, len);
    for (uint32_t k = off[g]; k < off[g + 1]; ++k)
      if (nbr[k] >= c->N || nbr[k] == g) return fail(c, TGSIM_EINVAL, "bad neighbour of %u", g);
  }
  if ((uint64_t)max_pubs * D > 0x100000000ull) return fail(c, TGSIM_EINVAL, "max_pubs * degree > 2^32");
  // host rows first (the only host allocations): a failure here leaves the previous graph intact
  const uint32_t base = off[c->lo], m = off[c->hi] - base;
  alloc_point(c);
  std::vector<uint32_t> rows_off(c->nloc + 1), rows_nbr(nbr + base, nbr + base + m);
  for (uint32_t l = 0; l <= c->nloc; ++l) rows_off[l] = off[c->lo + l] - base;
  std::vector<uint8_t> pub_seen(max_pubs, 0);
  HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
  Flood& f = c->d.fl;
  dfree(c, f.off); dfree(c, f.nbr); dfree(c, f.seen);
  f.off = f.nbr = f.seen = nullptr;
  c->fl_off.swap(rows_off);
  c->fl_nbr.swap(rows_nbr);
  f.D = D; f.max_pubs = max_pubs; f.wpp = (c->nloc + 31) / 32;
  const size_t words = (size_t)max_pubs * f.wpp;
  if (dalloc(c, &f.off, c->nloc + 1) || dalloc(c, &f.nbr, std::max<size_t>(m, 1)) || dalloc(c, &f.seen, words))
    return TGSIM_ENOMEM;
  HIPCK(c, hipMemcpy(f.off, c->fl_off.data(), (c->nloc + 1) * 4, hipMemcpyHostToDevice), "graph");
  if (m) HIPCK(c, hipMemcpy(f.nbr, c->fl_nbr.data(), (size_t)m * 4, hipMemcpyHostToDevice), "graph");
  HIPCK(c, hipMemset(f.seen, 0, words * 4), "graph");
  if (!f.cnt) {  // reaction scratch for every delivery a window can hold
    const size_t cap = (size_t)kNSub * c->d.subcap;
    if (dalloc(c, &f.cnt, cap) || dalloc(c, &f.first, cap) || dalloc(c, &f.bsum, (size_t)kFloodBlocks))
      return TGSIM_ENOMEM;
    f.cap = cap;
  }
  // TGSIM_SIDE_INSERT=1: the wheel insert on a side stream beside the flood's reaction - measured
  // slower (config 5: 0.400 -> 0.447 ms per window), so off unless asked for
  const char* si = getenv("TGSIM_SIDE_INSERT");
  if (!c->d.side && si && *si == '1') {
    HIPCK(c, hipStreamCreateWithFlags(&c->d.side, hipStreamNonBlocking), "side stream");
    HIPCK(c, hipEventCreateWithFlags(&c->d.side_ev, hipEventDisableTiming), "side stream");
    HIPCK(c, hipEventCreateWithFlags(&c->d.main_ev, hipEventDisableTiming), "side stream");
  }
  c->fl_pub_seen.swap(pub_seen);
  if (c->fl_npubs) c->life_ok = false;  // the earlier graph's publications may still be queued
  c->fl_npubs = 0;
  uint64_t h = fnv1a(0xCBF29CE484222325ull, c->fl_off.data(), c->fl_off.size() * 4);
  h = fnv1a(h, c->fl_nbr.data(), c->fl_nbr.size() * 4);
  c->fl_hash = fnv1a(h, &max_pubs, 4) | 1u;  // nonzero: a graph is set
  return TGSIM_OK;
}

static int tgsim_flood_publish_body(tgsim_ctx* c, const uint32_t* inst, const uint32_t* pubs, const int64_t* t,
                                   size_t n, uint32_t size);
extern "C" int tgsim_flood_publish(tgsim_ctx* c, const uint32_t* inst, const uint32_t* pubs, const int64_t* t,
                                   size_t n, uint32_t size) {
  return abi_guard(c, [&] { return tgsim_flood_publish_body(c, inst, pubs, t, n, size); }, false);
}
static int tgsim_flood_publish_body(tgsim_ctx* c, const uint32_t* inst, const uint32_t* pubs, const int64_t* t,
                                   size_t n, uint32_t size) {
  if (!c) return TGSIM_EINVAL;
  c->spec.valid = false;
  Flood& f = c->d.fl;
  if (!f.off) return fail(c, TGSIM_ESTATE, "no flood graph");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (n && (!inst || !pubs || !t)) return fail(c, TGSIM_EINVAL, "bad arguments");
  for (size_t i = 0; i < n; ++i)
    if (inst[i] >= c->N || pubs[i] >= f.max_pubs) return fail(c, TGSIM_EINVAL, "bad publication %zu", i);
  for (size_t i = 0; i < n; ++i)  // every shard sees the whole batch: the count is global
    if (!c->fl_pub_seen[pubs[i]]) { c->fl_pub_seen[pubs[i]] = 1; ++c->fl_npubs; }
  std::vector<uint32_t> src, dst, seq, sz, pairs;
  std::vector<int64_t> ts;
  for (size_t i = 0; i < n; ++i) {
    if (!is_local(c, inst[i])) continue;
    const uint32_t l = inst[i] - c->lo;
    for (uint32_t k = c->fl_off[l]; k < c->fl_off[l + 1]; ++k) {
      src.push_back(inst[i]); dst.push_back(c->fl_nbr[k]); seq.push_back(pubs[i] * f.D + (k - c->fl_off[l]));
      sz.push_back(size); ts.push_back(t[i]);
    }
    pairs.push_back(l); pairs.push_back(pubs[i]);
  }
  tgsim_msg_soa m{src.data(), dst.data(), seq.data(), sz.data(), ts.data()};
  int rc = tgsim_enqueue_body(c, &m, src.size());  // (not the entry point: it would join the side stream)
  if (rc) return rc;
  const uint32_t np = (uint32_t)(pairs.size() / 2);
  if (!np) return TGSIM_OK;
  if (np > f.mark_cap) {
    dfree(c, f.mark);
    f.mark = nullptr;
    if (dalloc(c, &f.mark, 2 * (size_t)np)) return TGSIM_ENOMEM;
    f.mark_cap = np;
  }
  uint8_t* pin = nullptr;
  rc = pin_acquire(c, c->pin_marks, pairs.size() * 4, &pin);
  if (rc) return rc;
  memcpy(pin, pairs.data(), pairs.size() * 4);
  HIPCK(c, hipMemcpyAsync(f.mark, pin, pairs.size() * 4, hipMemcpyHostToDevice, c->d.stream), "publish");
  HIPCK(c, launch_flood_mark(c->d, np), "publish");
  return pin_issued(c, c->pin_marks);
}

static int tgsim_flood_react_body(tgsim_ctx* c, uint32_t size, size_t* n_fwd);
extern "C" int tgsim_flood_react(tgsim_ctx* c, uint32_t size, size_t* n_fwd) {
  return abi_guard(c, [&] { return tgsim_flood_react_body(c, size, n_fwd); }, false);
}
static int tgsim_flood_react_body(tgsim_ctx* c, uint32_t size, size_t* n_fwd) {
  if (!c) return TGSIM_EINVAL;
  c->spec.valid = false;
  if (n_fwd) *n_fwd = 0;
  Flood& f = c->d.fl;
  if (!f.off) return fail(c, TGSIM_ESTATE, "no flood graph");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is on: flood workloads need message mode");
  // asynchronous: the delivery count, the forwards and the new staged count stay on the device
  HIPCK(c, launch_flood_react(c->d, c->staged_dev, c->n_staged, size, c->horizon), "flood react");
  c->staged_dev = true;
  c->win_m_inbox = f.D > 1 ? f.D - 1 : 0;  // per delivery of the sender's last inbox run
  if (n_fwd) {  // the caller asked for the count: one synchronisation
    const int rc = sync_and_check(c);
    if (rc) return rc;
    *n_fwd = c->d.h_sc->fl_total;
  }
  return TGSIM_OK;
}

// ============================== sequential probes ===========================
// plans/splitbrain/main.go:153-175 (one httpclient.Get after another, Timeout: 1 minute). Kernels in
// tgsim_probe.hip, oracle twin tgo_probe_*.

static int tgsim_probe_setup_body(tgsim_ctx* c, const uint32_t* order, uint32_t n_order, const tgsim_probe_config* cfg);
extern "C" int tgsim_probe_setup(tgsim_ctx* c, const uint32_t* order, uint32_t n_order, const tgsim_probe_config* cfg) {
  return abi_guard(c, [&] { return tgsim_probe_setup_body(c, order, n_order, cfg); });
}
static int tgsim_probe_setup_body(tgsim_ctx* c, const uint32_t* order, uint32_t n_order, const tgsim_probe_config* cfg) {
  // positions < 2^24: the reaction packs (position, arrival) into one 64-bit key (tgsim_probe.hip)
  if (!c || !order || !cfg || n_order == 0 || n_order >= (1u << 24)) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (cfg->timeout_ns <= 0 || cfg->window_ns <= 0 || cfg->request_bytes >= 0x80000000u || cfg->reply_bytes >= 0x80000000u)
    return fail(c, TGSIM_EINVAL, "bad probe configuration");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (int rc = need_transport(c)) return rc;  // sharded: the notices and the proposal are collective
  if (c->N > 0x3FFFFFFFu) return fail(c, TGSIM_ENOTSUP, "too many instances for probe tags");
  if (c->tcp_on || !c->fl_off.empty()) return fail(c, TGSIM_ESTATE, "probes run in message mode, without a flood graph");
  if (c->storm_on) return fail(c, TGSIM_ESTATE, "a storm reactor is set up: it owns the deliveries");
  for (uint32_t j = 0; j < n_order; ++j)
    if (order[j] >= c->N) return fail(c, TGSIM_EINVAL, "order[%u] is not an instance", j);
  HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
  ProbeDev& p = c->d.pr;
  for (void* q : {(void*)p.order, (void*)p.pos, (void*)p.state, (void*)p.refused, (void*)p.replied,
                  (void*)p.t_req, (void*)p.t_rep, (void*)p.t_reparr, (void*)p.t_done, (void*)p.out, (void*)p.sc,
                  (void*)p.ans, (void*)p.cur, (void*)p.alist, (void*)p.rqa, (void*)p.prop_all})
    dfree(c, q);
  p = ProbeDev{};
  c->probes = false;
  c->probe_need_react = false;
  const size_t nl = std::max<uint32_t>(c->nloc, 1), nn = std::max<uint32_t>(c->N, 1);
  if (dalloc(c, &p.order, n_order) || dalloc(c, &p.pos, nl) || dalloc(c, &p.state, nl) || dalloc(c, &p.refused, nl) ||
      dalloc(c, &p.replied, nl) || dalloc(c, &p.t_req, nl) || dalloc(c, &p.t_rep, nl) || dalloc(c, &p.t_reparr, nl) ||
      dalloc(c, &p.t_done, nl) || dalloc(c, &p.out, nl * n_order) || dalloc(c, &p.sc, 1) ||
      dalloc(c, &p.ans, nn) || dalloc(c, &p.cur, nn) || dalloc(c, &p.alist, nn) || dalloc(c, &p.rqa, nn) ||
      dalloc(c, &p.prop_all, (size_t)3 * c->S))
    return TGSIM_ENOMEM;
  hipStream_t st = c->d.stream;
  HIPCK(c, hipMemsetAsync(p.ans, 0, nn * 4, st), "probe setup");
  HIPCK(c, hipMemsetAsync(p.cur, 0, nn * 4, st), "probe setup");
  HIPCK(c, hipMemsetAsync(p.rqa, 0, nn * 8, st), "probe setup");  // no request arrived
  HIPCK(c, hipMemcpyAsync(p.order, order, (size_t)n_order * 4, hipMemcpyHostToDevice, st), "probe setup");
  HIPCK(c, hipMemsetAsync(p.state, 0, nl, st), "probe setup");
  HIPCK(c, hipMemsetAsync(p.out, 0, nl * n_order, st), "probe setup");
  HIPCK(c, hipMemsetAsync(p.sc, 0, sizeof(ProbeScalars), st), "probe setup");
  std::vector<int64_t> tmin(nl, INT64_MIN);
  HIPCK(c, hipMemcpyAsync(p.t_done, tmin.data(), nl * 8, hipMemcpyHostToDevice, st), "probe setup");
  HIPCK(c, hipStreamSynchronize(st), "probe setup");  // tmin goes out of scope
  p.n_order = n_order;
  p.lo = c->lo; p.nloc = c->nloc; p.N = c->N; p.S = c->S; p.shard = c->shard; p.xcap = c->d.xcap;
  p.xq = c->d.qc + ((size_t)3 * kNSub << 5);  // the exchange cursors' lines (idle between windows)
  p.xsend = c->d.xsend; p.xrecv = c->d.xrecv;
  p.req_bytes = cfg->request_bytes;
  p.rep_bytes = cfg->reply_bytes;
  p.timeout = cfg->timeout_ns;
  p.window = cfg->window_ns;
  c->probes = true;
  uint64_t h = fnv1a(0xCBF29CE484222325ull, order, (size_t)n_order * 4);
  h = fnv1a(h, &cfg->request_bytes, 4); h = fnv1a(h, &cfg->reply_bytes, 4);
  h = fnv1a(h, &cfg->timeout_ns, 8); h = fnv1a(h, &cfg->window_ns, 8);
  c->probe_hash = h | 1u;
  return TGSIM_OK;
}

// Probes stage on the device: behind the device-side count, which starts at the host's count.
static void probes_staged(tgsim_ctx* c) {
  c->spec.valid = false;
  c->staged_dev = true;
  c->win_m_extra += 1;                                        // one request per prober
  c->win_m_inbox = std::max<uint32_t>(c->win_m_inbox, 1u);    // one reply per request delivered last window
  c->win_inbox_max = std::max<uint64_t>(c->win_inbox_max, c->N);
}

static int tgsim_probe_start_body(tgsim_ctx* c, int64_t t0);
extern "C" int tgsim_probe_start(tgsim_ctx* c, int64_t t0) {
  return abi_guard(c, [&] { return tgsim_probe_start_body(c, t0); });
}
static int tgsim_probe_start_body(tgsim_ctx* c, int64_t t0) {
  if (!c) return TGSIM_EINVAL;
  if (!c->probes) return fail(c, TGSIM_ESTATE, "no probes set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (int rc = react_owed(c)) return rc;
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  if (t0 < c->horizon) return fail(c, TGSIM_ECAUSALITY, "t0 before the reaction horizon");
  HIPCK(c, launch_probe_start(c->d, c->staged_dev, c->n_staged, t0), "probe start");
  probes_staged(c);
  c->max_tsend_h = std::max(c->max_tsend_h, t0);
  return TGSIM_OK;
}

static int tgsim_probe_react_body(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active);
extern "C" int tgsim_probe_react(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active) {
  return abi_guard(c, [&] { return tgsim_probe_react_body(c, next_end, n_active); });
}
static int tgsim_probe_react_body(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active) {
  if (!c) return TGSIM_EINVAL;
  if (!c->probes) return fail(c, TGSIM_ESTATE, "no probes set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (!c->probe_need_react) return fail(c, TGSIM_ESTATE, "probes: no window since the last reaction");
  const bool on_dev = c->n_status_last == kStatusOnDevice;
  if (int rc = need_transport(c)) return rc;
  c->probe_need_react = false;
  if (c->S == 1) {
    HIPCK(c, launch_probe_react(c->d, c->staged_dev, c->n_staged, on_dev ? 0u : c->n_status_last,
                                on_dev ? &c->d.sc->n_msgs_last : nullptr), "probe react");
  } else {  // the peers' answers reach the probers' shards as notices; the proposal over every shard
    int rc = TGSIM_OK;
    HIPCK(c, launch_probe_react_pre(c->d, c->staged_dev, c->n_staged, on_dev ? 0u : c->n_status_last,
                                    on_dev ? &c->d.sc->n_msgs_last : nullptr), "probe react");
    if (c->tr.alltoall(c->tr.user, c->d.xsend, c->d.xrecv, (size_t)c->d.xcap * sizeof(tgsim_record), c->d.stream) != 0)
      rc = fail(c, TGSIM_EHIP, "transport all-to-all failed");
    if (!rc) HIPCK(c, launch_probe_react_post(c->d), "probe react");
    if (!rc && c->tr.allgather(c->tr.user, c->d.pr.sc->prop, c->d.pr.prop_all, 3 * sizeof(int64_t), c->d.stream) != 0)
      rc = fail(c, TGSIM_EHIP, "transport all-gather failed");
    if (!rc) HIPCK(c, launch_probe_prop(c->d), "probe react");
    if (rc) return shard_failed(c, rc);
  }
  probes_staged(c);
  if (!next_end && !n_active) return TGSIM_OK;  // asynchronous
  ProbeScalars ps;
  HIPCK(c, hipMemcpyAsync(&ps, c->d.pr.sc, sizeof(ps), hipMemcpyDeviceToHost, c->d.stream), "probe react");
  const int rc = sync_and_check(c);
  if (rc) return rc;
  if (next_end) *next_end = ps.next_end;
  if (n_active) *n_active = ps.n_active;
  return TGSIM_OK;
}

static int tgsim_probe_state_device_body(tgsim_ctx* c, const int64_t** next_end, const uint32_t** n_active);
extern "C" int tgsim_probe_state_device(tgsim_ctx* c, const int64_t** next_end, const uint32_t** n_active) {
  return abi_guard(c, [&] { return tgsim_probe_state_device_body(c, next_end, n_active); });
}
static int tgsim_probe_state_device_body(tgsim_ctx* c, const int64_t** next_end, const uint32_t** n_active) {
  if (!c) return TGSIM_EINVAL;
  if (!c->probes) return fail(c, TGSIM_ESTATE, "no probes set up");
  if (next_end) *next_end = &c->d.pr.sc->next_end;
  if (n_active) *n_active = &c->d.pr.sc->n_active;
  return TGSIM_OK;
}

static int tgsim_probe_results_body(tgsim_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap);
extern "C" int tgsim_probe_results(tgsim_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap) {
  return abi_guard(c, [&] { return tgsim_probe_results_body(c, outcome, t_done, cap); });
}
static int tgsim_probe_results_body(tgsim_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap) {
  if (!c) return TGSIM_EINVAL;
  if (!c->probes) return fail(c, TGSIM_ESTATE, "no probes set up");
  int rc = sync_and_check(c);
  if (rc) return rc;
  const size_t n = (size_t)c->nloc * c->d.pr.n_order;
  if (outcome) {
    if (cap < n) return fail(c, TGSIM_ECAPACITY, "outcome capacity %zu < %zu", cap, n);
    if (n) HIPCK(c, hipMemcpy(outcome, c->d.pr.out, n, hipMemcpyDeviceToHost), "probe results");
  }
  if (t_done && c->nloc) HIPCK(c, hipMemcpy(t_done, c->d.pr.t_done, (size_t)c->nloc * 8, hipMemcpyDeviceToHost), "probe results");
  return TGSIM_OK;
}

// ============================== storm plan reactor ==========================
// plans/benchmarks/storm.go:117-190: the dial semaphore, DialTimeout, writesem and conn.Write
// blocking on the send buffer, for every instance on the device. Kernels in tgsim_storm.hip, oracle
// twin tgo_storm_*.

static int tgsim_tcp_connect_body(tgsim_ctx* c, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* out);
static void storm_free(tgsim_ctx* c) {
  StormDev& s = c->d.sm;
  for (void* q : {(void*)s.dst, (void*)s.t_ready, (void*)s.state, (void*)s.flags, (void*)s.res, (void*)s.slot,
                  (void*)s.t_start, (void*)s.t_synarr, (void*)s.t_ackarr, (void*)s.t_done, (void*)s.t_rep,
                  (void*)s.emit, (void*)s.rem, (void*)s.infl, (void*)s.order, (void*)s.ring, (void*)s.claim,
                  (void*)s.dq, (void*)s.qh, (void*)s.ql, (void*)s.nh, (void*)s.slot_t, (void*)s.hold,
                  (void*)s.failed, (void*)s.t_last, (void*)s.sc, (void*)s.settled, (void*)s.wsegs, (void*)s.ans,
                  (void*)s.alist, (void*)s.prop_all})
    dfree(c, q);
  s = StormDev{};
  c->storm_on = false;
  c->storm_need_react = false;
}

static int tgsim_storm_setup_body(tgsim_ctx* c, const uint32_t* dst, const int64_t* t_ready, const tgsim_storm_config* cfg);
extern "C" int tgsim_storm_setup(tgsim_ctx* c, const uint32_t* dst, const int64_t* t_ready, const tgsim_storm_config* cfg) {
  return abi_guard(c, [&] { return tgsim_storm_setup_body(c, dst, t_ready, cfg); });
}
static int tgsim_storm_setup_body(tgsim_ctx* c, const uint32_t* dst, const int64_t* t_ready, const tgsim_storm_config* cfg) {
  if (!c || !cfg) return TGSIM_EINVAL;
  if (cfg->outgoing == 0 || cfg->concurrent == 0 || cfg->chunk_bytes == 0 || cfg->msg_window == 0 ||
      cfg->dial_timeout_ns <= 0 || cfg->window_ns <= 0 || cfg->syn_bytes >= 0x80000000u ||
      (uint64_t)cfg->chunk_bytes + cfg->header_bytes >= 0x80000000ull)
    return fail(c, TGSIM_EINVAL, "bad storm configuration");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->S != 1 && c->tcp_on) return fail(c, TGSIM_ENOTSUP, "TCP mode needs a single-shard context");
  if (int rc = need_transport(c)) return rc;  // sharded: the notices and the proposal are collective
  if (!c->fl_off.empty() || c->probes)
    return fail(c, TGSIM_ESTATE, "the storm reactor runs without a flood graph or probes");
  if (c->tcp_on && (!c->tcp.acks || c->td.n_conn || c->tw_n))
    return fail(c, TGSIM_ESTATE, "a TCP storm needs acks = 1 and a context without connections or writes yet");
  const uint64_t n_conn = (uint64_t)c->N * cfg->outgoing;
  const uint64_t nchunks = (cfg->data_bytes + cfg->chunk_bytes - 1) / cfg->chunk_bytes;
  if (n_conn > 0x3FFFFFFFull || nchunks * cfg->outgoing > 0x3FFFFFFFull)
    return fail(c, TGSIM_ENOTSUP, "too many connections or chunks for the storm's packet tags");
  if (n_conn && (!dst || !t_ready)) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  for (uint64_t h = 0; h < n_conn; ++h) {
    if (dst[h] >= c->N) return fail(c, TGSIM_EINVAL, "connection %llu: bad peer", (unsigned long long)h);
    if (t_ready[h] < c->now) return fail(c, TGSIM_ECAUSALITY, "connection %llu: t_ready before now", (unsigned long long)h);
  }
  // TCP mode: connection h = instance * outgoing + k; its SYN write and its chunks' writes get ids
  // reserved now, so the device writes them with no host bookkeeping
  uint64_t spc = 0, spcon = 0, tot_w = 0, tot_s = 0;
  if (c->tcp_on) {
    const uint64_t mss = c->td.mss, last = nchunks ? cfg->data_bytes - (nchunks - 1) * cfg->chunk_bytes : 0;
    spc = (cfg->chunk_bytes + mss - 1) / mss;
    spcon = 1 + (nchunks ? (nchunks - 1) * spc + (last + mss - 1) / mss : 0);
    tot_w = n_conn * (nchunks + 1);
    tot_s = n_conn * spcon;
    if (n_conn > c->tcp.max_writes || tot_w > c->tcp.max_writes || tot_s > c->tcp.max_segments)
      return fail(c, TGSIM_ECAPACITY, "TCP storm: %llu writes / %llu segments exceed the TCP capacities",
                  (unsigned long long)tot_w, (unsigned long long)tot_s);
  }
  HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
  storm_free(c);
  alloc_point(c);
  const uint32_t O = cfg->outgoing, C = cfg->concurrent, Hc = std::min(C, O);
  // per instance, its connections in dial FIFO order (t_ready, k): a Go channel queues blocked
  // senders in arrival order, and a goroutine arrives when its sleep ends
  std::vector<uint32_t> order(n_conn);
  for (uint32_t g = 0; g < c->N; ++g) {
    uint32_t* o = order.data() + (size_t)g * O;
    const int64_t* tr = t_ready + (size_t)g * O;
    for (uint32_t k = 0; k < O; ++k) o[k] = k;
    std::stable_sort(o, o + O, [&](uint32_t a, uint32_t b) { return tr[a] < tr[b]; });
  }
  StormDev& s = c->d.sm;
  const size_t nc = std::max<uint64_t>(n_conn, 1), nl = std::max<uint32_t>(c->nloc, 1);
  const size_t claim_words = std::max<uint64_t>((n_conn * nchunks + 31) / 32, 1);
  if (dalloc(c, &s.dst, nc) || dalloc(c, &s.t_ready, nc) || dalloc(c, &s.state, nc) || dalloc(c, &s.flags, nc) ||
      dalloc(c, &s.res, nc) || dalloc(c, &s.slot, nc) || dalloc(c, &s.t_start, nc) || dalloc(c, &s.t_synarr, nc) ||
      dalloc(c, &s.t_ackarr, nc) || dalloc(c, &s.t_done, nc) || dalloc(c, &s.t_rep, nc) || dalloc(c, &s.emit, nc) ||
      dalloc(c, &s.rem, nc) || dalloc(c, &s.infl, nc) || dalloc(c, &s.order, nc) || dalloc(c, &s.ring, nc) ||
      dalloc(c, &s.claim, claim_words) || dalloc(c, &s.dq, nl) || dalloc(c, &s.qh, nl) || dalloc(c, &s.ql, nl) ||
      dalloc(c, &s.nh, nl) || dalloc(c, &s.slot_t, nl * C) || dalloc(c, &s.hold, nl * Hc) ||
      dalloc(c, &s.failed, nl) || dalloc(c, &s.t_last, nl) || dalloc(c, &s.sc, 1) ||
      dalloc(c, &s.ans, nc) || dalloc(c, &s.alist, nc) || dalloc(c, &s.prop_all, (size_t)3 * c->S) ||
      (c->tcp_on && (dalloc(c, &s.settled, nc) || dalloc(c, &s.wsegs, nc)))) {
    storm_free(c);
    return TGSIM_ENOMEM;
  }
  hipStream_t st = c->d.stream;
  std::vector<int64_t> tmin(std::max(nl * C, nc), INT64_MIN), tmax(nc, INT64_MAX);
  HIPCK(c, hipMemcpyAsync(s.dst, dst, n_conn * 4, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemcpyAsync(s.t_ready, t_ready, n_conn * 8, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemcpyAsync(s.order, order.data(), n_conn * 4, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemcpyAsync(s.slot_t, tmin.data(), nl * C * 8, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemcpyAsync(s.t_last, tmin.data(), nl * 8, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemcpyAsync(s.t_done, tmin.data(), nc * 8, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemcpyAsync(s.t_synarr, tmax.data(), nc * 8, hipMemcpyHostToDevice, st), "storm setup");
  HIPCK(c, hipMemsetAsync(s.ans, 0, nc * 4, st), "storm setup");
  for (void* z : {(void*)s.state, (void*)s.flags, (void*)s.res}) HIPCK(c, hipMemsetAsync(z, 0, nc, st), "storm setup");
  for (void* z : {(void*)s.rem, (void*)s.infl, (void*)s.emit}) HIPCK(c, hipMemsetAsync(z, 0, nc * 4, st), "storm setup");
  HIPCK(c, hipMemsetAsync(s.claim, 0, claim_words * 4, st), "storm setup");
  for (void* z : {(void*)s.dq, (void*)s.qh, (void*)s.ql, (void*)s.nh}) HIPCK(c, hipMemsetAsync(z, 0, nl * 4, st), "storm setup");
  HIPCK(c, hipMemsetAsync(s.failed, 0, nl, st), "storm setup");
  HIPCK(c, hipMemsetAsync(s.sc, 0, sizeof(StormScalars), st), "storm setup");
  HIPCK(c, hipStreamSynchronize(st), "storm setup");  // the host vectors go out of scope
  s.O = O;
  s.C = C;
  s.Hc = Hc;
  s.nchunks = (uint32_t)nchunks;
  s.chunk = cfg->chunk_bytes;
  s.hdr = cfg->header_bytes;
  s.syn = cfg->syn_bytes;
  s.win = cfg->msg_window;
  s.data = cfg->data_bytes;
  s.timeout = cfg->dial_timeout_ns;
  s.window = cfg->window_ns;
  s.n_conn = (uint32_t)n_conn;
  s.phase = 0;
  s.lo = c->lo; s.N = c->N; s.S = c->S; s.shard = c->shard; s.xcap = c->d.xcap;
  s.xq = c->d.qc + ((size_t)3 * kNSub << 5);  // the exchange cursors' lines (idle between windows)
  s.xsend = c->d.xsend; s.xrecv = c->d.xrecv;
  if (c->tcp_on) {
    std::vector<uint32_t> src(n_conn);
    for (uint64_t h = 0; h < n_conn; ++h) src[h] = (uint32_t)(h / O);
    const uint64_t conn_lo = c->td.n_conn;
    int rc = tgsim_tcp_connect_body(c, src.data(), dst, n_conn, nullptr);  // connection ids 0 .. n_conn - 1
    if (rc) { storm_free(c); return rc; }
    c->storm_conn_lo = conn_lo;
    c->storm_conn_hi = c->td.n_conn;
    s.tcp = 1;
    s.mss = c->td.mss;
    s.spc = (uint32_t)spc;
    s.spcon = (uint32_t)spcon;
    s.W0 = (uint32_t)c->tw_n;
    s.S0 = (uint32_t)c->tsg_n;
    HIPCK(c, hipMemsetAsync(s.settled, 0, nc * 4, st), "storm setup");
    HIPCK(c, hipMemsetAsync(s.wsegs, 0, nc * 4, st), "storm setup");
    HIPCK(c, launch_storm_tcp_init(c->d, c->td), "storm setup");
    for (uint64_t h = 0; h < n_conn; ++h) c->conn_tail[h] = (uint32_t)(s.S0 + (h + 1) * spcon - 1);
    c->tw_n += tot_w;
    c->tsg_n += tot_s;
    c->tcp_seg_batched = c->tsg_n;
    c->tstats.writes += tot_w;
    c->tstats.segments += tot_s;
  }
  c->storm_on = true;
  c->storm_need_react = false;
  uint64_t h = fnv1a(0xCBF29CE484222325ull, dst, n_conn * 4);
  h = fnv1a(h, t_ready, n_conn * 8);
  c->storm_hash = fnv1a(h, cfg, sizeof(*cfg)) | 1u;
  return TGSIM_OK;
}

// TCP mode: what the connections' windows have room for leaves at the write times (the reactor's
// writes were linked onto the queues; tgsim_tcp_write does the same after a host write)
static int storm_tcp_release(tgsim_ctx* c) {
  if (!c->d.sm.tcp) return TGSIM_OK;
  HIPCK(c, launch_tcp_conn_release(c->d, c->td, kRelAtWrite, c->tcp_cur, true, 0), "storm tcp release");
  return TGSIM_OK;
}

// The reactor stages on the device, behind the device-side count. The queue-limit bound per sender:
// dial phase - its SYNs (one per connection) and a SYN-ACK per delivery of its last inbox; write
// phase - at most msg_window chunks per connection (a connection's buffer).
static void storm_staged(tgsim_ctx* c) {
  const StormDev& s = c->d.sm;
  c->spec.valid = false;
  c->staged_dev = true;
  if (s.tcp) {  // SYNs, then one chunk's segments per connection per reaction
    c->win_m_extra += (uint64_t)s.O * (s.phase == 0 ? 1u : s.spc);
  } else if (s.phase == 0) {
    c->win_m_extra += s.O;
    c->win_m_inbox = std::max<uint32_t>(c->win_m_inbox, 1u);
    c->win_inbox_max = std::max<uint64_t>(c->win_inbox_max, s.n_conn);
  } else {
    c->win_m_extra += (uint64_t)s.win * s.O;
  }
}

static int tgsim_storm_start_body(tgsim_ctx* c);
extern "C" int tgsim_storm_start(tgsim_ctx* c) {
  return abi_guard(c, [&] { return tgsim_storm_start_body(c); });
}
static int tgsim_storm_start_body(tgsim_ctx* c) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->d.sm.phase != 0) return fail(c, TGSIM_ESTATE, "the storm's dials have started");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (int rc = react_owed(c)) return rc;
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  HIPCK(c, launch_storm_start(c->d, c->td, c->staged_dev, c->n_staged, c->now), "storm start");
  storm_staged(c);
  return storm_tcp_release(c);
}

static int storm_read_scalars(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active) {
  StormScalars ss;
  HIPCK(c, hipMemcpyAsync(&ss, c->d.sm.sc, sizeof(ss), hipMemcpyDeviceToHost, c->d.stream), "storm react");
  const int rc = sync_and_check(c);
  if (rc) return rc;
  if (next_end) *next_end = ss.next_end;
  if (n_active) *n_active = ss.n_active;
  return TGSIM_OK;
}

static int tcp_snapshot(tgsim_ctx* c);
static int tgsim_storm_react_body(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active);
extern "C" int tgsim_storm_react(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active) {
  return abi_guard(c, [&] { return tgsim_storm_react_body(c, next_end, n_active); });
}
static int tgsim_storm_react_body(tgsim_ctx* c, int64_t* next_end, uint32_t* n_active) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (!c->storm_need_react) return fail(c, TGSIM_ESTATE, "storm: no window since the last reaction");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tgsim_tcp_react before tgsim_storm_react");
  const bool on_dev = c->n_status_last == kStatusOnDevice;
  if (int rc = need_transport(c)) return rc;
  c->storm_need_react = false;
  if (c->d.sm.tcp) {
    HIPCK(c, launch_storm_react(c->d, c->td, c->staged_dev, c->n_staged, on_dev ? 0u : c->n_status_last,
                                on_dev ? &c->d.sc->n_msgs_last : nullptr), "storm react");
    // the step can fail SYN writes (DialTimeout): the TCP counters as they stand after it
    if (int rc = tcp_snapshot(c)) return rc;
  } else {
    int rc = TGSIM_OK;
    HIPCK(c, launch_storm_react_pre(c->d, c->staged_dev, c->n_staged, on_dev ? 0u : c->n_status_last,
                                    on_dev ? &c->d.sc->n_msgs_last : nullptr), "storm react");
    if (c->S > 1 && c->tr.alltoall(c->tr.user, c->d.xsend, c->d.xrecv, (size_t)c->d.xcap * sizeof(tgsim_record),
                                   c->d.stream) != 0)  // the notices to the diallers' shards
      rc = fail(c, TGSIM_EHIP, "transport all-to-all failed");
    if (!rc) HIPCK(c, launch_storm_react_post(c->d, c->td), "storm react");
    if (!rc && c->S > 1) {  // the proposal over every shard
      if (c->tr.allgather(c->tr.user, c->d.sm.sc->prop, c->d.sm.prop_all, 3 * sizeof(int64_t), c->d.stream) != 0)
        rc = fail(c, TGSIM_EHIP, "transport all-gather failed");
      else HIPCK(c, launch_storm_prop(c->d), "storm react");
    }
    if (rc) return shard_failed(c, rc);
  }
  storm_staged(c);
  if (int rc = storm_tcp_release(c)) return rc;
  if (!next_end && !n_active) return TGSIM_OK;  // asynchronous
  return storm_read_scalars(c, next_end, n_active);
}

static int tgsim_storm_state_device_body(tgsim_ctx* c, const int64_t** next_end, const uint32_t** n_active);
extern "C" int tgsim_storm_state_device(tgsim_ctx* c, const int64_t** next_end, const uint32_t** n_active) {
  return abi_guard(c, [&] { return tgsim_storm_state_device_body(c, next_end, n_active); });
}
static int tgsim_storm_state_device_body(tgsim_ctx* c, const int64_t** next_end, const uint32_t** n_active) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (next_end) *next_end = &c->d.sm.sc->next_end;
  if (n_active) *n_active = &c->d.sm.sc->n_active;
  return TGSIM_OK;
}

static int tgsim_storm_dials_body(tgsim_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap);
extern "C" int tgsim_storm_dials(tgsim_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap) {
  return abi_guard(c, [&] { return tgsim_storm_dials_body(c, outcome, t_done, cap); });
}
static int tgsim_storm_dials_body(tgsim_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  // the local instances' connections [lo * O, hi * O)
  const size_t h0 = (size_t)c->lo * c->d.sm.O, n = (size_t)c->nloc * c->d.sm.O;
  if ((outcome || t_done) && cap < n) return fail(c, TGSIM_ECAPACITY, "dial capacity %zu < %zu", cap, n);
  int rc = sync_and_check(c);
  if (rc) return rc;
  if (outcome && n) HIPCK(c, hipMemcpy(outcome, c->d.sm.res + h0, n, hipMemcpyDeviceToHost), "storm dials");
  if (t_done && n) HIPCK(c, hipMemcpy(t_done, c->d.sm.t_done + h0, n * 8, hipMemcpyDeviceToHost), "storm dials");
  return TGSIM_OK;
}

static int tgsim_storm_write_start_body(tgsim_ctx* c, int64_t t0);
extern "C" int tgsim_storm_write_start(tgsim_ctx* c, int64_t t0) {
  return abi_guard(c, [&] { return tgsim_storm_write_start_body(c, t0); });
}
static int tgsim_storm_write_start_body(tgsim_ctx* c, int64_t t0) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->d.sm.phase != 0) return fail(c, TGSIM_ESTATE, "the write phase has started");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (int rc = react_owed(c)) return rc;
  int rc = sync_and_check(c);
  if (rc) return rc;
  if (t0 < c->horizon) return fail(c, TGSIM_ECAUSALITY, "t0 before the reaction horizon");
  // a goroutine writes only after its dial succeeded and "outgoing-dials-done" released, which needs
  // every dial (storm.go:156): the write phase starts once all of them are OK
  const size_t h0 = (size_t)c->lo * c->d.sm.O;
  std::vector<uint8_t> res((size_t)c->nloc * c->d.sm.O);
  if (!res.empty()) HIPCK(c, hipMemcpy(res.data(), c->d.sm.res + h0, res.size(), hipMemcpyDeviceToHost), "storm write start");
  int64_t bad = -1;
  for (size_t i = 0; i < res.size() && bad < 0; ++i)
    if (res[i] != TGSIM_PROBE_OK) bad = (int64_t)(h0 + i);
  if (c->S > 1) {  // every shard's dials (agreed: the phase starts everywhere or nowhere)
    if (int rc2 = need_transport(c)) return rc2;
    HIPCK(c, hipMemcpy(c->d_red2, &bad, 8, hipMemcpyHostToDevice), "storm write start");
    if (c->tr.allreduce_max_i64(c->tr.user, c->d_red2, 1, c->d.stream) != 0)
      return shard_failed(c, fail(c, TGSIM_EHIP, "transport all-reduce failed"));
    HIPCK(c, hipMemcpyAsync(&bad, c->d_red2, 8, hipMemcpyDeviceToHost, c->d.stream), "storm write start");
    HIPCK(c, hipStreamSynchronize(c->d.stream), "storm write start");
  }
  if (bad >= 0) return fail(c, TGSIM_ESTATE, "connection %lld has not dialled successfully", (long long)bad);
  c->d.sm.phase = 1;
  HIPCK(c, launch_storm_write_start(c->d, c->td, c->staged_dev, c->n_staged, t0), "storm write start");
  storm_staged(c);
  return storm_tcp_release(c);
}

static int tgsim_storm_results_body(tgsim_ctx* c, uint8_t* failed, int64_t* t_last, size_t cap, tgsim_storm_totals* tot);
extern "C" int tgsim_storm_results(tgsim_ctx* c, uint8_t* failed, int64_t* t_last, size_t cap, tgsim_storm_totals* tot) {
  return abi_guard(c, [&] { return tgsim_storm_results_body(c, failed, t_last, cap, tot); });
}
static int tgsim_storm_results_body(tgsim_ctx* c, uint8_t* failed, int64_t* t_last, size_t cap, tgsim_storm_totals* tot) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if ((failed || t_last) && cap < c->nloc) return fail(c, TGSIM_ECAPACITY, "result capacity %zu < %u", cap, c->nloc);
  int rc = sync_and_check(c);
  if (rc) return rc;
  const StormDev& s = c->d.sm;
  const size_t h0 = (size_t)c->lo * s.O, n = (size_t)c->nloc * s.O;  // the local connections
  std::vector<uint32_t> infl(n), rem(n);
  std::vector<uint8_t> res(n), fl(c->nloc);
  if (n) {
    // "in flight": message mode, chunks in the buffer; TCP, written chunks not yet settled
    if (s.tcp) {
      HIPCK(c, hipMemcpy(infl.data(), s.settled + h0, n * 4, hipMemcpyDeviceToHost), "storm results");
      HIPCK(c, hipMemcpy(rem.data(), s.rem + h0, n * 4, hipMemcpyDeviceToHost), "storm results");
      for (size_t h = 0; h < n; ++h) infl[h] = s.phase == 1 ? (s.nchunks - rem[h]) - infl[h] : 0u;
    } else {
      HIPCK(c, hipMemcpy(infl.data(), s.infl + h0, n * 4, hipMemcpyDeviceToHost), "storm results");
    }
    HIPCK(c, hipMemcpy(rem.data(), s.rem + h0, n * 4, hipMemcpyDeviceToHost), "storm results");
    HIPCK(c, hipMemcpy(res.data(), s.res + h0, n, hipMemcpyDeviceToHost), "storm results");
  }
  if (c->nloc) HIPCK(c, hipMemcpy(fl.data(), s.failed, c->nloc, hipMemcpyDeviceToHost), "storm results");
  for (size_t h = 0; h < n; ++h)
    if (infl[h] || (s.phase == 1 && rem[h])) fl[h / s.O] = 1;  // still in flight or unwritten
  if (failed) memcpy(failed, fl.data(), c->nloc);
  if (t_last && c->nloc) HIPCK(c, hipMemcpy(t_last, s.t_last, (size_t)c->nloc * 8, hipMemcpyDeviceToHost), "storm results");
  if (tot) {
    StormScalars ss;
    HIPCK(c, hipMemcpy(&ss, s.sc, sizeof(ss), hipMemcpyDeviceToHost), "storm results");
    *tot = tgsim_storm_totals{};
    tot->chunks_written = ss.written;
    tot->chunks_delivered = ss.delivered;
    tot->chunks_failed = ss.failed;
    tot->bytes_written = ss.bytes;
    for (size_t h = 0; h < n; ++h) {
      tot->dials_ok += res[h] == TGSIM_PROBE_OK;
      tot->dials_failed += res[h] == TGSIM_PROBE_REFUSED || res[h] == TGSIM_PROBE_TIMEOUT;
      tot->dials_pending += res[h] == TGSIM_PROBE_NONE;
      tot->conns_writing += s.phase == 1 && (rem[h] || infl[h]);
    }
  }
  return TGSIM_OK;
}

static int tgsim_storm_end_body(tgsim_ctx* c);
extern "C" int tgsim_storm_end(tgsim_ctx* c) {
  return abi_guard(c, [&] { return tgsim_storm_end_body(c); });
}
static int tgsim_storm_end_body(tgsim_ctx* c) {
  if (!c) return TGSIM_EINVAL;
  if (!c->storm_on) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
  storm_free(c);
  return TGSIM_OK;
}

// ============================== topics (sync.Client Publish / Subscribe) ===================
// [EXT sdk-go]; call sites plans/network/pingpong.go:219-245, plans/benchmarks/storm.go:232-255,
// plans/splitbrain/main.go:91-103. Positions come from the device signal path (a topic is a sync
// state); the entries and payload bytes are appended to device arenas in (topic, position) order,
// so a subscription is a few contiguous copies. Oracle twin: tgo_sync_publish / _subscribe.

template <typename T>
static int dgrow(tgsim_ctx* c, T** p, uint64_t used, uint64_t need_cap) {
  T* q = nullptr;
  if (dalloc(c, &q, need_cap)) return TGSIM_ENOMEM;
  if (used && *p) HIPCK(c, hipMemcpy(q, *p, used * sizeof(T), hipMemcpyDeviceToDevice), "topic grow");
  dfree(c, *p);
  *p = q;
  return TGSIM_OK;
}

static int tgsim_sync_publish_body(tgsim_ctx* c, const uint32_t* topics, const uint32_t* inst, const int64_t* t,
                                  const uint64_t* off, const uint8_t* payload, size_t n, uint32_t* pos_out);
extern "C" int tgsim_sync_publish(tgsim_ctx* c, const uint32_t* topics, const uint32_t* inst, const int64_t* t,
                                  const uint64_t* off, const uint8_t* payload, size_t n, uint32_t* pos_out) {
  return abi_guard(c, [&] { return tgsim_sync_publish_body(c, topics, inst, t, off, payload, n, pos_out); });
}
static int tgsim_sync_publish_body(tgsim_ctx* c, const uint32_t* topics, const uint32_t* inst, const int64_t* t,
                                  const uint64_t* off, const uint8_t* payload, size_t n, uint32_t* pos_out) {
  if (!c) return TGSIM_EINVAL;
  c->spec.valid = false;  // signal partials change: no speculative storm round
  if (n && (!topics || !inst || !t || !off || (off[n] && !payload))) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (n && off[0] != 0) return fail(c, TGSIM_EINVAL, "payload offsets must start at 0");
  for (size_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) return fail(c, TGSIM_EINVAL, "bad payload offsets");
  if (n == 0) return TGSIM_OK;
  if (c->tp_n + n > 0xFFFFFFFFull) return fail(c, TGSIM_ECAPACITY, "topic arena holds at most 2^32 - 1 entries");
  std::vector<uint32_t> pos(n);
  c->replicated_batch = true;  // topics are replicated: every shard publishes the same batch
  int rc = tgsim_sync_signal(c, topics, inst, t, n, pos.data());
  c->replicated_batch = false;
  if (rc) return rc;
  std::vector<uint32_t> ord(n);
  for (uint32_t i = 0; i < n; ++i) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
    return topics[a] != topics[b] ? topics[a] < topics[b] : pos[a] < pos[b];
  });
  const uint64_t bytes = off[n];
  if (c->tp_n + n > 0xFFFFFFFFull) return fail(c, TGSIM_ECAPACITY, "topic arena holds at most 2^32 - 1 entries");
  if (c->tp_n + n > c->tp_cap) {
    const uint64_t cap = std::max<uint64_t>(c->tp_n + n, 2 * c->tp_cap);
    if (dgrow(c, &c->tp_inst, c->tp_n, cap) || dgrow(c, &c->tp_t, c->tp_n, cap) ||
        dgrow(c, &c->tp_off, c->tp_n, cap) || dgrow(c, &c->tp_len, c->tp_n, cap))
      return TGSIM_ENOMEM;
    c->tp_cap = cap;
  }
  if (c->tp_nbytes + bytes > c->tp_bytes_cap) {
    const uint64_t cap = std::max<uint64_t>(c->tp_nbytes + bytes, 2 * c->tp_bytes_cap);
    if (dgrow(c, &c->tp_bytes, c->tp_nbytes, cap)) return TGSIM_ENOMEM;
    c->tp_bytes_cap = cap;
  }
  std::vector<uint32_t> si(n), sl(n);
  std::vector<int64_t> st(n);
  std::vector<uint64_t> so(n);
  std::vector<uint8_t> sb(bytes);
  uint64_t b = 0;
  for (size_t j = 0; j < n; ++j) {
    const uint32_t i = ord[j];
    const uint64_t len = off[i + 1] - off[i];
    si[j] = inst[i]; st[j] = t[i]; so[j] = c->tp_nbytes + b; sl[j] = (uint32_t)len;
    if (len) memcpy(sb.data() + b, payload + off[i], len);
    b += len;
  }
  const uint64_t e0 = c->tp_n;
  HIPCK(c, hipMemcpy(c->tp_inst + e0, si.data(), n * 4, hipMemcpyHostToDevice), "publish");
  HIPCK(c, hipMemcpy(c->tp_t + e0, st.data(), n * 8, hipMemcpyHostToDevice), "publish");
  HIPCK(c, hipMemcpy(c->tp_off + e0, so.data(), n * 8, hipMemcpyHostToDevice), "publish");
  HIPCK(c, hipMemcpy(c->tp_len + e0, sl.data(), n * 4, hipMemcpyHostToDevice), "publish");
  if (bytes) HIPCK(c, hipMemcpy(c->tp_bytes + c->tp_nbytes, sb.data(), bytes, hipMemcpyHostToDevice), "publish");
  if (c->topic_runs.size() < c->d.max_states) c->topic_runs.resize(c->d.max_states);
  for (size_t j = 0; j < n;) {
    size_t k = j;
    while (k < n && topics[ord[k]] == topics[ord[j]]) ++k;
    c->topic_runs[topics[ord[j]]].push_back({pos[ord[j]], (uint32_t)(k - j), e0 + j});
    j = k;
  }
  c->tp_n += n;
  c->tp_nbytes += bytes;
  c->tp_index_dirty = true;
  if (pos_out) memcpy(pos_out, pos.data(), n * 4);
  return TGSIM_OK;
}

static int tgsim_sync_subscribe_body(tgsim_ctx* c, uint32_t topic, uint32_t from, int64_t until_t, size_t cap,
                                    uint32_t* inst_out, int64_t* t_out, uint64_t* off_out, uint8_t* payload_out,
                                    size_t payload_cap, size_t* n_out, size_t* payload_bytes);
extern "C" int tgsim_sync_subscribe(tgsim_ctx* c, uint32_t topic, uint32_t from, int64_t until_t, size_t cap,
                                    uint32_t* inst_out, int64_t* t_out, uint64_t* off_out, uint8_t* payload_out,
                                    size_t payload_cap, size_t* n_out, size_t* payload_bytes) {
  return abi_guard(c, [&] { return tgsim_sync_subscribe_body(c, topic, from, until_t, cap, inst_out, t_out, off_out, payload_out, payload_cap, n_out, payload_bytes); });
}
static int tgsim_sync_subscribe_body(tgsim_ctx* c, uint32_t topic, uint32_t from, int64_t until_t, size_t cap,
                                    uint32_t* inst_out, int64_t* t_out, uint64_t* off_out, uint8_t* payload_out,
                                    size_t payload_cap, size_t* n_out, size_t* payload_bytes) {
  if (!c || !n_out || !payload_bytes || from == 0) return fail(c, TGSIM_EINVAL, "bad arguments");
  *n_out = 0; *payload_bytes = 0;
  if (topic >= c->d.max_states) return fail(c, TGSIM_EINVAL, "bad topic");
  if (topic >= c->topic_runs.size()) return TGSIM_OK;
  // the runs of the topic cover positions 1..count contiguously, in order
  struct Seg { uint64_t entry; uint32_t n; };
  std::vector<Seg> segs;
  size_t want = 0;
  for (const auto& r : c->topic_runs[topic]) {
    if (want >= cap) break;
    if (r.pos0 + r.len <= from) continue;
    const uint32_t skip = from > r.pos0 ? from - r.pos0 : 0u;
    const uint32_t k = (uint32_t)std::min<size_t>(r.len - skip, cap - want);
    segs.push_back({r.entry + skip, k});
    want += k;
  }
  std::vector<uint32_t> inst(want), len(want);
  std::vector<int64_t> tt(want);
  std::vector<uint64_t> eo(want);
  size_t at = 0;
  for (const Seg& s : segs) {
    HIPCK(c, hipMemcpy(inst.data() + at, c->tp_inst + s.entry, s.n * 4ull, hipMemcpyDeviceToHost), "subscribe");
    HIPCK(c, hipMemcpy(tt.data() + at, c->tp_t + s.entry, s.n * 8ull, hipMemcpyDeviceToHost), "subscribe");
    HIPCK(c, hipMemcpy(eo.data() + at, c->tp_off + s.entry, s.n * 8ull, hipMemcpyDeviceToHost), "subscribe");
    HIPCK(c, hipMemcpy(len.data() + at, c->tp_len + s.entry, s.n * 4ull, hipMemcpyDeviceToHost), "subscribe");
    at += s.n;
  }
  size_t k = 0, bytes = 0;  // times never decrease along the positions: the visible entries are a prefix
  while (k < want && tt[k] <= until_t) bytes += len[k++];
  *n_out = k;
  *payload_bytes = bytes;
  if (bytes > payload_cap) return fail(c, TGSIM_ECAPACITY, "payload capacity %zu < %zu", payload_cap, bytes);
  if (k && (!inst_out || !t_out || !off_out || (bytes && !payload_out))) return fail(c, TGSIM_EINVAL, "bad arguments");
  size_t b = 0, j = 0;
  for (const Seg& s : segs) {  // a segment's payloads are contiguous in the arena
    if (j >= k) break;
    const size_t m = std::min<size_t>(s.n, k - j);
    size_t nb = 0;
    for (size_t q = 0; q < m; ++q) nb += len[j + q];
    if (nb) HIPCK(c, hipMemcpy(payload_out + b, c->tp_bytes + eo[j], nb, hipMemcpyDeviceToHost), "subscribe");
    for (size_t q = 0; q < m; ++q) {
      inst_out[j + q] = inst[j + q]; t_out[j + q] = tt[j + q]; off_out[j + q] = b;
      b += len[j + q];
    }
    j += m;
  }
  if (off_out) off_out[k] = b;
  return TGSIM_OK;
}

// Device fan-out: the topic index (CSR over topics of the host's run lists) is rebuilt after a
// publish; counts, scan and inbox fill run on the ctx stream (tgsim_topics.hip).
static int upload_topic_index(tgsim_ctx* c) {
  const uint32_t K = c->d.max_states;
  std::vector<uint32_t> off(K + 1, 0), pos0, len;
  std::vector<uint64_t> entry;
  for (uint32_t k = 0; k < K; ++k) {
    if (k < c->topic_runs.size())
      for (const auto& r : c->topic_runs[k]) { pos0.push_back(r.pos0); len.push_back(r.len); entry.push_back(r.entry); }
    off[k + 1] = (uint32_t)pos0.size();
  }
  const size_t R = pos0.size();
  if (!c->ti_off && dalloc(c, &c->ti_off, (size_t)K + 1)) return TGSIM_ENOMEM;
  if (R > c->ti_cap) {
    const size_t cap = std::max<size_t>(R, 2 * c->ti_cap);
    HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
    dfree(c, c->ti_pos0); dfree(c, c->ti_len); dfree(c, c->ti_entry);
    c->ti_pos0 = c->ti_len = nullptr; c->ti_entry = nullptr;
    if (dalloc(c, &c->ti_pos0, cap) || dalloc(c, &c->ti_len, cap) || dalloc(c, &c->ti_entry, cap)) return TGSIM_ENOMEM;
    c->ti_cap = cap;
  }
  HIPCK(c, hipMemcpyAsync(c->ti_off, off.data(), (K + 1) * 4ull, hipMemcpyHostToDevice, c->d.stream), "topic index");
  if (R) {
    HIPCK(c, hipMemcpyAsync(c->ti_pos0, pos0.data(), R * 4, hipMemcpyHostToDevice, c->d.stream), "topic index");
    HIPCK(c, hipMemcpyAsync(c->ti_len, len.data(), R * 4, hipMemcpyHostToDevice, c->d.stream), "topic index");
    HIPCK(c, hipMemcpyAsync(c->ti_entry, entry.data(), R * 8, hipMemcpyHostToDevice, c->d.stream), "topic index");
  }
  HIPCK(c, hipStreamSynchronize(c->d.stream), "topic index");  // the host vectors go out of scope
  c->tp_index_dirty = false;
  return TGSIM_OK;
}

static int tgsim_sync_subscribe_device_body(tgsim_ctx* c, size_t n, const uint32_t* topics, const uint32_t* from,
                                           const int64_t* until_t, uint32_t cap_each, uint64_t* offsets_out,
                                           uint32_t* entries_out, size_t entries_cap);
extern "C" int tgsim_sync_subscribe_device(tgsim_ctx* c, size_t n, const uint32_t* topics, const uint32_t* from,
                                           const int64_t* until_t, uint32_t cap_each, uint64_t* offsets_out,
                                           uint32_t* entries_out, size_t entries_cap) {
  return abi_guard(c, [&] { return tgsim_sync_subscribe_device_body(c, n, topics, from, until_t, cap_each, offsets_out, entries_out, entries_cap); });
}
static int tgsim_sync_subscribe_device_body(tgsim_ctx* c, size_t n, const uint32_t* topics, const uint32_t* from,
                                           const int64_t* until_t, uint32_t cap_each, uint64_t* offsets_out,
                                           uint32_t* entries_out, size_t entries_cap) {
  if (!c || !offsets_out || (n && (!topics || !from || !until_t))) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (n >= 0xFFFFFFFFull) return fail(c, TGSIM_EINVAL, "too many subscribers");
  if (c->tp_index_dirty) {
    const int rc = upload_topic_index(c);
    if (rc) return rc;
  }
  if (n > c->sub_cap) {
    const size_t cap = std::max<size_t>(n, 2 * c->sub_cap);
    HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
    dfree(c, c->sub_cnt); dfree(c, c->sub_scan);
    c->sub_cnt = nullptr; c->sub_scan = nullptr;
    c->sub_scan_bytes = subscribe_scan_bytes((uint32_t)cap);
    if (dalloc(c, &c->sub_cnt, cap + 1) || dalloc(c, (uint8_t**)&c->sub_scan, c->sub_scan_bytes)) return TGSIM_ENOMEM;
    c->sub_cap = cap;
  }
  if (!c->sub_cnt) {
    c->sub_scan_bytes = subscribe_scan_bytes(0);
    if (dalloc(c, &c->sub_cnt, 1) || dalloc(c, (uint8_t**)&c->sub_scan, c->sub_scan_bytes)) return TGSIM_ENOMEM;
  }
  TopicIndex ti;
  ti.run_off = c->ti_off; ti.pos0 = c->ti_pos0; ti.len = c->ti_len; ti.entry = c->ti_entry; ti.t = c->tp_t;
  ti.n_topics = c->d.max_states;
  HIPCK(c, launch_subscribe(c->d, ti, (uint32_t)n, topics, from, until_t, cap_each, c->sub_cnt, c->sub_scan,
                            c->sub_scan_bytes, offsets_out, entries_out, entries_cap),
        "subscribe");
  return TGSIM_OK;
}

static int tgsim_topic_arena_device_body(tgsim_ctx* c, const uint32_t** inst, const int64_t** t, const uint64_t** off,
                                        const uint32_t** len, const uint8_t** payload, size_t* n);
extern "C" int tgsim_topic_arena_device(tgsim_ctx* c, const uint32_t** inst, const int64_t** t, const uint64_t** off,
                                        const uint32_t** len, const uint8_t** payload, size_t* n) {
  return abi_guard(c, [&] { return tgsim_topic_arena_device_body(c, inst, t, off, len, payload, n); });
}
static int tgsim_topic_arena_device_body(tgsim_ctx* c, const uint32_t** inst, const int64_t** t, const uint64_t** off,
                                        const uint32_t** len, const uint8_t** payload, size_t* n) {
  if (!c) return TGSIM_EINVAL;
  if (inst) *inst = c->tp_inst;
  if (t) *t = c->tp_t;
  if (off) *off = c->tp_off;
  if (len) *len = c->tp_len;
  if (payload) *payload = c->tp_bytes;
  if (n) *n = c->tp_n;
  return TGSIM_OK;
}

// ============================== TCP mode ===================================
// Host side of tgsim_tcp_*: segmentation (tgsim_tcp_send stages the packets), the reaction after
// every window (tgsim_tcp.hip; one synchronisation reads the retransmissions pending), the write
// table. Oracle twin: tgo_tcp_*.

namespace {
__global__ void k_fill_i64(int64_t* p, size_t n, int64_t v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
}  // namespace

static int tgsim_tcp_enable_body(tgsim_ctx* c, const tgsim_tcp_config* cfg);
extern "C" int tgsim_tcp_enable(tgsim_ctx* c, const tgsim_tcp_config* cfg) {
  return abi_guard(c, [&] { return tgsim_tcp_enable_body(c, cfg); });
}
static int tgsim_tcp_enable_body(tgsim_ctx* c, const tgsim_tcp_config* cfg) {
  if (!c || !cfg) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (int rc = need_transport(c)) return rc;  // sharded: every reaction forwards arrivals (collective)
  if (c->in_window || c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode already on or inside a window");
  if (c->n_staged || c->staged_dev) return fail(c, TGSIM_ESTATE, "messages already staged");
  if (!c->fl_off.empty()) return fail(c, TGSIM_ESTATE, "a flood graph is installed: TCP mode and floods exclude each other");
  if (c->probes) return fail(c, TGSIM_ESTATE, "probes are set up: probes run in message mode");
  if (c->storm_on) return fail(c, TGSIM_ESTATE, "a storm reactor is set up: it runs in message mode");
  tgsim_tcp_config t = *cfg;
  if (!t.mss) t.mss = 1448;
  if (!t.header_bytes) t.header_bytes = 52;
  if (!t.rto_ns) t.rto_ns = 200000000;
  if (!t.max_attempts) t.max_attempts = 16;
  if (!t.max_writes) t.max_writes = 1u << 22;
  if (!t.max_segments) t.max_segments = 1u << 24;
  if (t.max_attempts > 16 || t.rto_ns < 0 || t.max_segments > (1u << 28) || t.max_writes > (1u << 28) || t.acks > 1 ||
      (t.acks && t.max_segments > (1u << 27)))
    return fail(c, TGSIM_EINVAL, "bad TCP configuration");
  TcpDev& d = c->td;
  if (t.acks) {
    const size_t S = t.max_segments, R = (size_t)kNSub * c->d.subcap;  // per-window deliveries
    if (dalloc(c, &d.s_done, S) || dalloc(c, &d.bm_a, R / 64 + 1) || dalloc(c, &d.ack_idx, R) ||
        dalloc(c, &d.tb, (size_t)kTcpBatches) || dalloc(c, &d.plan_lo, (size_t)kTcpBatches + 1) ||
        dalloc(c, &d.plan_off, (size_t)kTcpBatches + 1))
      return TGSIM_ENOMEM;
    HIPCK(c, hipMemsetAsync(d.s_done, 0, S, c->d.stream), "tcp init");
    d.acks = 1;
    c->d.bkt_load = 2;  // every data packet is answered by an ACK: twice the copies per key
  }
  const size_t W = t.max_writes, S = t.max_segments;
  if (dalloc(c, &d.w_src, W) || dalloc(c, &d.w_dst, W) || dalloc(c, &d.w_rem, W) || dalloc(c, &d.w_state, W) ||
      dalloc(c, &d.w_tarr, W) || dalloc(c, &d.w_tmax, W) || dalloc(c, &d.w_fail, W) || dalloc(c, &d.s_w, S) || dalloc(c, &d.s_wire, S) ||
      dalloc(c, &d.s_att, S) || dalloc(c, &d.s_out, S) || dalloc(c, &d.s_mark, S) ||
      dalloc(c, &d.s_tatt, S) || dalloc(c, &d.s_arr, S) || dalloc(c, &d.s_tlast, S) || dalloc(c, &d.pend[0], S) ||
      dalloc(c, &d.pend[1], S) || dalloc(c, &d.pend_by, (size_t)c->N) || 
      dalloc(c, &d.bm_s, (size_t)c->d.cap_msgs / 64 + 1) || dalloc(c, &d.bm_r, (size_t)kNSub * c->d.subcap / 64 + 1) ||
      dalloc(c, &d.bm_d, (size_t)kNSub * c->d.subcap / 64 + 1) || dalloc(c, &d.part, (size_t)kTcpArriveBlocks) ||
      dalloc(c, &d.sc, (size_t)1))
    return TGSIM_ENOMEM;
  hipStream_t st = c->d.stream;
  HIPCK(c, hipMemsetAsync(d.w_state, 0, W * 4, st), "tcp init");
  HIPCK(c, hipMemsetAsync(d.s_att, 0, S * 4, st), "tcp init");
  HIPCK(c, hipMemsetAsync(d.s_out, 0, S * 4, st), "tcp init");
  HIPCK(c, hipMemsetAsync(d.s_mark, 0, S * 4, st), "tcp init");
  HIPCK(c, hipMemsetAsync(d.sc, 0, sizeof(TcpScalars), st), "tcp init");
  HIPCK(c, hipMemsetAsync(d.pend_by, 0, (size_t)c->N * 4, st), "tcp init");
  hipLaunchKernelGGL(k_fill_i64, dim3(1024), dim3(256), 0, st, d.w_tarr, W, INT64_MIN);
  hipLaunchKernelGGL(k_fill_i64, dim3(1024), dim3(256), 0, st, d.w_tmax, W, INT64_MIN);
  hipLaunchKernelGGL(k_fill_i64, dim3(1024), dim3(256), 0, st, d.w_fail, W, INT64_MAX);
  hipLaunchKernelGGL(k_fill_i64, dim3(1024), dim3(256), 0, st, d.s_arr, S, INT64_MAX);
  hipLaunchKernelGGL(k_fill_i64, dim3(1024), dim3(256), 0, st, d.s_tlast, S, INT64_MIN);
  HIPCK(c, hipGetLastError(), "tcp init");
  HIPCK(c, hipStreamSynchronize(st), "tcp init");
  if (hipHostMalloc((void**)&c->tcp_snap, 2 * sizeof(TcpScalars), hipHostMallocDefault) != hipSuccess)
    return fail(c, TGSIM_ENOMEM, "pinned TCP snapshots");
  for (hipEvent_t& e : c->tcp_ev) HIPCK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), "tcp init");
  d.mss = t.mss; d.hdr = t.header_bytes; d.max_att = t.max_attempts; d.rto = t.rto_ns; d.cap_w = W; d.cap_s = S;
  d.S = c->S; d.shard = c->shard; d.N = c->N; d.lo = c->lo; d.nloc = c->nloc; d.xcap = c->d.xcap; d.inv = shard_inv(c->N);
  d.xq = c->d.qc + ((size_t)3 * kNSub << 5);  // the exchange cursors' lines (idle between windows)
  d.xsend = c->d.xsend; d.xrecv = c->d.xrecv;
  c->tcp = t;
  c->tcp_on = true;
  c->tcp_hash = fnv1a(0xCBF29CE484222325ull, &t, sizeof(t)) | 1u;
  return TGSIM_OK;
}

static int tgsim_tcp_send_body(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n);
extern "C" int tgsim_tcp_send(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  return abi_guard(c, [&] { return tgsim_tcp_send_body(c, m, n); });
}
static int tgsim_tcp_send_body(tgsim_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (!c || !m) return TGSIM_EINVAL;
  c->spec.valid = false;
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->S != 1) return fail(c, TGSIM_ENOTSUP, "sharded TCP mode carries generated storm rounds (tgsim_tcp_gen_storm_round) only");
  if (c->td.n_conn) return fail(c, TGSIM_ESTATE, "a context with connections writes through tgsim_tcp_write");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tgsim_tcp_react after every window");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  if (!n) return TGSIM_OK;
  size_t nseg = 0;
  for (size_t i = 0; i < n; ++i) {
    if (m->src[i] >= c->N || m->dst[i] >= c->N) return fail(c, TGSIM_EINVAL, "write %zu: bad instance id", i);
    if (m->t_send[i] < c->horizon) return fail(c, TGSIM_ECAUSALITY, "write %zu: t_send before the horizon", i);
    if (m->size[i] >= 0x80000000u) return fail(c, TGSIM_EINVAL, "write %zu: size too large", i);
    nseg += m->size[i] ? (m->size[i] + c->tcp.mss - 1) / c->tcp.mss : 1;
  }
  if (c->tw_n + n > c->tcp.max_writes || c->tsg_n + nseg > c->tcp.max_segments)
    return fail(c, TGSIM_ECAPACITY, "TCP write / segment capacity");
  // write table (src, dst, segments left), segment table (write, wire size, attempt-0 time) and the
  // packets, built on the host: the segment count of every write is known here
  std::vector<uint32_t> w3(3 * n), s2(2 * nseg), p_src(nseg), p_dst(nseg), p_seq(nseg), p_size(nseg);
  std::vector<int64_t> s_t(nseg);
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t size = m->size[i], ns = size ? (size + c->tcp.mss - 1) / c->tcp.mss : 1;
    w3[i] = m->src[i]; w3[n + i] = m->dst[i]; w3[2 * n + i] = ns;
    for (uint32_t j = 0; j < ns; ++j, ++k) {
      const uint32_t pay = size ? (j + 1 < ns ? c->tcp.mss : size - j * c->tcp.mss) : 0;
      const uint32_t sid = (uint32_t)(c->tsg_n + k);
      // the write, and whether this is its only segment (tgsim_tcp.hip kSoleSeg)
      s2[k] = (uint32_t)(c->tw_n + i) | (ns == 1 ? 0x80000000u : 0u);
      s2[nseg + k] = pay + c->tcp.header_bytes; s_t[k] = m->t_send[i];
      p_src[k] = m->src[i]; p_dst[k] = m->dst[i]; p_seq[k] = sid << 4; p_size[k] = pay + c->tcp.header_bytes;
    }
  }
  // the packets first: enqueue_host's capacity and validation checks decide whether the writes
  // exist, so the tables below are uploaded only for writes the host counts
  tgsim_msg_soa p{p_src.data(), p_dst.data(), p_seq.data(), p_size.data(), s_t.data()};
  int rc = enqueue_host(c, &p, nseg);
  if (rc) return rc;
  uint8_t* pin = nullptr;
  rc = pin_acquire(c, c->pin_tcp, 12 * n + 16 * nseg, &pin);
  if (rc) return rc;
  memcpy(pin, s_t.data(), 8 * nseg);
  memcpy(pin + 8 * nseg, w3.data(), 12 * n);
  memcpy(pin + 8 * nseg + 12 * n, s2.data(), 8 * nseg);
  TcpDev& d = c->td;
  hipStream_t st = c->d.stream;
  const uint8_t* pw = pin + 8 * nseg;
  const uint8_t* ps = pw + 12 * n;
  HIPCK(c, hipMemcpyAsync(d.s_tatt + c->tsg_n, pin, 8 * nseg, hipMemcpyHostToDevice, st), "tcp send");
  HIPCK(c, hipMemcpyAsync(d.w_src + c->tw_n, pw, 4 * n, hipMemcpyHostToDevice, st), "tcp send");
  HIPCK(c, hipMemcpyAsync(d.w_dst + c->tw_n, pw + 4 * n, 4 * n, hipMemcpyHostToDevice, st), "tcp send");
  HIPCK(c, hipMemcpyAsync(d.w_rem + c->tw_n, pw + 8 * n, 4 * n, hipMemcpyHostToDevice, st), "tcp send");
  HIPCK(c, hipMemcpyAsync(d.s_w + c->tsg_n, ps, 4 * nseg, hipMemcpyHostToDevice, st), "tcp send");
  HIPCK(c, hipMemcpyAsync(d.s_wire + c->tsg_n, ps + 4 * nseg, 4 * nseg, hipMemcpyHostToDevice, st), "tcp send");
  rc = pin_issued(c, c->pin_tcp);
  if (rc) return rc;
  c->tw_n += n;
  c->tsg_n += nseg;
  c->tstats.writes += n;
  c->tstats.segments += nseg;
  c->tstats.packets += nseg;
  return TGSIM_OK;
}

static int tcp_refresh(tgsim_ctx* c);

static int tgsim_tcp_react_body(tgsim_ctx* c, size_t* n_done);
extern "C" int tgsim_tcp_react(tgsim_ctx* c, size_t* n_done) {
  return abi_guard(c, [&] { return tgsim_tcp_react_body(c, n_done); });
}
// The TCP counters into the next pinned snapshot, behind the work queued on the stream
static int tcp_snapshot(tgsim_ctx* c) {
  const uint32_t k = c->tcp_snap_slot;
  HIPCK(c, hipMemcpyAsync(&c->tcp_snap[k], c->td.sc, sizeof(TcpScalars), hipMemcpyDeviceToHost, c->d.stream),
        "tcp snapshot");
  HIPCK(c, hipEventRecord(c->tcp_ev[k], c->d.stream), "tcp snapshot");
  c->tcp_snap_cur[k] = c->tcp_cur;
  c->tcp_snap_live[k] = true;
  c->tcp_snap_slot = k ^ 1u;
  return TGSIM_OK;
}

static int tgsim_tcp_react_body(tgsim_ctx* c, size_t* n_done) {
  if (n_done) *n_done = 0;
  if (!c) return TGSIM_EINVAL;
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (!c->tcp_need_react) return TGSIM_OK;
  const bool on_dev = c->n_status_last == kStatusOnDevice;
  if (c->S > 1) {  // the data copies delivered here for other shards' writers go to them (collective)
    if (int rc = need_transport(c)) return rc;
    HIPCK(c, launch_tcp_fwd(c->d, c->td), "tcp forward");
    if (c->tr.alltoall(c->tr.user, c->d.xsend, c->d.xrecv, (size_t)c->d.xcap * sizeof(tgsim_record), c->d.stream) != 0)
      return shard_failed(c, fail(c, TGSIM_EHIP, "transport all-to-all failed"));
  }
  HIPCK(c, launch_tcp_react(c->d, c->td, c->tcp_cur, on_dev ? 0u : c->n_status_last,
                            on_dev ? &c->d.sc->n_msgs_last : nullptr, ++c->tcp_epoch, c->tcp_fill), "tcp react");
  if (c->td.n_conn) {  // the window's ACKs open the connections' windows: send what fits, at its end
    HIPCK(c, launch_tcp_conn_release(c->d, c->td, kRelAfterWindow, c->tcp_cur, c->staged_dev, c->n_staged), "tcp release");
    c->staged_dev = true;
  }
  c->tcp_fill = ~0u;
  c->tcp_need_react = false;
  const uint32_t k = c->tcp_snap_slot;
  if (int rc = tcp_snapshot(c)) return rc;
  if (!n_done) return TGSIM_OK;  // asynchronous: the counters arrive with a later synchronising call
  int rc = sync_and_check(c);
  if (rc) return rc;
  const uint32_t done = c->tcp_snap[k].done;
  rc = tcp_refresh(c);
  if (rc) return rc;
  *n_done = done;
  return TGSIM_OK;
}

// The TCP counters from the newest completed snapshot.
static int tcp_refresh(tgsim_ctx* c) {
  const uint32_t latest = c->tcp_snap_slot ^ 1u, older = c->tcp_snap_slot;
  for (uint32_t k : {latest, older}) {
    if (!c->tcp_snap_live[k]) continue;
    const hipError_t q = hipEventQuery(c->tcp_ev[k]);
    if (q == hipErrorNotReady) continue;
    HIPCK(c, q, "tcp snapshot");
    const TcpScalars& ts = c->tcp_snap[k];
    c->tstats.retransmissions = ts.retx;
    c->tstats.delivered = ts.delivered;
    c->tstats.failed = ts.failed;
    c->tstats.pending_retx = c->tcp.acks ? 0 : ts.pend_n[c->tcp_snap_cur[k]];  // acks: timers, not a pending list
    c->tstats.packets = c->tstats.segments + ts.released;
    c->tcp_snap_live[k] = false;
    if (k == latest) c->tcp_snap_live[older] = false;  // superseded (an older one leaves the latest in flight)
    break;
  }
  return TGSIM_OK;
}

static int tgsim_tcp_writes_body(tgsim_ctx* c, uint8_t* state, int64_t* t, size_t cap, size_t* n);
extern "C" int tgsim_tcp_writes(tgsim_ctx* c, uint8_t* state, int64_t* t, size_t cap, size_t* n) {
  return abi_guard(c, [&] { return tgsim_tcp_writes_body(c, state, t, cap, n); });
}
static int tgsim_tcp_writes_body(tgsim_ctx* c, uint8_t* state, int64_t* t, size_t cap, size_t* n) {
  if (!c || !n) return TGSIM_EINVAL;
  *n = c->tw_n;
  if (!c->tcp_on) return TGSIM_OK;
  if (c->tw_n > cap) return fail(c, TGSIM_ECAPACITY, "write capacity");
  int rc = sync_and_check(c);
  if (rc) return rc;
  const size_t W = c->tw_n;
  std::vector<uint32_t> st(W);
  std::vector<int64_t> ta(W), tf(W);
  if (W) {
    HIPCK(c, hipMemcpy(st.data(), c->td.w_state, W * 4, hipMemcpyDeviceToHost), "tcp writes");
    HIPCK(c, hipMemcpy(ta.data(), c->td.w_tarr, W * 8, hipMemcpyDeviceToHost), "tcp writes");
    HIPCK(c, hipMemcpy(tf.data(), c->td.w_fail, W * 8, hipMemcpyDeviceToHost), "tcp writes");
  }
  for (size_t i = 0; i < W; ++i) {
    // a failed write reports its earliest failure (key t * 2 + timeout), whatever failed first
    // a delivered write is marked by its time alone (tgsim_tcp.hip tcp_arrived)
    uint32_t s_i = ta[i] != INT64_MIN ? (uint32_t)TGSIM_TCP_DELIVERED : st[i];
    int64_t t_i = ta[i];
    if (s_i != TGSIM_TCP_PENDING && s_i != TGSIM_TCP_DELIVERED) {
      t_i = tf[i] >> 1;
      s_i = (tf[i] & 1) ? TGSIM_TCP_TIMEOUT : TGSIM_TCP_REFUSED;
    } else if (s_i == TGSIM_TCP_PENDING) {
      t_i = INT64_MIN;
    }
    if (state) state[i] = (uint8_t)s_i;
    if (t) t[i] = t_i;
  }
  return TGSIM_OK;
}

static int tgsim_tcp_get_stats_body(tgsim_ctx* c, tgsim_tcp_stats* out);
extern "C" int tgsim_tcp_get_stats(tgsim_ctx* c, tgsim_tcp_stats* out) {
  return abi_guard(c, [&] { return tgsim_tcp_get_stats_body(c, out); });
}
static int tgsim_tcp_get_stats_body(tgsim_ctx* c, tgsim_tcp_stats* out) {
  if (!c || !out) return TGSIM_EINVAL;
  if (c->tcp_on && (c->tcp_snap_live[0] || c->tcp_snap_live[1])) {  // an asynchronous reaction: its counters
    int rc = sync_and_check(c);
    if (rc) return rc;
    rc = tcp_refresh(c);
    if (rc) return rc;
  }
  *out = c->tstats;
  return TGSIM_OK;
}

static int tgsim_tcp_gen_storm_round_body(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                                         int64_t spread_ns, uint32_t state);
extern "C" int tgsim_tcp_gen_storm_round(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                                         int64_t spread_ns, uint32_t state) {
  return abi_guard(c, [&] { return tgsim_tcp_gen_storm_round_body(c, round, t0, fanout, size, spread_ns, state); });
}
static int tgsim_tcp_gen_storm_round_body(tgsim_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                                         int64_t spread_ns, uint32_t state) {
  if (!c) return TGSIM_EINVAL;
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->td.n_conn) return fail(c, TGSIM_ESTATE, "a context with connections writes through tgsim_tcp_write");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tgsim_tcp_react after every window");
  if (size > c->tcp.mss) return fail(c, TGSIM_EINVAL, "a storm write must fit one segment");
  if (fanout == 0 || fanout > 32) return fail(c, TGSIM_EINVAL, "bad fanout");
  const uint64_t n = (uint64_t)c->nloc * fanout;
  if (c->tw_n + n > c->tcp.max_writes || c->tsg_n + n > c->tcp.max_segments)
    return fail(c, TGSIM_ECAPACITY, "TCP write / segment capacity");
  if (c->S != 1) {  // the single run's segment ids on the wire (tgsim_tcp.hip tcp_wire): one fanout, 27/28 bits
    if (c->td.F && c->td.F != fanout) return fail(c, TGSIM_ENOTSUP, "sharded TCP storms keep one fanout");
    const uint64_t rounds = c->tsg_n / n + 1;
    if (rounds * c->N * fanout > (c->tcp.acks ? (1ull << 27) : (1ull << 28)))
      return fail(c, TGSIM_ECAPACITY, "TCP segment ids beyond the packets' seq bits");
    c->td.F = fanout;
  }
  const uint32_t base = c->n_staged;
  int rc = gen_storm_impl(c, round, t0, fanout, size, spread_ns, state);
  if (rc) return rc;
  HIPCK(c, launch_tcp_adopt(c->d, c->td, base, (uint32_t)n, (uint32_t)c->tw_n, (uint32_t)c->tsg_n), "tcp adopt");
  c->tw_n += n;
  c->tsg_n += n;
  c->tstats.writes += n;
  c->tstats.segments += n;
  c->tstats.packets += n;
  return TGSIM_OK;
}

// ---- TCP connections: congestion window and ACK clocking -------------------

static int tgsim_tcp_writes_range_body(tgsim_ctx* c, uint64_t first, size_t n, uint8_t* state, int64_t* t);
extern "C" int tgsim_tcp_writes_range(tgsim_ctx* c, uint64_t first, size_t n, uint8_t* state, int64_t* t) {
  return abi_guard(c, [&] { return tgsim_tcp_writes_range_body(c, first, n, state, t); });
}
static int tgsim_tcp_writes_range_body(tgsim_ctx* c, uint64_t first, size_t n, uint8_t* state, int64_t* t) {
  if (!c) return TGSIM_EINVAL;
  if (first + n > c->tw_n) return fail(c, TGSIM_EINVAL, "writes [%llu, +%zu) out of range", (unsigned long long)first, n);
  if (!n || !c->tcp_on) return TGSIM_OK;
  int rc = sync_and_check(c);
  if (rc) return rc;
  std::vector<uint32_t> st(n);
  std::vector<int64_t> ta(n), tf(n);
  HIPCK(c, hipMemcpy(st.data(), c->td.w_state + first, n * 4, hipMemcpyDeviceToHost), "tcp writes");
  HIPCK(c, hipMemcpy(ta.data(), c->td.w_tarr + first, n * 8, hipMemcpyDeviceToHost), "tcp writes");
  HIPCK(c, hipMemcpy(tf.data(), c->td.w_fail + first, n * 8, hipMemcpyDeviceToHost), "tcp writes");
  for (size_t i = 0; i < n; ++i) {  // the decoding of tgsim_tcp_writes
    uint32_t s_i = ta[i] != INT64_MIN ? (uint32_t)TGSIM_TCP_DELIVERED : st[i];
    int64_t t_i = ta[i];
    if (s_i != TGSIM_TCP_PENDING && s_i != TGSIM_TCP_DELIVERED) {
      t_i = tf[i] >> 1;
      s_i = (tf[i] & 1) ? TGSIM_TCP_TIMEOUT : TGSIM_TCP_REFUSED;
    } else if (s_i == TGSIM_TCP_PENDING) {
      t_i = INT64_MIN;
    }
    if (state) state[i] = (uint8_t)s_i;
    if (t) t[i] = t_i;
  }
  return TGSIM_OK;
}

// grow the device connection arrays to hold `need` connections (copying the live ones)
static int conn_grow(tgsim_ctx* c, uint32_t need) {
  TcpDev& t = c->td;
  if (need <= c->conn_cap) return TGSIM_OK;
  const uint32_t cap = std::max<uint32_t>({need, 2 * c->conn_cap, 1024u});
  HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
  uint32_t** u32[] = {&t.c_src, &t.c_dst, &t.c_cwnd, &t.c_ssth, &t.c_cnt, &t.c_flight, &t.c_queued, &t.c_head,
                      &t.c_acks, &t.c_broken, &t.c_una, &t.c_fack, &t.c_fr};
  for (uint32_t** a : u32)
    if (dgrow(c, a, t.n_conn, cap)) return TGSIM_ENOMEM;
  if (dgrow(c, &t.c_acked, t.n_conn, cap) || dgrow(c, &t.c_tloss, t.n_conn, cap) || dgrow(c, &t.c_tack, t.n_conn, cap))
    return TGSIM_ENOMEM;
  c->conn_cap = cap;
  return TGSIM_OK;
}

static int tgsim_tcp_connect_body(tgsim_ctx* c, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* out);
extern "C" int tgsim_tcp_connect(tgsim_ctx* c, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* out) {
  return abi_guard(c, [&] { return tgsim_tcp_connect_body(c, src, dst, n, out); });
}
static int tgsim_tcp_connect_body(tgsim_ctx* c, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* out) {
  if (!c) return TGSIM_EINVAL;
  if (c->storm_on) return fail(c, TGSIM_ESTATE, "a storm reactor owns the connections");
  if (!c->tcp_on || !c->tcp.acks) return fail(c, TGSIM_ESTATE, "connections need TCP mode with acks = 1");
  if (c->S != 1) return fail(c, TGSIM_ENOTSUP, "connections (their ACK clock) need a single-shard context");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->tw_n && !c->td.n_conn) return fail(c, TGSIM_ESTATE, "tcp_send writes exist: a context uses one or the other");
  if (n && (!src || !dst)) return fail(c, TGSIM_EINVAL, "bad arguments");
  for (size_t i = 0; i < n; ++i)
    if (src[i] >= c->N || dst[i] >= c->N) return fail(c, TGSIM_EINVAL, "connection %zu: bad instance id", i);
  TcpDev& t = c->td;
  if ((uint64_t)t.n_conn + n > c->tcp.max_writes) return fail(c, TGSIM_ECAPACITY, "connection capacity");
  if (!n) return TGSIM_OK;
  alloc_point(c);
  if (!t.w_conn) {  // first connection: the per-write / per-segment connection tables
    const size_t W = c->tcp.max_writes, S = c->tcp.max_segments;
    if (dalloc(c, &t.w_conn, W) || dalloc(c, &t.s_next, S) || dalloc(c, &t.s_ack1, S) || dalloc(c, &t.s_lost, S) ||
        dalloc(c, &t.s_tq, S))
      return TGSIM_ENOMEM;
    HIPCK(c, hipMemsetAsync(t.s_ack1, 0, S * 4, c->d.stream), "tcp connect");
    HIPCK(c, hipMemsetAsync(t.s_lost, 0, S, c->d.stream), "tcp connect");
    HIPCK(c, hipMemsetAsync(t.s_tq, 0, S, c->d.stream), "tcp connect");
  }
  const uint32_t n0 = t.n_conn, n1 = (uint32_t)(n0 + n);
  int rc = conn_grow(c, n1);
  if (rc) return rc;
  std::vector<uint32_t> a(src, src + n), b(dst, dst + n), iw(n, 10u), ss(n, 0x7FFFFFFFu), none(n, 0xFFFFFFFFu);
  std::vector<int64_t> never(n, INT64_MAX), none_t(n, INT64_MIN);
  hipStream_t st = c->d.stream;
  HIPCK(c, hipMemcpyAsync(t.c_src + n0, a.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_dst + n0, b.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_cwnd + n0, iw.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_ssth + n0, ss.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_head + n0, none.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_una + n0, none.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_tloss + n0, never.data(), n * 8, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_fr + n0, none.data(), n * 4, hipMemcpyHostToDevice, st), "tcp connect");
  HIPCK(c, hipMemcpyAsync(t.c_tack + n0, none_t.data(), n * 8, hipMemcpyHostToDevice, st), "tcp connect");
  for (uint32_t* z : {t.c_cnt, t.c_flight, t.c_queued, t.c_acks, t.c_broken, t.c_fack})
    HIPCK(c, hipMemsetAsync(z + n0, 0, n * 4, st), "tcp connect");
  HIPCK(c, hipMemsetAsync(t.c_acked + n0, 0, n * 8, st), "tcp connect");
  HIPCK(c, hipStreamSynchronize(st), "tcp connect");  // the host vectors go out of scope
  c->conn_src.insert(c->conn_src.end(), src, src + n);
  c->conn_dst.insert(c->conn_dst.end(), dst, dst + n);
  c->conn_tail.resize(n1, 0xFFFFFFFFu);
  for (size_t i = 0; i < n; ++i)
    if (out) out[i] = n0 + (uint32_t)i;
  t.n_conn = n1;
  return TGSIM_OK;
}

static int tgsim_tcp_write_body(tgsim_ctx* c, const uint32_t* conn, const uint32_t* size, const int64_t* t_send, size_t n);
extern "C" int tgsim_tcp_write(tgsim_ctx* c, const uint32_t* conn, const uint32_t* size, const int64_t* t_send, size_t n) {
  return abi_guard(c, [&] { return tgsim_tcp_write_body(c, conn, size, t_send, n); });
}
static int tgsim_tcp_write_body(tgsim_ctx* c, const uint32_t* conn, const uint32_t* size, const int64_t* t_send,
                                size_t n) {
  if (!c) return TGSIM_EINVAL;
  c->spec.valid = false;
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tgsim_tcp_react after every window");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->storm_on) return fail(c, TGSIM_ESTATE, "a storm reactor owns the connections");
  if (n && (!conn || !size || !t_send)) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (c->now_from_device) { int rc = sync_and_check(c); if (rc) return rc; }
  TcpDev& td = c->td;
  size_t nseg = 0;
  for (size_t i = 0; i < n; ++i) {
    if (conn[i] >= td.n_conn) return fail(c, TGSIM_EINVAL, "write %zu: no connection %u", i, conn[i]);
    if (conn[i] >= c->storm_conn_lo && conn[i] < c->storm_conn_hi)
      return fail(c, TGSIM_ESTATE, "write %zu: connection %u was a storm reactor's", i, conn[i]);
    if (t_send[i] < c->horizon) return fail(c, TGSIM_ECAUSALITY, "write %zu: t_send before the horizon", i);
    if (size[i] >= 0x80000000u) return fail(c, TGSIM_EINVAL, "write %zu: size too large", i);
    nseg += size[i] ? (size[i] + c->tcp.mss - 1) / c->tcp.mss : 1;
  }
  if (c->tw_n + n > c->tcp.max_writes || c->tsg_n + nseg > c->tcp.max_segments)
    return fail(c, TGSIM_ECAPACITY, "TCP write / segment capacity");
  if (!n) return TGSIM_OK;
  alloc_point(c);
  // write table (src, dst, segments, connection), segment table (write | sole, wire size, written
  // at, next on the connection) and one link per touched connection
  std::vector<uint32_t> w4(4 * n), s3(3 * nseg);
  std::vector<int64_t> s_t(nseg);
  std::vector<uint32_t> tail = c->conn_tail;  // updated copy: committed once the uploads are issued
  std::unordered_map<uint32_t, uint32_t> link_of;  // connection -> its quad
  std::vector<uint32_t> quads;
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t cn = conn[i], sz = size[i], ns = sz ? (sz + c->tcp.mss - 1) / c->tcp.mss : 1;
    const uint32_t wi = (uint32_t)(c->tw_n + i);
    w4[i] = c->conn_src[cn]; w4[n + i] = c->conn_dst[cn]; w4[2 * n + i] = ns; w4[3 * n + i] = cn;
    for (uint32_t j = 0; j < ns; ++j, ++k) {
      const uint32_t pay = sz ? (j + 1 < ns ? c->tcp.mss : sz - j * c->tcp.mss) : 0;
      const uint32_t sid = (uint32_t)(c->tsg_n + k);
      s3[k] = wi | (ns == 1 ? 0x80000000u : 0u);
      s3[nseg + k] = pay + c->tcp.header_bytes;
      s3[2 * nseg + k] = 0xFFFFFFFFu;
      s_t[k] = t_send[i];
      auto it = link_of.find(cn);
      if (it == link_of.end()) {  // the batch's first segment on cn: linked to the device queue
        link_of.emplace(cn, (uint32_t)(quads.size() / 4));
        quads.insert(quads.end(), {cn, tail[cn], sid, 0u});
      } else {                    // chained to the batch's previous segment on cn, here
        s3[2 * nseg + (tail[cn] - (uint32_t)c->tsg_n)] = sid;
      }
      quads[4 * link_of[cn] + 3] += 1;
      tail[cn] = sid;
    }
  }
  uint8_t* pin = nullptr;
  int rc = pin_acquire(c, c->pin_tcp, 16 * n + 20 * nseg + 4 * quads.size(), &pin);
  if (rc) return rc;
  uint8_t* pt = pin;
  uint8_t* pw = pt + 8 * nseg;
  uint8_t* ps = pw + 16 * n;
  uint8_t* pq = ps + 12 * nseg;
  memcpy(pt, s_t.data(), 8 * nseg);
  memcpy(pw, w4.data(), 16 * n);
  memcpy(ps, s3.data(), 12 * nseg);
  memcpy(pq, quads.data(), 4 * quads.size());
  const uint32_t nq = (uint32_t)(quads.size() / 4);
  if (quads.size() > c->link_cap) {
    HIPCK(c, hipStreamSynchronize(c->d.stream), "sync");
    dfree(c, c->link_dev);
    c->link_dev = nullptr;
    const size_t cap = std::max<size_t>(quads.size(), 2 * c->link_cap);
    if (dalloc(c, &c->link_dev, cap)) return TGSIM_ENOMEM;
    c->link_cap = cap;
  }
  hipStream_t st = c->d.stream;
  const uint64_t w0 = c->tw_n, s0 = c->tsg_n;
  HIPCK(c, hipMemcpyAsync(td.s_tatt + s0, pt, 8 * nseg, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.w_src + w0, pw, 4 * n, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.w_dst + w0, pw + 4 * n, 4 * n, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.w_rem + w0, pw + 8 * n, 4 * n, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.w_conn + w0, pw + 12 * n, 4 * n, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.s_w + s0, ps, 4 * nseg, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.s_wire + s0, ps + 4 * nseg, 4 * nseg, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(td.s_next + s0, ps + 8 * nseg, 4 * nseg, hipMemcpyHostToDevice, st), "tcp write");
  HIPCK(c, hipMemcpyAsync(c->link_dev, pq, 4 * quads.size(), hipMemcpyHostToDevice, st), "tcp write");
  rc = pin_issued(c, c->pin_tcp);
  if (rc) return rc;
  HIPCK(c, launch_tcp_link(c->d, td, c->link_dev, nq), "tcp write");
  // the windows' room goes now, at the write times
  HIPCK(c, launch_tcp_conn_release(c->d, td, kRelAtWrite, c->tcp_cur, c->staged_dev, c->n_staged), "tcp write");
  c->staged_dev = true;
  c->conn_tail.swap(tail);
  for (size_t i = 0; i < n; ++i) {  // the queue-limit bound: a sender's new segments (any may leave now)
    const uint32_t src = c->conn_src[conn[i]];
    if (!is_local(c, src)) continue;
    const uint32_t l = src - c->lo, ns = size[i] ? (size[i] + c->tcp.mss - 1) / c->tcp.mss : 1;
    if (c->hcnt[l] == 0) c->hcnt_touched.push_back(l);
    c->hcnt[l] += ns;
    c->win_m_host = std::max(c->win_m_host, c->hcnt[l]);
    c->max_tsend_h = std::max(c->max_tsend_h, t_send[i]);
  }
  c->tw_n += n;
  c->tsg_n += nseg;
  c->tcp_seg_batched = c->tsg_n;  // no timer batches: released segments' timers ride the pend lists
  c->tstats.writes += n;
  c->tstats.segments += nseg;
  return TGSIM_OK;
}

static int tgsim_tcp_conns_body(tgsim_ctx* c, uint32_t first, size_t n, uint64_t* acked, uint32_t* cwnd,
                                uint32_t* flight, uint32_t* queued);
extern "C" int tgsim_tcp_conns(tgsim_ctx* c, uint32_t first, size_t n, uint64_t* acked, uint32_t* cwnd,
                               uint32_t* flight, uint32_t* queued) {
  return abi_guard(c, [&] { return tgsim_tcp_conns_body(c, first, n, acked, cwnd, flight, queued); });
}
static int tgsim_tcp_conns_body(tgsim_ctx* c, uint32_t first, size_t n, uint64_t* acked, uint32_t* cwnd,
                                uint32_t* flight, uint32_t* queued) {
  if (!c) return TGSIM_EINVAL;
  const TcpDev& t = c->td;
  if ((uint64_t)first + n > t.n_conn) return fail(c, TGSIM_EINVAL, "connections [%u, +%zu) out of range", first, n);
  if (!n) return TGSIM_OK;
  int rc = sync_and_check(c);
  if (rc) return rc;
  if (acked) HIPCK(c, hipMemcpy(acked, t.c_acked + first, n * 8, hipMemcpyDeviceToHost), "tcp conns");
  if (cwnd) HIPCK(c, hipMemcpy(cwnd, t.c_cwnd + first, n * 4, hipMemcpyDeviceToHost), "tcp conns");
  if (flight) HIPCK(c, hipMemcpy(flight, t.c_flight + first, n * 4, hipMemcpyDeviceToHost), "tcp conns");
  if (queued) HIPCK(c, hipMemcpy(queued, t.c_queued + first, n * 4, hipMemcpyDeviceToHost), "tcp conns");
  return TGSIM_OK;
}

// ============================== window-boundary snapshot ===================================
// SURVEY.md 5 (checkpoint/resume, optional): the message path's whole state between windows as one
// opaque image - device: scalars (clock, wheel ring, counters), token buckets, queue occupancy,
// correlation states, the timing-wheel arena with its regions and slot directories, the last
// window's deliveries, the sync service (counts, times, chunks, the used part of the signal log and
// of the waiter table), the next window's staged messages, a flood's first-receipt bits, the probers'
// state, the topic logs; host: the configuration mirrors (shapes, correlations, flags, addresses, rules, pending
// resets), the clock, the queue-limit bound and the staging counters, the flood's publication set. Device tables compiled from the host
// mirrors are re-uploaded at the next window. Randomness needs no state (Philox is counter-based).
namespace {

// "TTGSNP" + a two-digit layout version: bump it whenever snap_regions changes (round 5
// changed the pend layout under version 01, so an older image was refused only by its byte total)
constexpr uint64_t kSnapMagic = 0x3430504E53475454ull;  // "TTGSNP04": 03 + staged messages, floods, probes
constexpr uint64_t kSnapMagicMask = 0x0000FFFFFFFFFFFFull;  // "TTGSNP" without the version

struct SnapHeader {
  uint64_t magic, bytes;
  uint32_t dev_scalars, N, S, shard, nloc, slots, cap_rec, cap_msgs, max_states, max_waiters;
  uint64_t max_signals, seed, cap_arena;
  uint64_t fl_hash, probe_hash, storm_hash;  // the flood graph / probe / storm setup the image needs (0: none)
  uint64_t tcp_hash, conn_hash;  // TCP mode's configuration and its connections (0: off)
};

struct SnapWriter {  // sizing pass when p == nullptr
  uint8_t* p;
  size_t n = 0;
  void raw(const void* src, size_t k) {
    if (p) memcpy(p + n, src, k);
    n += k;
  }
  template <class T> void val(const T& v) { raw(&v, sizeof(T)); }
  template <class T> void vec(const std::vector<T>& v) {
    val<uint64_t>(v.size());
    raw(v.data(), v.size() * sizeof(T));
  }
};

struct SnapReader {
  const uint8_t* p;
  size_t n, at = 0;
  bool ok = true;
  const uint8_t* take(size_t k) {
    if (!ok || k > n - at) { ok = false; return nullptr; }
    const uint8_t* q = p + at;
    at += k;
    return q;
  }
  template <class T> T val() {
    T v{};
    if (const uint8_t* q = take(sizeof(T))) memcpy(&v, q, sizeof(T));
    return v;
  }
  template <class T> bool vec(std::vector<T>& v, size_t expect = SIZE_MAX) {
    const uint64_t k = val<uint64_t>();
    if (!ok || (expect != SIZE_MAX && k != expect) || k > (n - at) / sizeof(T)) return ok = false;
    v.resize(k);
    if (const uint8_t* q = take(k * sizeof(T))) memcpy(v.data(), q, k * sizeof(T));
    return ok;
  }
};

// the device state regions (pointer, bytes), in image order
std::vector<std::pair<void*, size_t>> snap_regions(tgsim_ctx* c) {
  Dev& d = c->d;
  const size_t nl = std::max<size_t>(c->nloc, 1), phys = (size_t)kNSub * d.subcap;
  return {
      {d.sc, sizeof(DevScalars)},
      {d.X, 8 * nl},
      {d.pend, (4 * nl) << pend_shift(c->nloc)},
      {d.cor_last, 16 * nl},
      {d.arena, sizeof(tgsim_record) * d.cap_arena},
      {d.regions, sizeof(RegionDev) * kMaxRegions},
      {d.dirs, 4ull * kMaxRegions * (d.slots + 1)},
      {d.o_t, 8 * phys}, {d.o_src, 4 * phys}, {d.o_dst, 4 * phys}, {d.o_seq, 4 * phys},
      {d.o_size, 4 * phys}, {d.o_flags, 4 * phys}, {d.o_coff, 4 * phys},
      {d.inbox, 4 * ((size_t)c->nloc + 1)},
      {d.stats, 8ull * kNSub * 16},
      {d.sig_red, 8 * 4},
      {d.st_count, 4ull * d.max_states},
      {d.st_last, 8ull * d.max_states},
      {d.st_nchunks, 4ull * d.max_states},
      {d.st_chunks, sizeof(SigChunk) * d.max_states * kMaxChunksPerState},
      {d.sig_log, 8 * c->sig_log_used},
      {d.w_state, 4ull * c->n_waiters}, {d.w_target, 4ull * c->n_waiters},
      {d.w_twait, 8ull * c->n_waiters}, {d.w_release, 8ull * c->n_waiters},
  };
}
// ... then the staged messages (a reactor stages the next window's between windows), the flood's
// first-receipt bits and the probers' state
void snap_regions_more(tgsim_ctx* c, std::vector<std::pair<void*, size_t>>& v) {
  Dev& d = c->d;
  const size_t k = c->snap_staged;
  for (auto r : std::initializer_list<std::pair<void*, size_t>>{
           {d.m_t, 8 * k}, {d.m_src, 4 * k}, {d.m_dst, 4 * k}, {d.m_seq, 4 * k}, {d.m_size, 4 * k}})
    v.push_back(r);
  if (!c->fl_off.empty()) v.push_back({d.fl.seen, 4ull * d.fl.max_pubs * d.fl.wpp});
  if (c->tcp_on) {
    const TcpDev& t = c->td;
    const size_t W = c->tw_n, S = c->tsg_n, nc = t.n_conn;
    for (auto r : std::initializer_list<std::pair<void*, size_t>>{
             {t.w_src, 4 * W}, {t.w_dst, 4 * W}, {t.w_rem, 4 * W}, {t.w_state, 4 * W}, {t.w_tarr, 8 * W},
             {t.w_tmax, 8 * W}, {t.w_fail, 8 * W}, {t.s_w, 4 * S}, {t.s_wire, 4 * S}, {t.s_att, 4 * S},
             {t.s_out, 4 * S}, {t.s_mark, 4 * S}, {t.s_tatt, 8 * S}, {t.s_arr, 8 * S}, {t.s_tlast, 8 * S},
             {t.pend[0], 4 * S}, {t.pend[1], 4 * S}, {t.pend_by, 4ull * c->N}, {t.sc, sizeof(TcpScalars)}})
      v.push_back(r);
    if (t.acks)  // the timer ring, and the last reaction's ACKs (released at the next window start)
      for (auto r : std::initializer_list<std::pair<void*, size_t>>{
               {t.s_done, S}, {t.tb, sizeof(TcpBatch) * kTcpBatches}, {t.plan_lo, 4ull * (kTcpBatches + 1)},
               {t.plan_off, 4ull * (kTcpBatches + 1)}, {t.ack_idx, 4ull * c->snap_acks}})
        v.push_back(r);
    if (t.w_conn)
      for (auto r : std::initializer_list<std::pair<void*, size_t>>{
               {t.w_conn, 4 * W}, {t.s_next, 4 * S}, {t.s_ack1, 4 * S}, {t.s_lost, S}, {t.s_tq, S},
               {t.c_src, 4 * nc}, {t.c_dst, 4 * nc}, {t.c_cwnd, 4 * nc}, {t.c_ssth, 4 * nc}, {t.c_cnt, 4 * nc},
               {t.c_flight, 4 * nc}, {t.c_queued, 4 * nc}, {t.c_head, 4 * nc}, {t.c_acks, 4 * nc},
               {t.c_broken, 4 * nc}, {t.c_acked, 8 * nc}, {t.c_tloss, 8 * nc}, {t.c_una, 4 * nc},
               {t.c_fack, 4 * nc}, {t.c_tack, 8 * nc}, {t.c_fr, 4 * nc}})
        v.push_back(r);
  }
  if (c->storm_on) {
    const StormDev& m = d.sm;
    const size_t nc = std::max<uint32_t>(m.n_conn, 1), nl = std::max<uint32_t>(c->nloc, 1);
    const size_t claim_words = std::max<uint64_t>(((uint64_t)m.n_conn * m.nchunks + 31) / 32, 1);
    for (auto r : std::initializer_list<std::pair<void*, size_t>>{
             {m.dst, 4 * nc}, {m.t_ready, 8 * nc}, {m.state, nc}, {m.flags, nc}, {m.res, nc}, {m.slot, 4 * nc},
             {m.t_start, 8 * nc}, {m.t_synarr, 8 * nc}, {m.t_ackarr, 8 * nc}, {m.t_done, 8 * nc}, {m.t_rep, 8 * nc},
             {m.emit, 4 * nc}, {m.rem, 4 * nc}, {m.infl, 4 * nc}, {m.order, 4 * nc}, {m.ring, 4 * nc},
             {m.claim, 4 * claim_words}, {m.dq, 4 * nl}, {m.qh, 4 * nl}, {m.ql, 4 * nl}, {m.nh, 4 * nl},
             {m.slot_t, 8 * nl * m.C}, {m.hold, 4 * nl * m.Hc}, {m.failed, nl}, {m.t_last, 8 * nl},
             {m.sc, sizeof(StormScalars)}, {m.ans, 4 * nc}, {m.alist, 4 * nc}})
      v.push_back(r);
    if (m.tcp) {
      v.push_back({m.settled, 4 * nc});
      v.push_back({m.wsegs, 4 * nc});
    }
  }
  if (c->tp_n)
    for (auto r : std::initializer_list<std::pair<void*, size_t>>{
             {c->tp_inst, 4 * c->tp_n}, {c->tp_t, 8 * c->tp_n}, {c->tp_off, 8 * c->tp_n}, {c->tp_len, 4 * c->tp_n},
             {c->tp_bytes, c->tp_nbytes}})
      v.push_back(r);
  if (c->probes) {
    const ProbeDev& p = d.pr;
    const size_t nl = std::max<uint32_t>(c->nloc, 1), nn = std::max<uint32_t>(c->N, 1);
    for (auto r : std::initializer_list<std::pair<void*, size_t>>{
             {p.order, 4ull * p.n_order}, {p.pos, 4 * nl}, {p.state, nl}, {p.refused, nl}, {p.replied, nl},
             {p.t_req, 8 * nl}, {p.t_rep, 8 * nl}, {p.t_reparr, 8 * nl}, {p.t_done, 8 * nl},
             {p.out, nl * p.n_order}, {p.sc, sizeof(ProbeScalars)},
             {p.ans, 4 * nn}, {p.cur, 4 * nn}, {p.alist, 4 * nn}, {p.rqa, 8 * nn}})
      v.push_back(r);
  }
}

SnapHeader snap_header(tgsim_ctx* c) {
  SnapHeader h{};
  h.magic = kSnapMagic;
  h.dev_scalars = sizeof(DevScalars);
  h.N = c->N; h.S = c->S; h.shard = c->shard; h.nloc = c->nloc; h.slots = c->d.slots;
  h.cap_rec = c->d.cap_rec; h.cap_msgs = c->d.cap_msgs; h.max_states = c->d.max_states;
  h.max_waiters = c->d.max_waiters; h.max_signals = c->d.max_signals; h.seed = c->cfg.seed;
  h.cap_arena = c->d.cap_arena;
  h.fl_hash = c->fl_off.empty() ? 0 : c->fl_hash;
  h.probe_hash = c->probes ? c->probe_hash : 0;
  h.storm_hash = c->storm_on ? c->storm_hash : 0;
  h.tcp_hash = c->tcp_on ? c->tcp_hash : 0;
  h.conn_hash = 0;
  if (c->tcp_on) {
    uint64_t k = fnv1a(0xCBF29CE484222325ull, c->conn_src.data(), c->conn_src.size() * 4);
    h.conn_hash = fnv1a(k, c->conn_dst.data(), c->conn_dst.size() * 4) ^ c->td.n_conn;
  }
  return h;
}

// the host half; the same function writes (w.p set), sizes (w.p null)
void snap_host(tgsim_ctx* c, SnapWriter& w) {
  w.vec(c->shape_h); w.vec(c->flags_h); w.vec(c->ip_h); w.vec(c->rho_h); w.vec(c->corr_epoch);
  w.vec(c->corr_reset); w.vec(c->tb_reset); w.vec(c->st_last_h);
  w.val<uint64_t>(c->moved.size());
  for (const auto& kv : c->moved) { w.val(kv.first); w.val(kv.second); }
  w.val<uint64_t>(c->rules_h.size());
  for (const auto& r : c->rules_h) w.vec(r);
  w.val(c->now); w.val(c->horizon); w.val(c->n_status_last); w.val(c->sig_log_used); w.val(c->n_waiters);
  w.val(c->pend_bound); w.val(c->pend_exact);
  // staging between windows (round 6: the reactors' staged messages are captured, not refused)
  w.val(c->snap_staged); w.val(c->n_staged); w.val(c->staged_dev);
  w.val(c->win_m_host); w.val(c->win_m_extra); w.val(c->win_m_inbox); w.val(c->win_inbox_max); w.val(c->max_tsend_h);
  w.vec(c->hcnt); w.vec(c->hcnt_touched);
  w.val(c->fl_npubs); w.vec(c->fl_pub_seen); w.val(c->life_host); w.val(c->life_mult);
  w.val(c->d.sm.phase);  // the storm reactor's phase (dials / writes; its tables are regions)
  // TCP mode: the write / segment counts (they size the regions), the reaction's list parity and
  // epoch, the timer ring's cursors, the connections' queue tails, the counters the host keeps
  w.val(c->tw_n); w.val(c->tsg_n); w.val(c->tcp_cur); w.val(c->tcp_epoch); w.val(c->tcp_nb); w.val(c->tcp_fill);
  w.val(c->tcp_seg_batched); w.vec(c->conn_tail); w.val(c->tstats); w.val(c->storm_conn_lo); w.val(c->storm_conn_hi);
  w.val(c->snap_acks);
  w.val(c->tp_n); w.val(c->tp_nbytes);  // topics: the entry arenas (regions) and each topic's runs
  w.val<uint64_t>(c->topic_runs.size());
  for (const auto& v : c->topic_runs) w.vec(v);
}

int snap_refusal(tgsim_ctx* c) {
  if (c->in_window) return fail(c, TGSIM_ESTATE, "snapshot/restore: inside a window");
  if (c->ext.n)  // read in place by the next window: the caller's buffers are not the context's
    return fail(c, TGSIM_ESTATE, "snapshot/restore: a device batch is staged in place (tgsim_enqueue_device)");
  if (c->probe_need_react) return fail(c, TGSIM_ESTATE, "snapshot/restore: probes: tgsim_probe_react first");
  if (c->storm_need_react) return fail(c, TGSIM_ESTATE, "snapshot/restore: storm: tgsim_storm_react first");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "snapshot/restore: TCP mode: tgsim_tcp_react first");
  return TGSIM_OK;
}

}  // namespace

static int tgsim_snapshot_body(tgsim_ctx* c, void* buf, size_t cap, size_t* n);
extern "C" int tgsim_snapshot(tgsim_ctx* c, void* buf, size_t cap, size_t* n) {
  return abi_guard(c, [&] { return tgsim_snapshot_body(c, buf, cap, n); });
}
static int tgsim_snapshot_body(tgsim_ctx* c, void* buf, size_t cap, size_t* n) {
  if (!c || !n) return TGSIM_EINVAL;
  int rc = snap_refusal(c);
  if (rc) return rc;
  rc = sync_and_check(c);  // commits a deferred storm batch, settles the device clock
  if (rc) return rc;
  c->snap_staged = c->staged_dev ? std::min<uint32_t>(c->d.h_sc->n_msgs_dev, c->d.cap_msgs) : c->n_staged;
  c->snap_acks = 0;
  if (c->tcp_on && c->td.acks) {
    TcpScalars ts;
    HIPCK(c, hipMemcpy(&ts, c->td.sc, sizeof(ts), hipMemcpyDeviceToHost), "snapshot");
    c->snap_acks = std::min<uint32_t>(ts.ack_n, (uint32_t)(kNSub * c->d.subcap));
  }
  auto regs = snap_regions(c);
  snap_regions_more(c, regs);
  SnapWriter sz{nullptr};
  sz.val(SnapHeader{});
  snap_host(c, sz);
  for (const auto& r : regs) sz.n += r.second;
  *n = sz.n;
  if (!buf) return TGSIM_OK;
  if (cap < sz.n) return fail(c, TGSIM_ECAPACITY, "snapshot needs %zu bytes", sz.n);
  SnapHeader h = snap_header(c);
  h.bytes = sz.n;
  SnapWriter w{static_cast<uint8_t*>(buf)};
  w.val(h);
  snap_host(c, w);
  for (const auto& r : regs) {
    if (r.second) HIPCK(c, hipMemcpyAsync(w.p + w.n, r.first, r.second, hipMemcpyDeviceToHost, c->d.stream), "snapshot");
    w.n += r.second;
  }
  HIPCK(c, hipStreamSynchronize(c->d.stream), "snapshot");
  return TGSIM_OK;
}

static int tgsim_restore_body(tgsim_ctx* c, const void* buf, size_t n);
extern "C" int tgsim_restore(tgsim_ctx* c, const void* buf, size_t n) {
  return abi_guard(c, [&] { return tgsim_restore_body(c, buf, n); });
}
static int tgsim_restore_body(tgsim_ctx* c, const void* buf, size_t n) {
  if (!c || !buf) return TGSIM_EINVAL;
  c->spec = tgsim_ctx::StormSpec{};
  int rc = snap_refusal(c);
  if (rc) return rc;
  if (c->storm_pending) return fail(c, TGSIM_ESTATE, "restore: a storm round is pending");
  SnapReader r{static_cast<const uint8_t*>(buf), n};
  const SnapHeader h = r.val<SnapHeader>(), want = snap_header(c);
  if (r.ok && h.magic != kSnapMagic && (h.magic & kSnapMagicMask) == (kSnapMagic & kSnapMagicMask))
    return fail(c, TGSIM_EINVAL, "restore: snapshot layout version %.2s, this library reads %.2s",
                reinterpret_cast<const char*>(&h.magic) + 6, reinterpret_cast<const char*>(&kSnapMagic) + 6);
  if (!r.ok || h.magic != kSnapMagic || h.bytes != n) return fail(c, TGSIM_EINVAL, "restore: not a snapshot image");
  SnapHeader hc = h;
  hc.bytes = 0;
  if (memcmp(&hc, &want, sizeof(SnapHeader)) != 0)
    return fail(c, TGSIM_EINVAL, "restore: the image was taken from a context with another configuration");
  // host half into temporaries first: a malformed image leaves the context untouched
  std::vector<ShapeDev> shape; std::vector<uint8_t> flags; std::vector<uint32_t> ip, rho, epoch, creset, treset;
  std::vector<int64_t> stlast;
  r.vec(shape, c->nloc); r.vec(flags, c->N); r.vec(ip, c->N); r.vec(rho, 4 * (size_t)c->nloc);
  r.vec(epoch, c->nloc); r.vec(creset); r.vec(treset); r.vec(stlast);
  std::unordered_map<uint32_t, uint32_t> moved;
  const uint64_t nm = r.val<uint64_t>();
  for (uint64_t i = 0; r.ok && i < nm; ++i) {
    const uint32_t k = r.val<uint32_t>();
    moved[k] = r.val<uint32_t>();
  }
  std::vector<std::vector<RuleDev>> rules(r.val<uint64_t>() == c->nloc ? c->nloc : 0);
  if (rules.size() != c->nloc) r.ok = false;
  for (auto& v : rules) r.vec(v);
  const int64_t now = r.val<int64_t>(), horizon = r.val<int64_t>();
  const uint32_t n_status_last = r.val<uint32_t>();
  const uint64_t sig_used = r.val<uint64_t>();
  const uint32_t n_waiters = r.val<uint32_t>();
  const uint64_t pend_bound = r.val<uint64_t>();
  const bool pend_exact = r.val<bool>();
  const uint32_t snap_staged = r.val<uint32_t>(), n_staged = r.val<uint32_t>();
  const bool staged_dev = r.val<bool>();
  const uint32_t win_m_host = r.val<uint32_t>();
  const uint64_t win_m_extra = r.val<uint64_t>();
  const uint32_t win_m_inbox = r.val<uint32_t>();
  const uint64_t win_inbox_max = r.val<uint64_t>();
  const int64_t max_tsend_h = r.val<int64_t>();
  std::vector<uint32_t> hcnt, hcnt_touched;
  r.vec(hcnt, c->hcnt.size()); r.vec(hcnt_touched);
  const uint32_t fl_npubs = r.val<uint32_t>();
  std::vector<uint8_t> fl_pub_seen;
  r.vec(fl_pub_seen, c->fl_pub_seen.size());
  const uint64_t life_host = r.val<uint64_t>(), life_mult = r.val<uint64_t>();
  const uint32_t storm_phase = r.val<uint32_t>();
  const uint64_t tw_n = r.val<uint64_t>(), tsg_n = r.val<uint64_t>();
  const uint32_t tcp_cur = r.val<uint32_t>(), tcp_epoch = r.val<uint32_t>(), tcp_nb = r.val<uint32_t>(),
                 tcp_fill = r.val<uint32_t>();
  const uint64_t tcp_seg_batched = r.val<uint64_t>();
  std::vector<uint32_t> conn_tail;
  r.vec(conn_tail, c->conn_tail.size());
  const tgsim_tcp_stats tstats = r.val<tgsim_tcp_stats>();
  const uint64_t storm_conn_lo = r.val<uint64_t>(), storm_conn_hi = r.val<uint64_t>();
  const uint32_t snap_acks = r.val<uint32_t>();
  if (snap_acks > (uint64_t)kNSub * c->d.subcap || (snap_acks && !(c->tcp_on && c->td.acks))) r.ok = false;
  if (c->tcp_on && (tw_n > c->tcp.max_writes || tsg_n > c->tcp.max_segments)) r.ok = false;
  const uint64_t tp_n = r.val<uint64_t>(), tp_nbytes = r.val<uint64_t>();
  std::vector<std::vector<tgsim_ctx::TopicRun>> runs(std::min<uint64_t>(r.val<uint64_t>(), r.ok ? (uint64_t)c->d.max_states : 0));
  for (auto& v : runs) {
    r.vec(v);
    for (const auto& x : v)
      if (x.entry + x.len > tp_n) r.ok = false;
  }
  if (!r.ok || sig_used > c->d.max_signals || n_waiters > c->d.max_waiters || snap_staged > c->d.cap_msgs ||
      n_staged > c->d.cap_msgs || (!staged_dev && snap_staged != n_staged))
    return fail(c, TGSIM_EINVAL, "restore: truncated or inconsistent image");
  for (uint32_t l : hcnt_touched)
    if (l >= hcnt.size()) return fail(c, TGSIM_EINVAL, "restore: truncated or inconsistent image");
  const uint64_t sig_used0 = c->sig_log_used;
  const uint32_t n_waiters0 = c->n_waiters;
  if (tp_n > 0xFFFFFFFFull || tp_nbytes > (n - r.at)) return fail(c, TGSIM_EINVAL, "restore: truncated or inconsistent image");
  // the topic arenas grow to the image's (keeping their entries: a failure below changes nothing)
  if (tp_n > c->tp_cap) {
    if (dgrow(c, &c->tp_inst, c->tp_n, tp_n) || dgrow(c, &c->tp_t, c->tp_n, tp_n) ||
        dgrow(c, &c->tp_off, c->tp_n, tp_n) || dgrow(c, &c->tp_len, c->tp_n, tp_n))
      return TGSIM_ENOMEM;
    c->tp_cap = tp_n;
  }
  if (tp_nbytes > c->tp_bytes_cap) {
    if (dgrow(c, &c->tp_bytes, c->tp_nbytes, tp_nbytes)) return TGSIM_ENOMEM;
    c->tp_bytes_cap = tp_nbytes;
  }
  const uint32_t snap_staged0 = c->snap_staged;
  const uint64_t tp_n0 = c->tp_n, tp_nbytes0 = c->tp_nbytes, tw_n0 = c->tw_n, tsg_n0 = c->tsg_n;
  c->tw_n = tw_n; c->tsg_n = tsg_n;
  const uint32_t snap_acks0 = c->snap_acks;
  c->snap_acks = snap_acks;
  c->sig_log_used = sig_used;  // sizes the log / waiter / staged / topic regions below
  c->n_waiters = n_waiters;
  c->snap_staged = snap_staged;
  c->tp_n = tp_n; c->tp_nbytes = tp_nbytes;
  auto regs = snap_regions(c);
  snap_regions_more(c, regs);
  size_t need = r.at;
  for (const auto& g : regs) need += g.second;
  if (need != n) {
    c->sig_log_used = sig_used0;
    c->n_waiters = n_waiters0;
    c->snap_staged = snap_staged0;
    c->tp_n = tp_n0; c->tp_nbytes = tp_nbytes0;
    c->tw_n = tw_n0; c->tsg_n = tsg_n0;
    c->snap_acks = snap_acks0;
    return fail(c, TGSIM_EINVAL, "restore: image size mismatch");
  }
  HIPCK(c, hipStreamSynchronize(c->d.stream), "restore");
  size_t at = r.at;
  for (const auto& g : regs) {
    if (g.second) HIPCK(c, hipMemcpyAsync(g.first, r.p + at, g.second, hipMemcpyHostToDevice, c->d.stream), "restore");
    at += g.second;
  }
  HIPCK(c, hipStreamSynchronize(c->d.stream), "restore");
  c->shape_h.swap(shape); c->flags_h.swap(flags); c->ip_h.swap(ip); c->rho_h.swap(rho); c->corr_epoch.swap(epoch);
  c->corr_reset.swap(creset); c->tb_reset.swap(treset); c->st_last_h.swap(stlast); c->moved.swap(moved);
  c->rules_h.swap(rules);
  c->now = now; c->horizon = horizon; c->n_status_last = n_status_last;
  c->pend_bound = pend_bound; c->pend_exact = pend_exact;
  c->n_staged = n_staged; c->staged_dev = staged_dev;
  c->win_m_host = win_m_host; c->win_m_extra = win_m_extra; c->win_m_inbox = win_m_inbox;
  c->win_inbox_max = win_inbox_max; c->max_tsend_h = max_tsend_h;
  c->hcnt.swap(hcnt); c->hcnt_touched.swap(hcnt_touched);
  c->fl_npubs = fl_npubs; c->fl_pub_seen.swap(fl_pub_seen);
  c->life_host = life_host; c->life_mult = life_mult;
  c->topic_runs.swap(runs);
  c->tp_index_dirty = true;
  if (c->storm_on) c->d.sm.phase = storm_phase;
  c->storm_need_react = false;
  if (c->tcp_on) {
    c->tcp_cur = tcp_cur; c->tcp_epoch = tcp_epoch; c->tcp_nb = tcp_nb; c->tcp_fill = tcp_fill;
    c->tcp_seg_batched = tcp_seg_batched; c->conn_tail.swap(conn_tail); c->tstats = tstats;
    c->storm_conn_lo = storm_conn_lo; c->storm_conn_hi = storm_conn_hi;
    c->tcp_need_react = false;
    c->tcp_snap_live[0] = c->tcp_snap_live[1] = false;
    if (int rc2 = tcp_snapshot(c)) return rc2;  // the restored counters, for tgsim_tcp_stats
  }
  c->probe_need_react = false;
  c->life_ok = false;  // the restored wheel's copies predate this context's lifetime counts
  c->now_from_device = false;
  c->shape_dirty = c->flags_dirty = c->ip_dirty = c->rules_dirty = true;  // re-uploaded at the next window
  c->d.ever_limited = true;  // the restored wheel may hold copies of a sender limited before the snapshot
  memcpy(c->d.h_sc, r.p + r.at, sizeof(DevScalars));
  return check_device_errors(c);
}
