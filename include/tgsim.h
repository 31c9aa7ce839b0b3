/*
 * tgsim.h — C ABI of the MI355X-native Testground network simulator (runner "local:mi355x").
 *
 * This is the drop-in boundary for Testground's per-message data path. Today that path is
 *   sidecar.Network.ConfigureNetwork          (reference pkg/sidecar/instance.go:37-42)
 *     -> NetlinkLink.Shape / AddRules          (pkg/sidecar/link.go:155-217)
 *     -> handleRoutingPolicy                   (pkg/sidecar/route.go:102-117)
 *     -> host-kernel HTB + netem + FIB per packet, and
 *   sync.Client SignalEntry / Barrier          (sdk-go [EXT]; call sites pkg/sidecar/sidecar_handler.go:40-79)
 * Every entry point below names the reference interface it replaces. A Go runner binds it through
 * cgo; the Python package testground_amd binds it through ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only; no torch/HIP types. Host pointers unless a name says "_device".
 *  - Return 0 on success, a negative TGSIM_E* code on error; tgsim_last_error() has the message.
 *  - One ctx per OS thread (the HIP current device is per thread). A ctx is not thread-safe.
 *  - Simulated time is int64 nanoseconds since run start, always >= 0.
 *  - Instances are global ids 0..n_instances-1. A ctx owns shard [lo, hi) of them (sharding.md in
 *    DESIGN.md): shaping state of senders in the shard, inboxes of receivers in the shard.
 *  - The semantics of every call are pinned in DESIGN.md section 2 ("Pinned semantics").
 */
#ifndef TGSIM_H
#define TGSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TGSIM_ABI_VERSION 2

/* ---- error codes ------------------------------------------------------------------------- */
enum {
  TGSIM_OK = 0,
  TGSIM_EINVAL = -1,              /* bad argument (kernel/netlink would return EINVAL) */
  TGSIM_ENOMEM = -2,              /* allocation failed */
  TGSIM_EHIP = -3,                /* HIP runtime error */
  TGSIM_ECAPACITY = -4,           /* a configured capacity was exceeded (resize and rerun) */
  TGSIM_ECAUSALITY = -5,          /* a send/signal time lies before the current window start */
  TGSIM_ENOTSUP = -6,             /* feature not supported by this build */
  TGSIM_EUNSUPPORTED_NETWORK = -7,/* docker_network.go:52-55 "unsupported network: %s" */
  TGSIM_ESTATE = -8,              /* call out of protocol order */
  TGSIM_ENODEV = -9               /* no HIP device / library built without device code */
};

/* ---- sdk-go network types ----------------------------------------------------------------- */
/* network.FilterAction (sdk-go network/types.go [EXT]): iota order Accept, Reject, Drop. */
enum { TGSIM_FILTER_ACCEPT = 0, TGSIM_FILTER_REJECT = 1, TGSIM_FILTER_DROP = 2 };
/* network.RoutingPolicyType: "allow_all" / "deny_all"; any other value (incl. "") acts as deny
 * (route.go:105-113). */
enum { TGSIM_POLICY_DENY_ALL = 0, TGSIM_POLICY_ALLOW_ALL = 1 };

/* network.LinkShape (sdk-go [EXT]) field for field; consumed at link.go:155-181. */
typedef struct tgsim_link_shape {
  int64_t latency_ns;      /* time.Duration */
  int64_t jitter_ns;       /* time.Duration */
  uint64_t bandwidth_bps;  /* bits per second, 0 = unlimited (link.go:156-159) */
  float loss;              /* percent */
  float corrupt;
  float corrupt_corr;
  float reorder;
  float reorder_corr;
  float duplicate;
  float duplicate_corr;
  int32_t filter;          /* FilterAction; only meaningful inside a rule (link.go:185-186) */
} tgsim_link_shape;

/* network.LinkRule: Subnet + LinkShape. Only Shape.filter is used (link.go:185-186 TODO). */
typedef struct tgsim_link_rule {
  uint32_t subnet_ip;      /* IPv4, host byte order (a.b.c.d = a<<24|b<<16|c<<8|d) */
  uint32_t prefix_len;     /* 0..32 */
  tgsim_link_shape shape;
} tgsim_link_rule;

/* network.Config (sdk-go [EXT]) minus the callback fields, which the sidecar handler consumes
 * (sidecar_handler.go:75-79) and which therefore live one layer up (testground_amd.sidecar). */
typedef struct tgsim_network_config {
  const char* network;         /* must be "default" */
  int32_t enable;              /* bool */
  int32_t routing_policy;      /* TGSIM_POLICY_* */
  tgsim_link_shape default_shape;
  const tgsim_link_rule* rules;
  size_t n_rules;
  int32_t has_ipv4;            /* cfg.IPv4 != nil */
  uint32_t ipv4;               /* host byte order */
} tgsim_network_config;

/* ---- simulator configuration ---------------------------------------------------------------- */
typedef struct tgsim_config {
  uint32_t n_instances;        /* total instances in the run (all shards) */
  uint32_t shard_id;           /* this ctx's shard (rank) */
  uint32_t n_shards;           /* world size; instances split into contiguous ranges */
  uint32_t device;             /* HIP device ordinal */
  uint64_t seed;               /* Philox key (run seed) */
  uint32_t data_subnet;        /* data network base address, host byte order (e.g. 16.0.0.0) */
  uint32_t data_prefix_len;    /* e.g. 16 (runner/common.go:28-40) */
  int64_t wheel_slot_ns;       /* timing-wheel slot width; 0 = default 1 ms */
  uint32_t wheel_slots;        /* slots per wheel region; 0 = default 2048 */
  uint32_t reserved0;
  uint64_t max_msgs_per_window;/* staged-message capacity per window */
  uint64_t max_records;        /* capacity of every per-window record batch and of the wheel arena */
  uint64_t exchange_cap;       /* records per peer block of one window's all-to-all (n_shards > 1): a
                                  header + up to exchange_cap - 1 due copies to that peer (at least
                                  513: 8 slices of (exchange_cap - 1) / 8, any producer may fill any
                                  slice); more is TGSIM_ECAPACITY */
  uint32_t max_states;         /* sync states (dense ids 0..max_states-1); 0 = default 4096 */
  uint32_t max_waiters;        /* barrier waiters; 0 = default 65536 */
  uint64_t max_signals;        /* signal log capacity over the run; 0 = default 2^24 */
} tgsim_config;

/* ---- message / delivery records --------------------------------------------------------------- */
/* Input messages, struct of arrays (24 B per message). (src, seq) must be unique over a run. */
typedef struct tgsim_msg_soa {
  const uint32_t* src;     /* sender instance id */
  const uint32_t* dst;     /* receiver instance id, or TGSIM_DST_EXTERNAL */
  const uint32_t* seq;     /* per-sender message id (Philox counter word) */
  const uint32_t* size;    /* bytes, < 2^31 */
  const int64_t* t_send;   /* ns */
} tgsim_msg_soa;

#define TGSIM_DST_EXTERNAL 0xFFFFFFFFu  /* a host outside the data network (plans/network/traffic.go) */
/* A time argument equal to TGSIM_T_NOW means "the current window start as the device knows it":
 * lets a run of device-ended windows (tgsim_advance_to_barrier, tgsim_advance_begin_device) go on
 * without a host round trip (accepted by tgsim_gen_storm_round's t0 and tgsim_sync_barrier's t_wait). */
#define TGSIM_T_NOW INT64_MIN

/* Per-message status (1 byte each, in enqueue order). Low nibble = code, high bits = flags. */
enum {
  TGSIM_ST_QUEUED = 0,      /* >= 1 copy entered the egress queue */
  TGSIM_ST_LOST = 1,        /* netem loss draw (and no duplicate) */
  TGSIM_ST_DROPPED = 2,     /* blackhole route: LinkRule Drop (link.go:209-210) */
  TGSIM_ST_REJECTED = 3,    /* prohibit route: LinkRule Reject (link.go:206-207), sender gets EACCES */
  TGSIM_ST_UNREACHABLE = 4, /* no route (disabled link / external under DenyAll) */
  TGSIM_ST_EXTERNAL = 5,    /* routed out via the control network (AllowAll) - leaves the simulation */
  TGSIM_ST_DEST_DOWN = 6,   /* receiver's data link disabled (Enable=false) at send time */
  TGSIM_ST_LOCAL = 7,       /* src == dst: loopback, unshaped, delivered at t_send */
  TGSIM_ST_OVERLIMIT = 8,   /* netem queue full: tail-dropped at enqueue (limit TGSIM_NETEM_LIMIT) */
  TGSIM_ST_FLAG_DUP = 0x10,         /* a duplicate clone was created */
  TGSIM_ST_FLAG_CLONE_LOST = 0x20,  /* ... and the clone's own loss draw hit */
  TGSIM_ST_FLAG_DUP_CANCEL = 0x40,  /* duplicate and loss both hit: exactly one copy sent */
  TGSIM_ST_FLAG_OVERLIMIT = 0x80    /* the original copy was tail-dropped by the queue limit (a clone
                                       that did not enter the queue, by loss or limit, is CLONE_LOST) */
};

/* Netem's queue limit in packets. link.go:169-179 builds the netem qdisc without a Limit, and
 * vishvananda/netlink v1.1.0 NewNetem then sends its default of 1000 [EXT]. A copy is tail-dropped
 * at enqueue when this many copies of the same sender, enqueued before it, are still queued (their
 * departure time is not before its enqueue time): DESIGN.md 2.3a. */
#define TGSIM_NETEM_LIMIT 1000u

/* Delivery / in-flight record flags (tgsim_record.meta, tgsim_delivery_soa.flags). */
enum {
  TGSIM_F_CLONE = 1u << 0,      /* this copy is the netem duplicate */
  TGSIM_F_CORRUPT = 1u << 1,    /* one bit flipped: byte corrupt_off, bit (flags>>4)&7 */
  TGSIM_F_REORDERED = 1u << 2,  /* took the reorder path (sent without delay) */
  TGSIM_F_STAGE_D = 1u << 3,    /* internal: t is the delivery time (else the netem ready time) */
  TGSIM_F_LOCAL = 1u << 7,      /* loopback delivery */
  TGSIM_F_WHEEL = 1u << 8       /* internal: the record is counted in its sender's queue occupancy
                                   (it entered the sender shard's timing wheel) */
};
#define TGSIM_F_BIT_SHIFT 4

/* In-flight record, 32 B. This is also the wire format of the cross-shard exchange. */
typedef struct tgsim_record {
  int64_t t;              /* stage A: netem time_to_send; stage D: delivery time */
  uint32_t src, dst, seq, size;
  uint32_t meta;          /* TGSIM_F_* | corrupt bit << 4 */
  uint32_t corrupt_off;   /* corrupted byte offset */
} tgsim_record;

/* Deliveries of one window, struct of arrays, sorted by (dst, t_deliver, src, seq, clone-first). */
typedef struct tgsim_delivery_soa {
  int64_t* t_deliver;
  uint32_t* src;
  uint32_t* dst;
  uint32_t* seq;
  uint32_t* size;
  uint32_t* flags;
  uint32_t* corrupt_off;
} tgsim_delivery_soa;

/* Cumulative counters of a ctx (this shard). */
typedef struct tgsim_stats {
  uint64_t msgs_in, copies, lost, dropped, rejected, unreachable, external, dest_down, local;
  uint64_t delivered, windows, inflight;
  uint64_t tb_items;   /* copies that went through the token bucket */
  uint64_t extracted;  /* records read back from the timing wheel */
  uint64_t inserted;   /* records written into the timing wheel */
  uint64_t overlimit;  /* copies tail-dropped by the netem queue limit */
} tgsim_stats;

typedef struct tgsim_ctx tgsim_ctx;

/* ---- lifecycle ----------------------------------------------------------------------------- */
const char* tgsim_version(void);
int tgsim_abi_version(void);
/* Replaces: NewNetlinkLink per instance (link.go:47-115) + sidecar bring-up (docker_reactor.go:132-270).
 * Every instance starts as after the sidecar's initial Config{Network:"default", Enable:true}
 * (sidecar_handler.go:26-29): link enabled, unshaped, unlimited, external routing disabled
 * (zero RoutingPolicy => deny, route.go:105-113), ip = data_subnet + 2 + id. */
int tgsim_create(const tgsim_config* cfg, tgsim_ctx** out);
void tgsim_destroy(tgsim_ctx* ctx);
const char* tgsim_last_error(const tgsim_ctx* ctx);
/* Use an external hipStream_t (e.g. torch's current stream) for all work. NULL = own stream. */
int tgsim_set_stream(tgsim_ctx* ctx, void* hip_stream);
int tgsim_shard_range(const tgsim_ctx* ctx, uint32_t* lo, uint32_t* hi);
int tgsim_sync(tgsim_ctx* ctx); /* wait for the stream, surface device-side errors */
int tgsim_get_stats(tgsim_ctx* ctx, tgsim_stats* out);
int64_t tgsim_now(const tgsim_ctx* ctx); /* current window start (host view) */
/* Reaction horizon = start of the last completed window. Messages may be staged with
 * t_send >= horizon, so an instance can answer a delivery of the last window at its delivery time
 * (conservative PDES: with window length <= lookahead the answer cannot land in a window that was
 * already delivered; a record that would is delivered late, in the current window, with its own
 * time - DESIGN.md 2.8). */
int64_t tgsim_horizon(const tgsim_ctx* ctx);

/* ---- network configuration (sidecar.Network, pkg/sidecar/instance.go:37-42) -------------------
 * tgsim_configure_network replaces DockerNetwork.ConfigureNetwork (docker_network.go:51-148) for
 * one instance, in docker apply order: policy -> enable/disable -> IP change -> Shape -> AddRules.
 * Takes effect for messages sent at or after the current window start. In a sharded run call it on
 * EVERY shard (ip/enable/policy tables are replicated; shape/rules are kept by the owning shard). */
int tgsim_configure_network(tgsim_ctx* ctx, uint32_t instance, const tgsim_network_config* cfg);
/* The same call in a named runner's apply order. TGSIM_APPLY_DOCKER is tgsim_configure_network.
 * TGSIM_APPLY_K8S follows K8sNetwork.ConfigureNetwork (k8s_network.go:43-176): Enable=false only
 * disconnects and leaves the routing policy as it was; otherwise (re)connect -> Shape -> AddRules ->
 * policy, so a failing Shape or AddRules leaves the policy unchanged. A reconnect with IPv4 nil keeps
 * the instance's current address (the CNI IPAM's choice is not modelled). */
enum { TGSIM_APPLY_DOCKER = 0, TGSIM_APPLY_K8S = 1 };
int tgsim_configure_network_order(tgsim_ctx* ctx, uint32_t instance, const tgsim_network_config* cfg, int32_t order);
/* Lower-level pieces of the same call. */
int tgsim_set_shape(tgsim_ctx* ctx, uint32_t instance, const tgsim_link_shape* shape); /* Shape, link.go:155 */
int tgsim_set_shapes(tgsim_ctx* ctx, const uint32_t* instances, const tgsim_link_shape* shapes, size_t n);
int tgsim_add_rules(tgsim_ctx* ctx, uint32_t instance, const tgsim_link_rule* rules, size_t n); /* AddRules, link.go:187 */
int tgsim_set_policy(tgsim_ctx* ctx, uint32_t instance, int32_t policy); /* handleRoutingPolicy, route.go:102 */
int tgsim_set_enabled(tgsim_ctx* ctx, uint32_t instance, int32_t enabled, int32_t has_ip, uint32_t ip);
int tgsim_get_ip(const tgsim_ctx* ctx, uint32_t instance, uint32_t* ip);

/* ---- data path (replaces the host kernel's HTB/netem/FIB per packet) ----------------------------- */
/* Stage messages for the next window (host SoA, copied). t_send must be >= tgsim_horizon(). */
int tgsim_enqueue(tgsim_ctx* ctx, const tgsim_msg_soa* msgs, size_t n);
/* Stage messages already in device memory (SoA arrays of n elements, on this device, complete on the
 * context's stream). When they are the first messages staged for the window (and no probe or storm
 * reactor is set up) they are not copied: the window reads them in place, so the arrays must stay
 * unchanged until that window's work on the context's stream has run (stream order, or the next
 * synchronising call); otherwise they are copied during the call. */
int tgsim_enqueue_device(tgsim_ctx* ctx, const tgsim_msg_soa* dev_msgs, size_t n);
/* Run one window [now, t_end): shape + route staged messages, token-bucket the copies whose netem
 * time is < t_end, deliver everything due before t_end. A sharded ctx needs a transport
 * (tgsim_comm_init / tgsim_set_transport): the window's exchange runs inside the call, which is
 * then collective - every shard calls it with the same t_end. A host-staged message sent at or
 * after t_end is refused with ECAUSALITY before anything changes (the context stays usable). */
int tgsim_advance(tgsim_ctx* ctx, int64_t t_end);
/* tgsim_advance without the closing synchronisation: everything stays queued on the ctx stream and
 * device-side errors surface at the next synchronising call (tgsim_sync, a copy, stats). */
int tgsim_advance_async(tgsim_ctx* ctx, int64_t t_end);
/* Same, with t_end = release time of a barrier waiter + offset, read on the device (no host sync).
 * Sharded: collective, as tgsim_advance (the barrier's state is replicated on every shard). */
int tgsim_advance_to_barrier(tgsim_ctx* ctx, uint32_t waiter, int64_t offset_ns);
/* ---- cross-shard transport: one exchange per window, inside tgsim_advance* -----
 * The exchange buffers are peer-major blocks of exchange_cap records; record 0 of a block is a header
 * and only records due in the window cross shards. A block of at least 8 * 64 + 1 records is eight
 * slices of (exchange_cap - 1) / 8 records, each filled by the producers of one XCD, and the header's
 * eight 32-bit words are the slices' counts; a smaller block is one slice whose count is the header's
 * .t. The layout is the library's own: a transport only moves whole blocks. Blocks travel whole
 * (their capacity is the device-known bound), so no count is read back by the host.
 * Native: RCCL over xGMI, one communicator rank per shard, owned by the ctx. unique_id comes from
 * tgsim_comm_unique_id on one rank and is distributed by the caller; tgsim_comm_init is collective
 * (every rank calls it; nranks = n_shards, rank = shard_id). */
#define TGSIM_COMM_ID_BYTES 128
int tgsim_comm_unique_id(uint8_t out[TGSIM_COMM_ID_BYTES]);
int tgsim_comm_init(tgsim_ctx* ctx, const uint8_t unique_id[TGSIM_COMM_ID_BYTES], uint32_t nranks, uint32_t rank);
/* Caller-supplied transport (MPI, gloo, a Go channel, one process driving several contexts).
 * Pointers are device pointers and stream the ctx's hipStream_t: an op is enqueued on that stream or
 * completed before it returns. Each returns 0 on success. */
typedef struct tgsim_transport {
  void* user;
  /* block p (block_bytes) of send -> block <this rank> of rank p's recv, for every p */
  int (*alltoall)(void* user, const void* send, void* recv, size_t block_bytes, void* stream);
  /* element-wise MAX over the ranks of n int64 at buf, in place */
  int (*allreduce_max_i64)(void* user, int64_t* buf, size_t n, void* stream);
  /* bytes at send of every rank -> recv[rank * bytes] */
  int (*allgather)(void* user, const void* send, void* recv, size_t bytes, void* stream);
  /* optional (NULL: none): a shard whose sharded call fails calls it, so the other ranks' pending
   * and later collectives return an error instead of waiting for this one; the context then refuses
   * sharded calls (TGSIM_ESTATE). The native communicator (tgsim_comm_init) is aborted the same way
   * (ncclCommAbort). */
  void (*abort)(void* user);
} tgsim_transport;
int tgsim_set_transport(tgsim_ctx* ctx, const tgsim_transport* transport);  /* NULL: none */
/* A shard that stops early (its run was cancelled, or the caller gave up on it) aborts its side of
 * the shard group: the transport's abort callback / ncclCommAbort, so no peer waits for it; the
 * context then refuses sharded calls. A failing sharded call does this by itself. */
int tgsim_comm_abort(tgsim_ctx* ctx);

/* Sharded window protocol without a transport: begin (sender side) -> caller all-to-alls the exchange buffers
 * (n_shards * exchange_cap records each way, peer-major; the first record of each peer block is a
 * header, above) on the same stream -> end (receiver side). */
int tgsim_advance_begin(tgsim_ctx* ctx, int64_t t_end);
int tgsim_exchange_buffers(tgsim_ctx* ctx, void** send_device, void** recv_device, size_t* bytes);
/* Use caller-owned device buffers (e.g. tensors a collective library reads/writes in place) for the
 * exchange; each must hold n_shards * exchange_cap records (tgsim_exchange_buffers' size). */
int tgsim_set_exchange_buffers(tgsim_ctx* ctx, void* send_device, void* recv_device, size_t bytes);
/* advance_begin with t_end = *t_end_device + offset read on the device (e.g. after an all-reduce). */
int tgsim_advance_begin_device(tgsim_ctx* ctx, const int64_t* t_end_device, int64_t offset_ns);
int tgsim_advance_end(tgsim_ctx* ctx);
/* Results of the last window. Copying forces a stream sync. */
int tgsim_delivery_count(tgsim_ctx* ctx, size_t* n);
int tgsim_copy_deliveries(tgsim_ctx* ctx, tgsim_delivery_soa* out, size_t cap, size_t* n);
int tgsim_copy_inbox_offsets(tgsim_ctx* ctx, uint32_t* out, size_t cap); /* shard-local dst -> offset */
int tgsim_copy_status(tgsim_ctx* ctx, uint8_t* out, size_t cap, size_t* n);
int tgsim_deliveries_device(tgsim_ctx* ctx, tgsim_delivery_soa* out_device_ptrs);

/* ---- sync service (sdk-go sync.Client [EXT]; sync-service v0.1.0) ------------------------------ */
/* SignalEntry for a batch of (state, instance, t) events. seq_out[i] = 1-based sequence number in
 * (t, instance) order among all signals of that state (NULL = not needed). Batches of one state
 * must not go back in time. Sharded with a transport: collective; each shard passes its own
 * instances' signals, the library all-gathers them (every shard keeps the whole, replicated sync
 * state, so barriers resolve on every shard). Sharded without one: every shard passes the same
 * (caller-gathered) batch. */
int tgsim_sync_signal(tgsim_ctx* ctx, const uint32_t* states, const uint32_t* instances,
                      const int64_t* t, size_t n, uint32_t* seq_out);
/* Barrier(state, target) registered at time t_wait: releases at max(t_wait, time of the
 * target-th signal). Returns a waiter id. */
int tgsim_sync_barrier(tgsim_ctx* ctx, uint32_t state, uint32_t target, int64_t t_wait,
                       uint32_t* waiter_out);
/* release_out = release time, or -1 while pending. */
int tgsim_sync_poll(tgsim_ctx* ctx, uint32_t waiter, int64_t* release_out);
int tgsim_sync_count(tgsim_ctx* ctx, uint32_t state, uint32_t* count_out);
/* sync.Client Publish / Subscribe [EXT sdk-go; call sites plans/network/pingpong.go:219-245,
 * plans/benchmarks/storm.go:232-255, plans/splitbrain/main.go:91-103]: ordered topics with full
 * history replay, kept in device memory. A topic is a sync state id (shared id space): publishing
 * counts like SignalEntry, so an entry's 1-based position follows (t, instance) order inside a
 * batch and batches of one topic must not go back in time (ECAUSALITY). Entry i of a batch is
 * (topics[i], instances[i], t[i], payload[payload_off[i] .. payload_off[i+1])); payload_off has
 * n+1 entries starting at 0. pos_out (optional) receives the positions. */
int tgsim_sync_publish(tgsim_ctx* ctx, const uint32_t* topics, const uint32_t* instances, const int64_t* t,
                       const uint64_t* payload_off, const uint8_t* payload, size_t n, uint32_t* pos_out);
/* The entries of `topic` from position `from` (1-based) on whose time is <= until_t, in position
 * order, at most `cap` of them: instances, times, payload offsets (n_out + 1 prefix offsets into
 * payload_out) and bytes. *n_out / *payload_bytes: entries and bytes returned — or, with
 * ECAPACITY when the bytes exceed payload_cap, the sizes needed. */
int tgsim_sync_subscribe(tgsim_ctx* ctx, uint32_t topic, uint32_t from, int64_t until_t, size_t cap,
                         uint32_t* instances_out, int64_t* t_out, uint64_t* payload_off_out,
                         uint8_t* payload_out, size_t payload_cap, size_t* n_out, size_t* payload_bytes);
/* Subscribe for a batch of subscribers on the device (the address-exchange fan-out: every instance
 * reads every entry of one topic, storm.go:232-255), asynchronous on the ctx stream, no host read.
 * Subscriber i reads topic topics[i] from position from[i] (1-based) on, the entries whose time is
 * <= until_t[i], at most cap_each of them (a topic >= max_states or from 0 reads none). All arrays are
 * device memory. offsets_out[0..n] (uint64): exclusive prefix of the per-subscriber counts, so
 * offsets_out[n] is the total. entries_out (NULL = counts only): subscriber i's inbox is
 * entries_out[offsets_out[i] .. offsets_out[i+1]), the arena entry ids (tgsim_topic_arena_device) in
 * position order; ids past entries_cap are not written (compare offsets_out[n] with it). */
int tgsim_sync_subscribe_device(tgsim_ctx* ctx, size_t n, const uint32_t* topics, const uint32_t* from,
                                const int64_t* until_t, uint32_t cap_each, uint64_t* offsets_out,
                                uint32_t* entries_out, size_t entries_cap);
/* The topic arena in device memory (valid until the next tgsim_sync_publish): per entry id its
 * publishing instance, time, payload offset into payload and payload length. */
int tgsim_topic_arena_device(tgsim_ctx* ctx, const uint32_t** instances, const int64_t** t,
                             const uint64_t** payload_off, const uint32_t** payload_len, const uint8_t** payload,
                             size_t* n_entries);

/* ---- profiling: HIP-event timing of kernel classes on the ctx stream ---------------------------- */
/* mask: bit k enables timing of kernel class k (0..tgsim_kernel_classes()-1); 0 disables. */
int tgsim_profile_set(tgsim_ctx* ctx, uint32_t mask);
/* Cumulative milliseconds and launch counts per kernel class (forces a sync). */
int tgsim_profile_read(tgsim_ctx* ctx, double* ms, uint64_t* launches, size_t cap, size_t* n);
int tgsim_kernel_classes(void);
const char* tgsim_kernel_name(int kernel_class);
/* Cumulative implementation counters (forces a sync), for attributing SURVEY.md 8(d) bytes to the
 * kernels that move them: [0] messages decided in the sequential queue-limit / correlation lane
 * (k_shape_seq), [1] token-bucket copies of senders with long runs (k_rest), [2] deliveries of long
 * inboxes (written by the wheel-insert launch's k_rest part), [3] deferred messages decided by the whole-sender
 * closed form (k_shape_seq_wide), [4] of [2], deliveries of long inboxes sorted whole by one workgroup in
 * LDS (experiment builds with -DTGSIM_WHOLE_SORT only; 0 in the product). *n = the count (5). */
int tgsim_kernel_counters(tgsim_ctx* ctx, uint64_t* out, size_t cap, size_t* n);
/* Test hook: the nth host allocation point from now (tgsim_add_rules, tgsim_flood_set_graph) throws
 * std::bad_alloc inside the library; the entry point returns TGSIM_ENOMEM and the context stays
 * usable (no C++ exception ever crosses this ABI). 0 disarms. */
int tgsim_debug_fail_alloc(tgsim_ctx* ctx, uint32_t nth);

/* ---- synthetic workloads (device generators) --------------------------------------- */
/* Gossip storm round (config 4): every instance of this shard sends `fanout` messages of `size`
 * bytes to Philox-chosen distinct peers at t0 + U[0, spread_ns), seq = round*fanout + k, and signals
 * `state` at its last send time. Staged for the next window; the signal batch is kept on the device
 * (count-only). Sharded with a transport: collective (the batch's first / last time is
 * MAX-reduced over the shards and every shard commits the whole batch of n_instances signals). */
int tgsim_gen_storm_round(tgsim_ctx* ctx, uint32_t round, int64_t t0, uint32_t fanout,
                          uint32_t size, int64_t spread_ns, uint32_t state);
/* Sharded runs without a transport: the storm round's signals are not committed by the generator;
 * this writes the shard's latest signal time of the last generated round (int64) to device memory,
 * where a MAX all-reduce across shards yields the release time of SignalAndWait(state, n_instances). */
int tgsim_storm_release_device(tgsim_ctx* ctx, int64_t* out_device);

/* ---- flood workload (1M-instance random-regular pubsub) --------------
 * A publication floods a fixed graph: an instance forwards it, on its first receipt, to every
 * neighbour except the sender; duplicates are dropped (first-receipt dedup). Replaces the per-peer
 * re-publish loops of pubsub/gossip test plans (message fan-out as in plans/benchmarks/storm.go:
 * 98-190; peers from the address exchange of plans/network/pingpong.go:219-245). Messages carry
 * seq = pub * D + neighbour slot (D = max degree), so (src, seq) stays unique per run.
 * set_graph: CSR over all N instances (offsets[N+1], degree <= 64, no self loops); resets the
 *   first-receipt state; max_pubs * D <= 2^32.
 * publish: instance inst[i] originates pub[i] at t[i] (>= horizon): it is marked as having seen it
 *   and sends it to all its neighbours (shard-local instances only; others are ignored).
 * react: for every delivery of the last window, in inbox order, a first receipt forwards at
 *   max(t_deliver, horizon); *n_forwarded = messages staged. Deliveries whose seq / D >= max_pubs
 *   are not flood messages: EINVAL. */
int tgsim_flood_set_graph(tgsim_ctx* ctx, const uint32_t* offsets, const uint32_t* neighbors, uint32_t max_pubs);
int tgsim_flood_publish(tgsim_ctx* ctx, const uint32_t* instances, const uint32_t* pubs, const int64_t* t,
                        size_t n, uint32_t size);
int tgsim_flood_react(tgsim_ctx* ctx, uint32_t size, size_t* n_forwarded);

/* ---- window-boundary snapshot (SURVEY.md 5 checkpoint/resume) ---------------------------------
 * The whole message-path state between windows as an opaque image: in-flight records (the timing
 * wheel), token buckets, queue occupancy, netem correlation states, every configuration table
 * (shapes, rules, routing policy, link enable, addresses), the sync service (counts, signal log,
 * barrier waiters), the clock and the last window's deliveries. Philox draws are counter-based, so
 * a run restored into a fresh context continues bit for bit as the uninterrupted run would.
 * tgsim_snapshot(ctx, NULL, 0, &n) returns the size; it synchronises the context. The image is
 * restored into a context created with the same configuration: per shard, a sharded run snapshots
 * every shard and sets the transport of the restored contexts again. The staged messages of the
 * next window are part of the image (host or device enqueues, a flood reaction's forwards, the probes'
 * requests), and so are the topic logs, a flood's first-receipt state, the probers' state and the
 * storm reactor's, and in TCP mode the writes, segments, retransmission timers, ACK clock and connections:
 * the restoring context must have the same flood graph (tgsim_flood_set_graph, same max_pubs), probe
 * setup (tgsim_probe_setup, same order and configuration), storm setup (tgsim_storm_setup, same
 * arguments) or TCP mode (tgsim_tcp_enable, same configuration; tgsim_tcp_connect, same pairs) before
 * tgsim_restore, else EINVAL. Both calls need a window boundary (ESTATE: inside a window, a probe,
 * storm or TCP reaction owed, or a tgsim_enqueue_device batch staged in place). A malformed
 * or foreign image is EINVAL and leaves the context unchanged. */
int tgsim_snapshot(tgsim_ctx* ctx, void* buf, size_t cap, size_t* n);
int tgsim_restore(tgsim_ctx* ctx, const void* buf, size_t n);

/* ---- sequential probes: request / reply, one at a time per instance ----------
 * plans/splitbrain/main.go:153-175: every node GETs each peer in turn with http.Client{Timeout: 1
 * minute}; the next GET starts when the previous one returned. Here every local instance probes
 * order[0..n_order) except itself, in that order: a request (request_bytes, seq = TGSIM_PROBE_REQ |
 * its position in order) whose first arrival at the peer is answered by one reply (reply_bytes,
 * seq = TGSIM_PROBE_REP | the prober) at max(arrival, horizon). A probe ends
 *   TGSIM_PROBE_REFUSED at its send time when the prober's route refuses the request (blackhole,
 *     prohibit, no route: connect() fails at once - a local route error is immediate [EXT]);
 *   TGSIM_PROBE_OK at the reply's first arrival, if that is before the deadline (send + timeout);
 *   TGSIM_PROBE_TIMEOUT at the deadline otherwise (lost request or reply, a peer whose reply its
 *     own routes drop, a disabled peer);
 * and the next probe leaves at max(end, horizon). Call tgsim_probe_react after every window. It
 * also proposes the next window's end: one window_ns later while anything is staged or in flight,
 * else the earliest pending deadline + 1 (idle stretches cost one window). Message mode (not with TCP
 * mode or a flood graph). Sharded (a transport attached): setup, start and react are collective; a
 * prober's state lives on its shard, the answer to it on its peer's, the reply's notice crosses in
 * the exchange blocks and the window proposal is folded over every shard. */
#define TGSIM_PROBE_REQ 0x40000000u
#define TGSIM_PROBE_REP 0xC0000000u
typedef struct tgsim_probe_config {
  uint32_t request_bytes, reply_bytes;  /* wire bytes of a request / a reply */
  int64_t timeout_ns;                   /* per probe (> 0) */
  int64_t window_ns;                    /* window length while messages are staged or in flight (> 0) */
} tgsim_probe_config;
enum { TGSIM_PROBE_NONE = 0, TGSIM_PROBE_OK = 1, TGSIM_PROBE_REFUSED = 2, TGSIM_PROBE_TIMEOUT = 3 };

int tgsim_probe_setup(tgsim_ctx* ctx, const uint32_t* order, uint32_t n_order, const tgsim_probe_config* cfg);
/* Every local instance sends its first probe at t0 (>= horizon). */
int tgsim_probe_start(tgsim_ctx* ctx, int64_t t0);
/* After a window: resolve probes, stage replies and next requests (device-side staging). next_end /
 * n_active non-NULL: synchronise and return the proposed window end and the instances still probing;
 * both NULL: asynchronous (see tgsim_probe_next_end_device). */
int tgsim_probe_react(tgsim_ctx* ctx, int64_t* next_end, uint32_t* n_active);
/* Device address of the proposed window end (for tgsim_advance_begin_device: no host round trip)
 * and of the count of instances still probing. */
int tgsim_probe_state_device(tgsim_ctx* ctx, const int64_t** next_end_device, const uint32_t** n_active_device);
/* outcome[l * n_order + j] = TGSIM_PROBE_* of local instance l's probe of order[j] (NONE for itself
 * and probes not yet ended); t_done[l] = when its last probe ended (INT64_MIN while probing). */
int tgsim_probe_results(tgsim_ctx* ctx, uint8_t* outcome, int64_t* t_done, size_t cap_outcome);

/* ---- storm plan reactor: dials and paced writes on the device -----------------
 * plans/benchmarks/storm.go:117-190, per instance: `outgoing` goroutines, each sleeping until its
 * t_ready (conn_delay_ms), then dialling its peer under the dial semaphore `sem` (concurrent slots,
 * FIFO in (t_ready, connection) order; net.DialTimeout, storm.go:141-152), and - once every dial is
 * done and "outgoing-dials-done" released - writing data_bytes in chunk_bytes writes, each under the
 * write semaphore `writesem` (storm.go:158-183), where conn.Write returns once the chunk fits the
 * connection's send buffer and blocks its goroutine, holding its slot, while the buffer is full.
 * Connection h = instance * outgoing + k (k < outgoing) goes to dst[h]. Message mode:
 *  - a dial is a SYN (syn_bytes, seq = TGSIM_STORM_SYN | k) that the peer answers at its first
 *    arrival with a SYN-ACK (seq = TGSIM_STORM_SYNACK | h) at max(arrival, horizon); the dial ends
 *    TGSIM_PROBE_OK at the SYN-ACK's first arrival before the deadline (start + dial_timeout_ns),
 *    TGSIM_PROBE_REFUSED at its start when the dialler's route refuses the SYN, TGSIM_PROBE_TIMEOUT
 *    at the deadline otherwise; its semaphore slot is free from its end on;
 *  - a write is one message of payload + header_bytes (seq = TGSIM_STORM_DATA | k * n_chunks + j,
 *    n_chunks = ceil(data_bytes / chunk_bytes)); a connection's buffer holds msg_window chunks that
 *    have neither arrived (first copy) nor failed (a status other than QUEUED).
 * After every window, tgsim_storm_react resolves dials, answers SYNs, starts the dials the semaphore
 * admits (those due before the next window's end), and in the write phase runs each instance's
 * writesem round at the window's end over the room the window's arrivals and failures freed, all
 * staged on the device behind the device-side staged count. It proposes the next window's end
 * (window_ns later while anything is staged or in flight, else the next deadline + 1 or the next
 * dial's start). Message mode (not with probes or a flood graph); sharded contexts (a transport
 * attached) run the reactor collectively, each shard its own instances' dials and writes
 * (DESIGN.md 2.14); TCP mode (acks = 1, below) needs a single-shard context.
 * Like probes, it owns each window's statuses and deliveries: staging or the next window before the
 * reaction is ESTATE. */
#define TGSIM_STORM_SYN 0x40000000u
#define TGSIM_STORM_DATA 0x80000000u
#define TGSIM_STORM_SYNACK 0xC0000000u
typedef struct tgsim_storm_config {
  uint32_t outgoing;          /* connections per instance (conn_outgoing), >= 1 */
  uint32_t concurrent;        /* width of the dial and write semaphores (concurrent_dials), >= 1 */
  uint32_t chunk_bytes;       /* bytes per conn.Write (storm.go:23 buffersize: 4096), >= 1 */
  uint32_t header_bytes;      /* wire overhead added to every chunk */
  uint64_t data_bytes;        /* bytes each connection writes (data_size_kb * 1024) */
  uint32_t syn_bytes;         /* wire bytes of a SYN and of a SYN-ACK */
  uint32_t msg_window;        /* chunks a connection's send buffer holds (>= 1) */
  int64_t dial_timeout_ns;    /* net.DialTimeout (storm.go:144: 30 s), > 0 */
  int64_t window_ns;          /* window length while traffic is staged or in flight, > 0 */
} tgsim_storm_config;
typedef struct tgsim_storm_totals {
  uint64_t chunks_written, chunks_delivered, chunks_failed, bytes_written;
  uint32_t dials_ok, dials_failed, dials_pending, conns_writing;  /* conns_writing: chunks left or in flight */
} tgsim_storm_totals;
/* dst[h], t_ready[h] (>= tgsim_now) for every connection h < n_instances * outgoing; resets the reactor. */
int tgsim_storm_setup(tgsim_ctx* ctx, const uint32_t* dst, const int64_t* t_ready, const tgsim_storm_config* cfg);
/* Stage the dials the semaphores admit before tgsim_now + window_ns (the first reaction). */
int tgsim_storm_start(tgsim_ctx* ctx);
/* After every window (see above). next_end / n_active non-NULL: synchronise and return the proposed
 * window end and the connections still dialling (dial phase) or writing / in flight (write phase);
 * both NULL: asynchronous (tgsim_storm_state_device). */
int tgsim_storm_react(tgsim_ctx* ctx, int64_t* next_end, uint32_t* n_active);
int tgsim_storm_state_device(tgsim_ctx* ctx, const int64_t** next_end_device, const uint32_t** n_active_device);
/* Per connection: dial outcome TGSIM_PROBE_* (NONE while pending) and its end time. */
int tgsim_storm_dials(tgsim_ctx* ctx, uint8_t* outcome, int64_t* t_done, size_t cap);
/* The write phase: every connection's goroutine takes writesem at t0 (>= horizon; the release of
 * "outgoing-dials-done", storm.go:156), in connection order. */
int tgsim_storm_write_start(tgsim_ctx* ctx, int64_t t0);
/* Per instance: failed = a chunk of it failed (lost, tail-dropped, refused) or is still in flight;
 * t_last = when its last conn.Write returned (INT64_MIN: none); totals. Any output may be NULL. */
int tgsim_storm_results(tgsim_ctx* ctx, uint8_t* failed, int64_t* t_last, size_t cap, tgsim_storm_totals* totals);
/* Detach the reactor: windows no longer need tgsim_storm_react. */
int tgsim_storm_end(tgsim_ctx* ctx);

/* ---- TCP-level mode ----------------------------------
 * The reference plans move application data over TCP (plans/benchmarks/storm.go:127-180 dials and
 * writes in chunks, plans/network/pingpong.go:73-104 times round trips over a connection); with loss
 * the message-level model undercounts what the receiver sees. In TCP mode an application write
 * (tgsim_tcp_send) becomes ceil(size / mss) segments, each a packet of payload + header_bytes on
 * the wire through the unchanged netem / HTB / FIB path. A segment's attempt fails when none of its
 * copies enters the egress queue, or every copy that does arrives corrupted (the TCP checksum drops
 * it); attempt a + 1 is then sent at max(t_a + rto * 2^a, the time the failure is known), up to
 * max_attempts attempts (then the write fails). A route that refuses the packet (prohibit / no
 * route) fails the write at once. A segment arrives with its first intact copy; a write completes
 * when its last segment arrives. While TCP mode is on, all traffic is TCP (tgsim_enqueue is
 * refused). Packet seq = segment id * 16 + attempt (segment ids count from 0 in send order, < 2^28).
 * Sharded contexts (a transport attached) carry generated storm rounds (tgsim_tcp_gen_storm_round, one
 * fanout) and react collectively: a data copy delivered on another shard is forwarded to its writer's
 * shard after the window and settled there, its ACK leaves from the receiver's shard, and the
 * segment ids on the wire are the single-shard run's, so a sharded run equals it;
 * tgsim_tcp_send and connections need a single-shard context (TGSIM_ENOTSUP).
 *
 * acks = 1 adds the reverse path: every intact data copy the receiver gets is answered by an ACK
 * packet (header_bytes, seq = TGSIM_TCP_ACK_BIT | the data packet's seq) sent at max(arrival, the
 * next window's start) through the receiver's egress. Attempt a of a segment arms a timer at
 * t_a + rto * 2^a; at the start of each window, every timer of an attempt sent in an earlier window
 * that falls before the window's end fires unless an intact ACK of the segment arrived in an
 * earlier window: attempt a + 1 leaves at max(timer, window start) (spurious retransmissions
 * included), and after max_attempts attempts the segment gives up (the write fails, TIMEOUT at the
 * timer, if it has not completed). A write's outcome is its first event in window order: a write
 * that failed stays failed. Segment ids < 2^27. The congestion window and fast retransmit are the
 * connections' (below); not modelled: delayed ACKs, SACK. */
#define TGSIM_TCP_ACK_BIT 0x80000000u
typedef struct tgsim_tcp_config {
  uint32_t mss;           /* payload bytes per segment; 0 = 1448 */
  uint32_t header_bytes;  /* wire overhead per segment (IPv4 + TCP with timestamps); 0 = 52 */
  int64_t rto_ns;         /* first retransmission timeout; 0 = 200 ms (Linux TCP_RTO_MIN) */
  uint32_t max_attempts;  /* attempts per segment, 1..16; 0 = 16 */
  uint32_t acks;          /* 1: ACK packets on the reverse path and retransmission timers (above) */
  uint64_t max_writes;    /* write-table capacity over the run; 0 = 2^22, at most 2^28 */
  uint64_t max_segments;  /* segment-table capacity over the run; 0 = 2^24 */
} tgsim_tcp_config;

enum { TGSIM_TCP_PENDING = 0, TGSIM_TCP_DELIVERED = 1, TGSIM_TCP_TIMEOUT = 2, TGSIM_TCP_REFUSED = 3 };

typedef struct tgsim_tcp_stats {
  uint64_t writes, segments, packets, retransmissions, delivered, failed, pending_retx;
} tgsim_tcp_stats;

int tgsim_tcp_enable(tgsim_ctx* ctx, const tgsim_tcp_config* cfg);
/* Application writes (src, dst, seq = the write's order key on its connection, size, t_send), staged
 * like tgsim_enqueue (t_send >= tgsim_horizon). Write ids count from 0 in send order. */
int tgsim_tcp_send(tgsim_ctx* ctx, const tgsim_msg_soa* writes, size_t n);
/* After every window, before staging for the next: account the window's packets (queued copies) and
 * deliveries (arrivals, corrupt copies), schedule retransmissions (staged by the window that covers
 * their time), complete writes. *n_completed = writes delivered or failed in this call. NULL: the
 * reaction is only queued on the context stream (no synchronisation; its counters reach
 * tgsim_tcp_get_stats / tgsim_tcp_writes, which synchronise, and device errors the next synchronising
 * call). */
int tgsim_tcp_react(tgsim_ctx* ctx, size_t* n_completed);
/* Per write id: state TGSIM_TCP_* and time (arrival of its last segment, or the failure time). */
int tgsim_tcp_writes(tgsim_ctx* ctx, uint8_t* state_out, int64_t* t_out, size_t cap, size_t* n);
int tgsim_tcp_get_stats(tgsim_ctx* ctx, tgsim_tcp_stats* out);
/* tgsim_gen_storm_round as TCP writes (TCP mode; size <= mss: one segment per write), generated on
 * the device: the round's messages become writes with ids in generation order (instance-major). */
int tgsim_tcp_gen_storm_round(tgsim_ctx* ctx, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                              int64_t spread_ns, uint32_t state);
/* Writes ids [first, first + n): state and time as tgsim_tcp_writes (a range, so a caller polling
 * the unsettled tail of a long run reads O(range), not O(writes so far)). */
int tgsim_tcp_writes_range(tgsim_ctx* ctx, uint64_t first, size_t n, uint8_t* state_out, int64_t* t_out);

/* ---- TCP connections: congestion window and ACK clocking (acks = 1 only) -------
 * plans/benchmarks/storm.go:141-183 dials a connection and writes 4 KiB chunks into it; the socket
 * sends while its congestion window allows. A connection (src -> dst) queues the segments of its
 * writes in write order and keeps a window [EXT Linux tcp_cong.c Reno, RFC 5681]: cwnd starts at
 * 10 segments (IW10), ssthresh unbounded; segments leave while the flight (sent, neither ACKed nor
 * given up) is below cwnd - a write's segments at its t_send if the window has room then, the rest
 * at the end of the window in which ACKs opened room (ACKs are processed window by window, as they
 * are sent: tgsim_tcp_config.acks). Each first ACK of a segment: flight - 1 and, below ssthresh,
 * cwnd + 1 (slow start), else one more segment per cwnd ACKs (congestion avoidance); cwnd <= 65535.
 * The first retransmission timeout of a connection in a window sets cwnd = 1 and, unless cwnd was
 * already 1 (the same loss episode), ssthresh = max(cwnd / 2, 2); the retransmitted segments
 * themselves are not held back. A refused segment (local
 * route error) breaks the connection: its queued writes fail (REFUSED). A context uses either
 * connections or tgsim_tcp_send / tgsim_tcp_gen_storm_round, not both. Connection ids count from 0. */
int tgsim_tcp_connect(tgsim_ctx* ctx, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* conn_out);
/* Writes (conn[i], size[i], t_send[i] >= horizon) appended to their connections' send queues in
 * call order; write ids continue tgsim_tcp_writes' numbering. */
int tgsim_tcp_write(tgsim_ctx* ctx, const uint32_t* conn, const uint32_t* size, const int64_t* t_send, size_t n);
/* Per connection [first, first + n): segments ACKed so far (cumulative), cwnd, flight, queued
 * (written, not yet sent) - any output may be NULL. Synchronises. */
int tgsim_tcp_conns(tgsim_ctx* ctx, uint32_t first, size_t n, uint64_t* acked, uint32_t* cwnd, uint32_t* flight,
                    uint32_t* queued);

#ifdef __cplusplus
}
#endif
#endif /* TGSIM_H */
