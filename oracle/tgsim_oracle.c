/*
 * tgsim_oracle.c — TEST INFRASTRUCTURE ONLY (see tgsim_oracle.h for the rules and parity status).
 *
 * Single-threaded, deliberately literal restatement of the pinned semantics in DESIGN.md section 2.
 * Data structures are the obvious ones (sorted vectors, a binary heap, qsort), so that the GPU
 * implementation, which uses radix bucketing, LDS bitonic sorts, max-plus scans and a slotted
 * timing wheel, is checked against something independent of its own structure.
 */
#include "tgsim_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NEG_INF (INT64_MIN / 4)
#define TB_CLAMP ((int64_t)1 << 61)
#define COST_CLAMP ((uint64_t)1 << 52)
#define EXTERNAL_IP 0x08080808u /* TGSIM_DST_EXTERNAL is modelled as 8.8.8.8 */

/* ============================== primitives ================================================= */

/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox.h). Constants are the published ones. */
void tgo_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Go's uint32(x) of a float on amd64: CVTTS?2SQ to int64 (0x8000000000000000 when out of range or
 * NaN), then the low 32 bits. */
static uint32_t go_u32_of_double(double v) {
  if (!(v > -9.2233720368547758e18 && v < 9.2233720368547758e18)) return 0u;
  return (uint32_t)(uint64_t)(int64_t)v;
}

/* vishvananda/netlink v1.1.0 Percentage2u32 [EXT] (called for Loss/Duplicate/Reorder/Corrupt from
 * NewNetem, which link.go:169-179 feeds): 100 -> MaxUint32, else uint32(MaxUint32 * (pct/100)) with
 * the untyped constant converted to float32 and the product computed in float32. */
uint32_t tgo_percentage2u32(float pct) {
  if (pct == 100.0f) return 0xFFFFFFFFu;
  volatile float q = pct / 100.0f;
  volatile float v = 4294967296.0f * q;
  return go_u32_of_double((double)v);
}

/* netlink time2Tick: uint32(float64(us) * tickInUsec), tickInUsec = 1000/64 = 15.625 from
 * /proc/net/psched "000003e8 00000040 000f4240 3b9aca00" [EXT]. us*15.625 is exact in float64. */
uint32_t tgo_time2tick(uint32_t us) { return (uint32_t)(((uint64_t)us * 125u) >> 3); }

/* pkg/sidecar/link.go:143-151 toMicroseconds: Duration.Microseconds() (truncating division), capped
 * at MaxUint32, then uint32() (negative values wrap). */
uint32_t tgo_to_microseconds(int64_t ns) {
  int64_t us = ns / 1000;
  if (us > (int64_t)0xFFFFFFFFu) us = 0xFFFFFFFFu;
  return (uint32_t)(uint64_t)us;
}

/* Linux psched_ratecfg_precompute__ [EXT] (net/sched/sch_generic.c): the HTB class rate as a
 * multiply-shift of the byte count: l2t_ns(len) = (len * mult) >> shift. */
void tgo_ratecfg(uint64_t rate, uint32_t* mult, uint32_t* shift) {
  uint64_t factor = 1000000000ull;
  *mult = 1; *shift = 0;
  if (rate == 0) return;
  for (;;) {
    *mult = (uint32_t)(factor / rate);
    if ((*mult & (1u << 31)) || (factor & (1ull << 63))) break;
    factor <<= 1;
    (*shift)++;
  }
}

typedef struct {
  int64_t mu;        /* netem latency, ns */
  int32_t sigma;     /* netem jitter, ns, as the s32 argument of tabledist */
  uint32_t loss_t, dup_t, corrupt_t, reorder_t;
  uint32_t mult, shift; /* HTB rate */
  int64_t tau;       /* HTB buffer, ns */
  int limited;       /* Bandwidth != 0 */
  uint32_t dup_rho, corrupt_rho, reorder_rho; /* netem correlations (Percentage2u32) */
  int corr;          /* some correlated draw is used: the sender's messages run in (t, seq) order */
} oshape;

/* LinkShape -> the netem/HTB state the kernel ends up with.
 * link.go:155-181 (Shape), netlink NewHtbClass/NewNetem [EXT], sch_htb/sch_netem change paths [EXT]. */
static int derive_shape(const tgsim_link_shape* s, oshape* o, char* err, size_t errlen) {
  memset(o, 0, sizeof(*o));
  /* HTB: link.go:156-167; rate = Bandwidth/8 bytes/s (netlink NewHtbClass); the kernel refuses a
   * zero rate (htb_change_class: !hopt->rate.rate && !rate64 -> EINVAL). */
  uint64_t bw = s->bandwidth_bps == 0 ? UINT64_MAX : s->bandwidth_bps;
  uint64_t rate = bw / 8;
  if (rate == 0) {
    if (err) snprintf(err, errlen, "invalid htb rate: %llu bits/s", (unsigned long long)s->bandwidth_bps);
    return TGSIM_EINVAL;
  }
  o->limited = s->bandwidth_bps != 0;
  tgo_ratecfg(rate, &o->mult, &o->shift);
  /* buffer = uint32(rate/Hz + mtu) bytes, Hz = 1e9 (hrtimer psched), mtu = 1600; then
   * Xmittime = time2Tick(uint32(1e6 * (buffer/rate))) ticks; kernel: ns = ticks << 6. */
  uint32_t buf_bytes = go_u32_of_double((double)rate / 1e9 + 1600.0);
  uint32_t buf_us = go_u32_of_double(1000000.0 * ((double)buf_bytes / (double)rate));
  o->tau = (int64_t)tgo_time2tick(buf_us) << 6;
  /* netem: link.go:169-179 -> netlink NewNetem: latency = time2Tick(us); jitter converted only when
   * the converted latency is > 0; kernel stores ticks << 6 ns; tabledist takes sigma as s32. */
  uint32_t lat_ticks = tgo_time2tick(tgo_to_microseconds(s->latency_ns));
  uint32_t jit_us = tgo_to_microseconds(s->jitter_ns);
  uint32_t jit_ticks = lat_ticks > 0 ? tgo_time2tick(jit_us) : jit_us;
  o->mu = (int64_t)lat_ticks << 6;
  o->sigma = (int32_t)(uint32_t)((uint64_t)jit_ticks << 6);
  o->loss_t = tgo_percentage2u32(s->loss);
  o->dup_t = tgo_percentage2u32(s->duplicate);
  o->corrupt_t = tgo_percentage2u32(s->corrupt);
  o->reorder_t = tgo_percentage2u32(s->reorder);
  /* correlations: netlink Percentage2u32 of CorruptCorr / ReorderCorr / DuplicateCorr (link.go:
   * 173-178); netem draws through get_crandom only when the probability is non-zero [EXT] */
  o->dup_rho = s->duplicate_corr != 0.0f ? tgo_percentage2u32(s->duplicate_corr) : 0;
  o->corrupt_rho = s->corrupt_corr != 0.0f ? tgo_percentage2u32(s->corrupt_corr) : 0;
  o->reorder_rho = s->reorder_corr != 0.0f ? tgo_percentage2u32(s->reorder_corr) : 0;
  o->corr = (o->dup_rho && o->dup_t) || (o->corrupt_rho && o->corrupt_t) || (o->reorder_rho && o->reorder_t);
  return TGSIM_OK;
}

int tgo_derive_shape(const tgsim_link_shape* s, int64_t out[10]) {
  oshape o;
  int rc = derive_shape(s, &o, NULL, 0);
  if (rc) return rc;
  out[0] = o.mu; out[1] = o.sigma; out[2] = o.loss_t; out[3] = o.dup_t; out[4] = o.corrupt_t;
  out[5] = o.reorder_t; out[6] = o.mult; out[7] = o.shift; out[8] = o.tau; out[9] = o.limited;
  return 0;
}

/* pkg/runner/common.go:28-40 nextDataNetwork: 16+n/256 . n%256 .0.0/16, gateway .1, >4095 exhausted. */
int tgo_next_data_network(int n, uint32_t* subnet, uint32_t* prefix_len, uint32_t* gw) {
  if (n > 4095 || n < 0) return TGSIM_EINVAL;
  uint32_t a = 16u + (uint32_t)n / 256u, b = (uint32_t)n % 256u;
  *subnet = (a << 24) | (b << 16);
  *prefix_len = 16;
  *gw = *subnet | 1u;
  return TGSIM_OK;
}

/* Linux netem tabledist() uniform branch [EXT]: sigma==0 -> mu; else ((rnd % (2*(u32)sigma)) + mu) - sigma. */
static int64_t tabledist(int64_t mu, int32_t sigma, uint32_t rnd) {
  if (sigma == 0) return mu;
  uint32_t m = 2u * (uint32_t)sigma;
  if (m == 0) return mu;
  return (int64_t)(rnd % m) + mu - (int64_t)sigma;
}

static uint64_t l2t_ns(const oshape* s, uint32_t len) {
  uint64_t c = ((uint64_t)len * s->mult) >> s->shift;
  return c > COST_CLAMP ? COST_CLAMP : c;
}

/* ============================== context ===================================================== */

typedef struct { uint32_t prefix, plen; int32_t action; } orule;
typedef struct { orule* v; size_t n, cap; } orules;
typedef struct { uint32_t* src; uint32_t* dst; uint32_t* seq; uint32_t* size; int64_t* t; size_t n, cap; } omsgs;
typedef struct { tgsim_record* v; size_t n, cap; } orecs;
typedef struct { int64_t* t; size_t n, cap; } otimes;
typedef struct { uint32_t state, target; int64_t t_wait; } owaiter;

typedef struct otopic { uint32_t* inst; int64_t* t; uint64_t* off; uint32_t* len; size_t n, cap; } otopic;

struct tgo_ctx {
  tgsim_config cfg;
  uint32_t N, lo, hi, nloc, S;
  uint32_t data_net, data_mask, data_len;
  uint64_t seed;
  oshape* shape;      /* [nloc] */
  int64_t* X;         /* [nloc] HTB token state as the time tokens reach 0 */
  orules* rules;      /* [nloc] sorted by (plen desc, prefix asc) */
  uint8_t* enabled;   /* [N] */
  uint8_t* allow_ext; /* [N] */
  uint32_t* ip;       /* [N] */
  uint32_t* id_of;    /* [2^(32-len)] ip - data_net -> id, or UINT32_MAX */
  size_t id_of_n;
  int64_t now, t_end;
  int64_t horizon;    /* start of the last completed window: earliest admissible t_send */
  int in_window;
  omsgs staged;
  uint8_t* status; size_t n_status, status_cap;
  orecs heap;         /* pending records, min-heap on t */
  orecs A, D;         /* per-window scratch */
  uint32_t* pend;     /* [nloc] copies of local sender l in the pending heap (its queue beyond the window) */
  orecs out;          /* deliveries of the last window (sorted) */
  uint32_t* inbox;    /* [nloc+1] */
  tgsim_record* xsend; tgsim_record* xrecv; size_t xcap;
  orecs* outbox;      /* [S] */
  orecs tcp_rx;       /* sharded TCP: data copies other shards delivered for this shard's writers */
  tgsim_stats stats;
  otimes* sig;        /* per state: signal times in seq order */
  size_t n_states;
  owaiter* waiters; size_t n_waiters, waiters_cap;
  int64_t storm_release;
  uint32_t* cl;       /* [nloc][3] netem crandom state (dup, corrupt, reorder): last answer */
  uint32_t* epoch;    /* [nloc] Shape calls so far (seeds the state a Shape call re-initialises) */
  /* topics: per state id, entries in position order; payload bytes in one buffer */
  struct otopic* topics; size_t n_topics;
  uint8_t* tp_bytes; size_t tp_nbytes, tp_cap;
  /* flood (config 5): local rows of the graph, first-receipt bits [max_pubs][nloc] */
  uint32_t* fl_off; uint32_t* fl_nbr; uint32_t* fl_seen;
  uint32_t fl_D, fl_max_pubs, fl_wpp;
  /* cross-shard transport (tgsim_set_transport): host buffers, stream NULL */
  tgsim_transport tr;
  int has_tr, replicated_batch, tr_aborted;
  /* TCP mode: writes, segments, segments with a retransmission scheduled */
  int tcp_on, tcp_need_react;
  uint32_t tcp_F;     /* sharded TCP: the generated storm rounds' fanout (tcp_wire / tcp_local) */
  tgsim_tcp_config tcp;
  struct otcpw* tw; size_t tw_n, tw_cap;
  struct otcps* tsg; size_t tsg_n, tsg_cap;
  uint32_t* tpend; size_t tpend_n, tpend_cap;
  struct otack* tack; size_t tack_n, tack_cap;  /* acks = 1: ACK packets for the next window */
  struct otcpc* tc; size_t tc_n, tc_cap;        /* connections (tgsim_tcp_connect) */
  uint64_t sm_conn_lo, sm_conn_hi;               /* a TCP storm's connections: host writes refused */
  tgsim_tcp_stats tstats;
  /* sequential probes (tgsim_probe_*) */
  struct oprobe* pr; uint32_t* pr_order; uint8_t* pr_out; uint32_t pr_n; tgsim_probe_config pr_cfg;
  /* the answering side of the probes (per prober g, on every shard: the requests its peers on this
   * shard received): last position answered + 1, the position being answered in this reaction + 1,
   * its requests' first arrival; the probers answered in this reaction */
  uint32_t *pr_ans, *pr_cur, *pr_list; int64_t* pr_rqa; size_t pr_list_n;
  int pr_need_react;  /* a window ended with probes set up: tgo_probe_react before staging or the next window */
  /* storm plan reactor (tgsim_storm_*) */
  struct ostorm* sm;
  int sm_need_react;
  char err[512];
};

typedef struct otcpw { uint32_t src, dst, remaining, state; int64_t t; uint32_t conn; } otcpw;
typedef struct otcps {
  uint32_t w, wire, attempt, outstanding, arrived, touched;
  int64_t t_att, arrival, t_last;
  uint32_t acked, gave_up;  /* acks = 1 */
  uint32_t next, unsent;    /* connections: the connection's next segment; queued, not yet sent */
  uint32_t lost;            /* connections: marked lost at a timeout, waiting to be resent under cwnd */
} otcps;
/* a TCP connection: congestion window and the queue of its unsent segments */
typedef struct otcpc {
  uint32_t src, dst, cwnd, ssthresh, cnt, flight, queued, head, tail, acks, broken;
  uint64_t acked;
  int64_t tloss;            /* the window's earliest expired timer (INT64_MAX: none): a loss episode */
  uint32_t una;             /* no segment before it is outstanding (advanced lazily at a timeout) */
  uint32_t facks;           /* the window's first ACKs of segments in flight (not marked lost) */
  int64_t tack;             /* the window's latest first-ACK arrival (INT64_MIN: none) */
  uint32_t fr;              /* the segment last fast-retransmitted (TCP_NOSEG: none) */
} otcpc;
#define TCP_NOSEG 0xFFFFFFFFu
#define TCP_IW 10u
#define TCP_CWND_CLAMP 65535u
typedef struct otack { uint32_t src, dst, seq; int64_t t; } otack;

static int fail(tgo_ctx* c, int code, const char* fmt, ...) {
  if (c) { va_list ap; va_start(ap, fmt); vsnprintf(c->err, sizeof(c->err), fmt, ap); va_end(ap); }
  return code;
}

static int grow(void** p, size_t* cap, size_t need, size_t elem) {
  if (need <= *cap) return 0;
  size_t nc = *cap ? *cap : 64;
  while (nc < need) nc *= 2;
  void* q = realloc(*p, nc * elem);
  if (!q) return TGSIM_ENOMEM;
  *p = q; *cap = nc;
  return 0;
}
static int recs_push(orecs* r, const tgsim_record* x) {
  if (grow((void**)&r->v, &r->cap, r->n + 1, sizeof(tgsim_record))) return TGSIM_ENOMEM;
  r->v[r->n++] = *x;
  return 0;
}

/* min-heap on t */
static int heap_push(orecs* h, const tgsim_record* x) {
  if (recs_push(h, x)) return TGSIM_ENOMEM;
  size_t i = h->n - 1;
  while (i) {
    size_t p = (i - 1) / 2;
    if (h->v[p].t <= h->v[i].t) break;
    tgsim_record t = h->v[p]; h->v[p] = h->v[i]; h->v[i] = t; i = p;
  }
  return 0;
}
static tgsim_record heap_pop(orecs* h) {
  tgsim_record top = h->v[0];
  h->v[0] = h->v[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < h->n && h->v[l].t < h->v[m].t) m = l;
    if (r < h->n && h->v[r].t < h->v[m].t) m = r;
    if (m == i) break;
    tgsim_record t = h->v[m]; h->v[m] = h->v[i]; h->v[i] = t; i = m;
  }
  return top;
}

static uint32_t shard_of(const tgo_ctx* c, uint32_t g) {
  /* shard k owns [floor(k*N/S), floor((k+1)*N/S)) */
  uint32_t k = (uint32_t)(((uint64_t)g * c->S) / c->N);
  while (k + 1 < c->S && (uint32_t)(((uint64_t)(k + 1) * c->N) / c->S) <= g) ++k;
  while (k > 0 && (uint32_t)(((uint64_t)k * c->N) / c->S) > g) --k;
  return k;
}

static const tgsim_link_shape ZERO_SHAPE;

int tgo_create(const tgsim_config* cfg, tgo_ctx** out) {
  *out = NULL;
  if (!cfg || cfg->n_instances == 0 || cfg->n_shards == 0 || cfg->shard_id >= cfg->n_shards)
    return TGSIM_EINVAL;
  if (cfg->data_prefix_len < 1 || cfg->data_prefix_len > 30) return TGSIM_EINVAL;
  tgo_ctx* c = (tgo_ctx*)calloc(1, sizeof(tgo_ctx));
  if (!c) return TGSIM_ENOMEM;
  c->cfg = *cfg;
  c->N = cfg->n_instances; c->S = cfg->n_shards;
  c->lo = (uint32_t)(((uint64_t)cfg->shard_id * c->N) / c->S);
  c->hi = (uint32_t)(((uint64_t)(cfg->shard_id + 1) * c->N) / c->S);
  c->nloc = c->hi - c->lo;
  c->seed = cfg->seed;
  c->data_len = cfg->data_prefix_len;
  c->data_mask = 0xFFFFFFFFu << (32 - c->data_len);
  c->data_net = cfg->data_subnet & c->data_mask;
  c->id_of_n = (size_t)1 << (32 - c->data_len);
  if ((uint64_t)c->N + 2 > c->id_of_n) { free(c); return TGSIM_EINVAL; }
  c->shape = (oshape*)calloc(c->nloc ? c->nloc : 1, sizeof(oshape));
  c->X = (int64_t*)calloc(c->nloc ? c->nloc : 1, sizeof(int64_t));
  c->pend = (uint32_t*)calloc(c->nloc ? c->nloc : 1, sizeof(uint32_t));
  c->rules = (orules*)calloc(c->nloc ? c->nloc : 1, sizeof(orules));
  c->enabled = (uint8_t*)calloc(c->N, 1);
  c->allow_ext = (uint8_t*)calloc(c->N, 1);
  c->ip = (uint32_t*)calloc(c->N, sizeof(uint32_t));
  c->id_of = (uint32_t*)malloc(c->id_of_n * sizeof(uint32_t));
  c->inbox = (uint32_t*)calloc(c->nloc + 1, sizeof(uint32_t));
  c->outbox = (orecs*)calloc(c->S, sizeof(orecs));
  c->xcap = cfg->exchange_cap ? cfg->exchange_cap : 1024;
  c->xsend = (tgsim_record*)calloc((size_t)c->S * c->xcap, sizeof(tgsim_record));
  c->xrecv = (tgsim_record*)calloc((size_t)c->S * c->xcap, sizeof(tgsim_record));
  if (!c->shape || !c->X || !c->pend || !c->rules || !c->enabled || !c->allow_ext || !c->ip || !c->id_of ||
      !c->inbox || !c->outbox || !c->xsend || !c->xrecv) {
    tgo_destroy(c);
    return TGSIM_ENOMEM;
  }
  memset(c->id_of, 0xFF, c->id_of_n * sizeof(uint32_t));
  oshape z;
  derive_shape(&ZERO_SHAPE, &z, NULL, 0);
  for (uint32_t i = 0; i < c->nloc; ++i) { c->shape[i] = z; c->X[i] = NEG_INF; }
  for (uint32_t g = 0; g < c->N; ++g) {
    c->enabled[g] = 1;
    c->allow_ext[g] = 0; /* sidecar init config has the zero RoutingPolicy => disable (route.go:105-113) */
    c->ip[g] = c->data_net + 2u + g;
    c->id_of[c->ip[g] - c->data_net] = g;
  }
  *out = c;
  return TGSIM_OK;
}

static void sm_free(tgo_ctx* c);
void tgo_destroy(tgo_ctx* c) {
  if (!c) return;
  free(c->fl_off); free(c->fl_nbr); free(c->fl_seen);
  free(c->tw); free(c->tsg); free(c->tpend); free(c->tack); free(c->tc);
  free(c->pr); free(c->pr_order); free(c->pr_out);
  free(c->pr_ans); free(c->pr_cur); free(c->pr_list); free(c->pr_rqa);
  sm_free(c);
  free(c->cl); free(c->epoch);
  for (size_t i = 0; i < c->n_topics; ++i) {
    free(c->topics[i].inst); free(c->topics[i].t); free(c->topics[i].off); free(c->topics[i].len);
  }
  free(c->topics); free(c->tp_bytes);
  if (c->rules) for (uint32_t i = 0; i < c->nloc; ++i) free(c->rules[i].v);
  if (c->outbox) for (uint32_t i = 0; i < c->S; ++i) free(c->outbox[i].v);
  if (c->sig) for (size_t i = 0; i < c->n_states; ++i) free(c->sig[i].t);
  free(c->sig); free(c->waiters);
  free(c->shape); free(c->X); free(c->rules); free(c->enabled); free(c->allow_ext); free(c->ip);
  free(c->id_of); free(c->inbox); free(c->outbox); free(c->xsend); free(c->xrecv);
  free(c->staged.src); free(c->staged.dst); free(c->staged.seq); free(c->staged.size); free(c->staged.t);
  free(c->status); free(c->heap.v); free(c->A.v); free(c->D.v); free(c->pend); free(c->out.v);
  free(c->tcp_rx.v);
  free(c);
}

const char* tgo_last_error(const tgo_ctx* c) { return c ? c->err : "null context"; }
int64_t tgo_now(const tgo_ctx* c) { return c->now; }
int64_t tgo_horizon(const tgo_ctx* c) { return c->horizon; }

static int is_local(const tgo_ctx* c, uint32_t g) { return g >= c->lo && g < c->hi; }

/* ============================== network configuration ======================================= */

/* NetlinkLink.Shape, link.go:155-183: HTB first (setHtb), then netem. */
int tgo_set_shape(tgo_ctx* c, uint32_t g, const tgsim_link_shape* s) {
  if (g >= c->N || !s) return fail(c, TGSIM_EINVAL, "bad instance %u", g);
  oshape o;
  int rc = derive_shape(s, &o, c->err, sizeof(c->err));
  if (rc) return rc;
  if (is_local(c, g)) {
    uint32_t l = g - c->lo;
    c->shape[l] = o;
    /* netem_change -> get_correlation -> init_crandom: every Shape re-seeds the state [EXT]; the
     * kernel seeds it from prandom, here from Philox(g, epoch, 0, "CORR") */
    if (!c->cl) {
      c->cl = (uint32_t*)calloc((size_t)c->nloc * 3 + 1, 4);
      c->epoch = (uint32_t*)calloc((size_t)c->nloc + 1, 4);
      if (!c->cl || !c->epoch) return fail(c, TGSIM_ENOMEM, "oom");
    }
    uint32_t ctr[4] = {g, ++c->epoch[l], 0, 0x434F5252u /* "CORR" */}, out[4];
    uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
    tgo_philox4x32_10(ctr, key, out);
    c->cl[3 * l] = out[0]; c->cl[3 * l + 1] = out[1]; c->cl[3 * l + 2] = out[2];
  }
  return TGSIM_OK;
}

int tgo_set_shapes(tgo_ctx* c, const uint32_t* inst, const tgsim_link_shape* shapes, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    int rc = tgo_set_shape(c, inst[i], &shapes[i]);
    if (rc) return rc;
  }
  return TGSIM_OK;
}

static int rule_cmp(uint32_t pa, uint32_t la, uint32_t pb, uint32_t lb) {
  if (la != lb) return la > lb ? -1 : 1; /* longer prefixes first */
  if (pa != pb) return pa < pb ? -1 : 1;
  return 0;
}
static size_t rule_find(const orules* r, uint32_t prefix, uint32_t plen, int* found) {
  size_t lo = 0, hi = r->n;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    int c = rule_cmp(r->v[mid].prefix, r->v[mid].plen, prefix, plen);
    if (c < 0) lo = mid + 1; else hi = mid;
  }
  *found = lo < r->n && r->v[lo].prefix == prefix && r->v[lo].plen == plen;
  return lo;
}

/* NetlinkLink.AddRules, link.go:187-217. Accept deletes the blackhole and prohibit routes for the
 * subnet (errors ignored); Reject/Drop RouteReplace a PROHIBIT/BLACKHOLE route (the kernel rejects
 * a prefix with host bits set: EINVAL, returned, later rules not applied). */
int tgo_add_rules(tgo_ctx* c, uint32_t g, const tgsim_link_rule* rules, size_t n) {
  if (g >= c->N) return fail(c, TGSIM_EINVAL, "bad instance %u", g);
  for (size_t i = 0; i < n; ++i) {
    uint32_t plen = rules[i].prefix_len;
    if (plen > 32) return fail(c, TGSIM_EINVAL, "invalid prefix length %u", plen);
    uint32_t mask = plen ? 0xFFFFFFFFu << (32 - plen) : 0u;
    uint32_t prefix = rules[i].subnet_ip;
    int action = rules[i].shape.filter;
    if (!is_local(c, g)) {
      if (action != TGSIM_FILTER_ACCEPT && (prefix & ~mask)) return fail(c, TGSIM_EINVAL, "invalid prefix for given prefix length");
      continue;
    }
    orules* r = &c->rules[g - c->lo];
    int found;
    if (action == TGSIM_FILTER_ACCEPT) {
      size_t at = rule_find(r, prefix & mask, plen, &found);
      if (found && (prefix & ~mask) == 0) {
        memmove(&r->v[at], &r->v[at + 1], (r->n - at - 1) * sizeof(orule));
        r->n--;
      }
      continue;
    }
    if (action != TGSIM_FILTER_REJECT && action != TGSIM_FILTER_DROP)
      return fail(c, TGSIM_EINVAL, "unknown filter action %d", action);
    if (prefix & ~mask) return fail(c, TGSIM_EINVAL, "invalid prefix for given prefix length");
    size_t at = rule_find(r, prefix, plen, &found);
    if (found) { r->v[at].action = action; continue; }
    if (grow((void**)&r->v, &r->cap, r->n + 1, sizeof(orule))) return fail(c, TGSIM_ENOMEM, "oom");
    memmove(&r->v[at + 1], &r->v[at], (r->n - at) * sizeof(orule));
    r->v[at].prefix = prefix; r->v[at].plen = plen; r->v[at].action = action;
    r->n++;
  }
  return TGSIM_OK;
}

/* route.go:102-117: AllowAll enables external routes, DenyAll and every other value disables. */
int tgo_set_policy(tgo_ctx* c, uint32_t g, int32_t policy) {
  if (g >= c->N) return fail(c, TGSIM_EINVAL, "bad instance %u", g);
  c->allow_ext[g] = policy == TGSIM_POLICY_ALLOW_ALL;
  return TGSIM_OK;
}

static int set_ip(tgo_ctx* c, uint32_t g, uint32_t ip) {
  if ((ip & c->data_mask) != c->data_net) return fail(c, TGSIM_EINVAL, "ip outside the data subnet");
  uint32_t off = ip - c->data_net;
  if (off == 0 || off == (uint32_t)(c->id_of_n - 1) || off == 1)
    return fail(c, TGSIM_EINVAL, "reserved address");
  if (c->id_of[off] != UINT32_MAX && c->id_of[off] != g) return fail(c, TGSIM_EINVAL, "address already in use");
  c->id_of[c->ip[g] - c->data_net] = UINT32_MAX;
  c->ip[g] = ip;
  c->id_of[off] = g;
  return TGSIM_OK;
}

/* Link disconnect / (re)connect, docker_network.go:65-133. A new link is a new HTB class + netem
 * qdisc (link.go:47-115): unshaped, unlimited, bucket full. Blackhole/prohibit routes live in the
 * netns routing table and survive. */
int tgo_set_enabled(tgo_ctx* c, uint32_t g, int32_t enabled, int32_t has_ip, uint32_t ip) {
  if (g >= c->N) return fail(c, TGSIM_EINVAL, "bad instance %u", g);
  if (!enabled) { c->enabled[g] = 0; return TGSIM_OK; }
  if (c->enabled[g] && has_ip && ip != c->ip[g]) c->enabled[g] = 0; /* disconnect to change ip */
  if (!c->enabled[g]) {
    if (has_ip) { int rc = set_ip(c, g, ip); if (rc) return rc; }
    c->enabled[g] = 1;
    if (is_local(c, g)) {
      derive_shape(&ZERO_SHAPE, &c->shape[g - c->lo], NULL, 0);
      c->X[g - c->lo] = NEG_INF;
    }
  }
  return TGSIM_OK;
}

/* DockerNetwork.ConfigureNetwork, docker_network.go:51-148, in its order. */
int tgo_configure_network(tgo_ctx* c, uint32_t g, const tgsim_network_config* cfg) {
  if (!cfg || g >= c->N) return fail(c, TGSIM_EINVAL, "bad arguments");
  const char* net = cfg->network ? cfg->network : "";
  if (strcmp(net, "default") != 0) return fail(c, TGSIM_EUNSUPPORTED_NETWORK, "unsupported network: %s", net);
  int rc = tgo_set_policy(c, g, cfg->routing_policy);
  if (rc) return rc;
  if (!cfg->enable) return tgo_set_enabled(c, g, 0, 0, 0);
  rc = tgo_set_enabled(c, g, 1, cfg->has_ipv4, cfg->ipv4);
  if (rc) return rc;
  rc = tgo_set_shape(c, g, &cfg->default_shape);
  if (rc) return rc;
  return tgo_add_rules(c, g, cfg->rules, cfg->n_rules);
}

/* K8sNetwork.ConfigureNetwork, k8s_network.go:43-176: Enable=false returns after the disconnect
 * (k8s_network.go:50-61, the policy is not applied); otherwise Shape -> AddRules -> policy
 * (k8s_network.go:166-174). A reconnect with IPv4 nil keeps the current address (IPAM not modelled). */
int tgo_configure_network_order(tgo_ctx* c, uint32_t g, const tgsim_network_config* cfg, int32_t order) {
  if (order == TGSIM_APPLY_DOCKER) return tgo_configure_network(c, g, cfg);
  if (!cfg || g >= c->N || order != TGSIM_APPLY_K8S) return fail(c, TGSIM_EINVAL, "bad arguments");
  const char* net = cfg->network ? cfg->network : "";
  if (strcmp(net, "default") != 0) return fail(c, TGSIM_EUNSUPPORTED_NETWORK, "unsupported network: %s", net);
  if (!cfg->enable) return tgo_set_enabled(c, g, 0, 0, 0);
  int rc = tgo_set_enabled(c, g, 1, cfg->has_ipv4, cfg->ipv4);
  if (rc) return rc;
  rc = tgo_set_shape(c, g, &cfg->default_shape);
  if (rc) return rc;
  rc = tgo_add_rules(c, g, cfg->rules, cfg->n_rules);
  if (rc) return rc;
  return tgo_set_policy(c, g, cfg->routing_policy);
}

int tgo_get_ip(const tgo_ctx* c, uint32_t g, uint32_t* ip) {
  if (g >= c->N) return TGSIM_EINVAL;
  *ip = c->ip[g];
  return TGSIM_OK;
}

/* ============================== data path =================================================== */

static int enqueue_impl(tgo_ctx* c, const tgsim_msg_soa* m, size_t n);
static int react_owed(tgo_ctx* c) {
  if (c->pr_need_react) return fail(c, TGSIM_ESTATE, "probes: probe_react after every window");
  if (c->sm_need_react) return fail(c, TGSIM_ESTATE, "storm: storm_react after every window");
  return TGSIM_OK;
}
int tgo_enqueue(tgo_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode: traffic goes through tcp_send");
  if (react_owed(c)) return TGSIM_ESTATE;
  return enqueue_impl(c, m, n);
}
static int enqueue_impl(tgo_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (c->in_window) return fail(c, TGSIM_ESTATE, "enqueue inside a window");
  omsgs* s = &c->staged;
  size_t need = s->n + n;
  if (need > s->cap) {
    size_t nc = s->cap ? s->cap : 1024;
    while (nc < need) nc *= 2;
    s->src = (uint32_t*)realloc(s->src, nc * 4); s->dst = (uint32_t*)realloc(s->dst, nc * 4);
    s->seq = (uint32_t*)realloc(s->seq, nc * 4); s->size = (uint32_t*)realloc(s->size, nc * 4);
    s->t = (int64_t*)realloc(s->t, nc * 8);
    if (!s->src || !s->dst || !s->seq || !s->size || !s->t) return fail(c, TGSIM_ENOMEM, "oom");
    s->cap = nc;
  }
  for (size_t i = 0; i < n; ++i) {
    if (m->src[i] >= c->N || (m->dst[i] >= c->N && m->dst[i] != TGSIM_DST_EXTERNAL))
      return fail(c, TGSIM_EINVAL, "message %zu: bad instance id", i);
    if (!is_local(c, m->src[i])) return fail(c, TGSIM_EINVAL, "message %zu: sender not in this shard", i);
    if (m->t_send[i] < c->horizon) return fail(c, TGSIM_ECAUSALITY, "message %zu: t_send before the reaction horizon", i);
    if (m->size[i] >= 0x80000000u) return fail(c, TGSIM_EINVAL, "message %zu: size too large", i);
  }
  memcpy(s->src + s->n, m->src, n * 4); memcpy(s->dst + s->n, m->dst, n * 4);
  memcpy(s->seq + s->n, m->seq, n * 4); memcpy(s->size + s->n, m->size, n * 4);
  memcpy(s->t + s->n, m->t_send, n * 8);
  s->n = need;
  return TGSIM_OK;
}

enum { R_NONE = 0, R_DATA, R_DEFAULT, R_DROP, R_REJECT };

/* Longest-prefix match over the sender's netns routing table: its blackhole/prohibit routes
 * (link.go:187-217), the data network's connected route (present while the link is enabled), the
 * default route via the control network (present under AllowAll, route.go:68-100). An equal-length
 * rule replaces the route it collides with (RouteReplace). Linear scan: obviously correct. */
static int route_lookup(const tgo_ctx* c, uint32_t g, uint32_t dst_ip) {
  int data_ok = c->enabled[g] && ((dst_ip & c->data_mask) == c->data_net);
  const orules* r = &c->rules[g - c->lo];
  for (size_t i = 0; i < r->n; ++i) {
    uint32_t plen = r->v[i].plen;
    if (data_ok && c->data_len > plen) return R_DATA;
    uint32_t mask = plen ? 0xFFFFFFFFu << (32 - plen) : 0u;
    if ((dst_ip & mask) == r->v[i].prefix) return r->v[i].action == TGSIM_FILTER_DROP ? R_DROP : R_REJECT;
  }
  if (data_ok) return R_DATA;
  if (c->allow_ext[g]) return R_DEFAULT;
  return R_NONE;
}

static void draw(const tgo_ctx* c, uint32_t seq, uint32_t src, uint32_t clone, uint32_t blk, uint32_t out[4]) {
  uint32_t ctr[4] = {seq, src, clone | (blk << 1), 0x4E45544Du /* "NETM" */};
  uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
  tgo_philox4x32_10(ctr, key, out);
}

/* netem get_crandom [EXT sch_netem.c]: the next answer leans on the last one by rho / 2^32. */
static uint32_t crandom(uint32_t* last, uint32_t rho, uint32_t value) {
  if (!last || rho == 0) return value;
  uint64_t r = (uint64_t)rho + 1;
  uint32_t ans = (uint32_t)(((uint64_t)value * ((1ull << 32) - r) + (uint64_t)*last * r) >> 32);
  *last = ans;
  return ans;
}

/* netem_enqueue [EXT sch_netem.c] for one copy, up to the queue-limit check: (clone only) its own
 * loss draw, then the corruption draw. Returns 0 if the copy is lost. */
static int netem_pre(tgo_ctx* c, const oshape* sh, uint32_t src, uint32_t dst, uint32_t seq, uint32_t size,
                     uint32_t clone, uint32_t* cl, tgsim_record* rec) {
  uint32_t r0[4];
  draw(c, seq, src, clone, 0, r0);
  if (clone && sh->loss_t && sh->loss_t >= r0[1]) return 0;
  rec->src = src; rec->dst = dst; rec->seq = seq; rec->size = size;
  rec->meta = clone ? TGSIM_F_CLONE : 0; rec->corrupt_off = 0;
  if (sh->corrupt_t) {
    uint32_t r1[4];
    draw(c, seq, src, clone, 1, r1);
    if (sh->corrupt_t >= crandom(cl ? cl + 1 : NULL, sh->corrupt_rho, r1[0]) && size > 0) {
      rec->meta |= TGSIM_F_CORRUPT | ((r1[2] % 8u) << TGSIM_F_BIT_SHIFT);
      rec->corrupt_off = r1[1] % size;
    }
  }
  return 1;
}

/* ... after the queue-limit check (the copy is queued): reorder-or-delay. */
static void netem_post(tgo_ctx* c, const oshape* sh, int64_t t_send, uint32_t* cl, tgsim_record* rec) {
  uint32_t r0[4];
  draw(c, rec->seq, rec->src, (rec->meta & TGSIM_F_CLONE) ? 1u : 0u, 0, r0);
  if (sh->reorder_t && !(sh->reorder_t < crandom(cl ? cl + 2 : NULL, sh->reorder_rho, r0[3]))) {
    /* gap == 1 when reorder > 0 (netlink NewNetem) */
    rec->meta |= TGSIM_F_REORDERED;
    rec->t = t_send;
  } else {
    int64_t delay = tabledist(sh->mu, sh->sigma, r0[2]);
    rec->t = t_send + (delay > 0 ? delay : 0);
  }
  if (!sh->limited) rec->meta |= TGSIM_F_STAGE_D; /* unlimited HTB: departs when netem releases it */
}

static _Thread_local const omsgs* g_sort_msgs; /* qsort context of cmp_msg_order (one per thread: shards of one run may share a process) */
static int cmp_msg_order(const void* a, const void* b) {
  size_t i = *(const size_t*)a, j = *(const size_t*)b;
  const omsgs* m = g_sort_msgs;
  if (m->src[i] != m->src[j]) return m->src[i] < m->src[j] ? -1 : 1;
  if (m->t[i] != m->t[j]) return m->t[i] < m->t[j] ? -1 : 1;
  if (m->seq[i] != m->seq[j]) return m->seq[i] < m->seq[j] ? -1 : 1;
  return i < j ? -1 : i > j;
}

static int cmp_tb(const void* a, const void* b) {
  const tgsim_record* x = (const tgsim_record*)a; const tgsim_record* y = (const tgsim_record*)b;
  if (x->src != y->src) return x->src < y->src ? -1 : 1;
  if (x->t != y->t) return x->t < y->t ? -1 : 1;
  if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
  uint32_t rx = (x->meta & TGSIM_F_CLONE) ? 0 : 1, ry = (y->meta & TGSIM_F_CLONE) ? 0 : 1;
  return rx < ry ? -1 : rx > ry;
}
static int cmp_dl(const void* a, const void* b) {
  const tgsim_record* x = (const tgsim_record*)a; const tgsim_record* y = (const tgsim_record*)b;
  if (x->dst != y->dst) return x->dst < y->dst ? -1 : 1;
  if (x->t != y->t) return x->t < y->t ? -1 : 1;
  if (x->src != y->src) return x->src < y->src ? -1 : 1;
  if (x->seq != y->seq) return x->seq < y->seq ? -1 : 1;
  uint32_t rx = (x->meta & TGSIM_F_CLONE) ? 0 : 1, ry = (y->meta & TGSIM_F_CLONE) ? 0 : 1;
  return rx < ry ? -1 : rx > ry;
}

/* The pending set: every copy of a local sender that has not yet departed (reached its delivery
 * time) waits in the heap; pend[l] counts local sender l's (its netem queue beyond this window). */
static int pend_push(tgo_ctx* c, const tgsim_record* r) {
  if (heap_push(&c->heap, r)) return TGSIM_ENOMEM;
  if (is_local(c, r->src)) c->pend[r->src - c->lo]++;
  return 0;
}
static tgsim_record pend_pop(tgo_ctx* c) {
  tgsim_record r = heap_pop(&c->heap);
  if (is_local(c, r.src)) c->pend[r.src - c->lo]--;
  return r;
}

/* A stage-D record (t = delivery time) of this window's sender side: delivered here if due and
 * local, exchanged if due and remote (only due records cross shards), pending otherwise. */
static int route_record(tgo_ctx* c, const tgsim_record* r) {
  if (r->t >= c->t_end) return pend_push(c, r);
  uint32_t p = shard_of(c, r->dst);
  if (p == c->cfg.shard_id) return recs_push(&c->D, r);
  return recs_push(&c->outbox[p], r);
}
/* A copy out of netem: token bucket now (A), pending, or (unlimited) a stage-D record. */
static int route_copy(tgo_ctx* c, const tgsim_record* r) {
  if (r->meta & TGSIM_F_STAGE_D) return route_record(c, r);
  if (r->t < c->t_end) return recs_push(&c->A, r);
  return pend_push(c, r);
}

/* ---- the netem queue limit -------------------------------------------------
 * Per sender, in enqueue order (t_send, seq, clone first), a copy enqueued at t is tail-dropped when
 * TGSIM_NETEM_LIMIT copies of that sender, enqueued before it, are still queued: departure d > t (a
 * copy occupies the queue over [enqueue, departure): one leaving at t has left - a zero-delay packet
 * is dequeued in the same dev_queue_xmit that enqueued it [EXT]). A copy still waiting for its HTB
 * turn (netem time >= t, departure not yet known) counts as queued. Counted within a window: the copies pending at the window start (pend + those extracted now) and
 * those queued in this window. An extracted stage-A copy's departure comes from the HTB GCRA run in
 * (netem time, seq, clone first) order as the enqueue times pass it - the same recurrence, in the
 * same order, as the token bucket below. Obvious structures: two binary heaps per sender. */
typedef struct { int64_t e; uint32_t seq, rank, size; } ou;  /* a queued copy without departure yet */
typedef struct { ou* v; size_t n, cap; } ouheap;               /* min on (e, seq, clone first) */
typedef struct { int64_t* v; size_t n, cap; } odheap;          /* min departure time */

static int ou_less(const ou* a, const ou* b) {
  if (a->e != b->e) return a->e < b->e;
  if (a->seq != b->seq) return a->seq < b->seq;
  return a->rank < b->rank;
}
static int ou_push(ouheap* h, ou x) {
  if (grow((void**)&h->v, &h->cap, h->n + 1, sizeof(ou))) return TGSIM_ENOMEM;
  size_t i = h->n++;
  h->v[i] = x;
  while (i) {
    size_t p = (i - 1) / 2;
    if (!ou_less(&h->v[i], &h->v[p])) break;
    ou t = h->v[p]; h->v[p] = h->v[i]; h->v[i] = t; i = p;
  }
  return 0;
}
static ou ou_pop(ouheap* h) {
  ou top = h->v[0];
  h->v[0] = h->v[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < h->n && ou_less(&h->v[l], &h->v[m])) m = l;
    if (r < h->n && ou_less(&h->v[r], &h->v[m])) m = r;
    if (m == i) break;
    ou t = h->v[m]; h->v[m] = h->v[i]; h->v[i] = t; i = m;
  }
  return top;
}
static int od_push(odheap* h, int64_t x) {
  if (grow((void**)&h->v, &h->cap, h->n + 1, sizeof(int64_t))) return TGSIM_ENOMEM;
  size_t i = h->n++;
  h->v[i] = x;
  while (i) {
    size_t p = (i - 1) / 2;
    if (h->v[p] <= h->v[i]) break;
    int64_t t = h->v[p]; h->v[p] = h->v[i]; h->v[i] = t; i = p;
  }
  return 0;
}
static void od_pop(odheap* h) {
  h->v[0] = h->v[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < h->n && h->v[l] < h->v[m]) m = l;
    if (r < h->n && h->v[r] < h->v[m]) m = r;
    if (m == i) break;
    int64_t t = h->v[m]; h->v[m] = h->v[i]; h->v[i] = t; i = m;
  }
}

typedef struct { uint32_t src; tgsim_record r; } oext;  /* a copy extracted (due) this window */
static int cmp_ext(const void* a, const void* b) {
  const oext* x = (const oext*)a; const oext* y = (const oext*)b;
  return x->src < y->src ? -1 : x->src > y->src;
}

/* One sender's staged messages (ord[a..b), enqueue order) through netem_enqueue with the limit. */
static int sender_window(tgo_ctx* c, const size_t* ord, size_t a, size_t b, const oext* ext, size_t ne,
                         ouheap* U, odheap* K) {
  omsgs* s = &c->staged;
  const uint32_t src = s->src[ord[a]], l = src - c->lo;
  const oshape* sh = &c->shape[l];
  uint32_t* cl = sh->corr ? c->cl + 3 * (size_t)l : NULL;
  U->n = K->n = 0;
  for (size_t j = 0; j < ne; ++j) {
    const tgsim_record* r = &ext[j].r;
    if (r->meta & TGSIM_F_STAGE_D) { if (od_push(K, r->t)) return TGSIM_ENOMEM; }
    else {
      ou u = {r->t, r->seq, (r->meta & TGSIM_F_CLONE) ? 0u : 1u, r->size};
      if (ou_push(U, u)) return TGSIM_ENOMEM;
    }
  }
  int64_t X = c->X[l];
  for (size_t k = a; k < b; ++k) {
    const size_t i = ord[k];
    const uint32_t dst = s->dst[i], seq = s->seq[i], size = s->size[i];
    const int64_t ts = s->t[i];
    /* departures up to ts: the GCRA over the queued copies whose netem time has passed */
    while (U->n && U->v[0].e < ts) {
      ou u = ou_pop(U);
      int64_t d = u.e > X ? u.e : X;
      int64_t base = X > u.e - sh->tau ? X : u.e - sh->tau;
      int64_t nx = base + (int64_t)l2t_ns(sh, u.size);
      X = nx > TB_CLAMP ? TB_CLAMP : nx;
      if (od_push(K, d)) return TGSIM_ENOMEM;
    }
    while (K->n && K->v[0] <= ts) od_pop(K);
    uint32_t r0[4];
    draw(c, seq, src, 0, 0, r0);
    int count = 1;
    int dup = sh->dup_t && sh->dup_t >= crandom(cl, sh->dup_rho, r0[0]);
    if (dup) ++count;
    int lost = sh->loss_t && sh->loss_t >= r0[1];
    if (lost) --count;
    if (count == 0) { c->status[i] = TGSIM_ST_LOST; c->stats.lost++; continue; }
    uint8_t st = TGSIM_ST_QUEUED;
    int queued = 0;
    if (dup && lost) st |= TGSIM_ST_FLAG_DUP_CANCEL;
    tgsim_record rec;
    for (uint32_t clone = (count == 2) ? 1u : 0u;; --clone) {
      /* the clone is enqueued first, through the root qdisc, duplication off */
      if (netem_pre(c, sh, src, dst, seq, size, clone, cl, &rec)) {
        const uint64_t occ = (uint64_t)c->pend[l] + U->n + K->n;
        if (occ >= TGSIM_NETEM_LIMIT) {  /* sch_netem: sch->q.qlen >= sch->limit -> drop */
          c->stats.overlimit++;
          st |= clone ? TGSIM_ST_FLAG_CLONE_LOST : TGSIM_ST_FLAG_OVERLIMIT;
        } else {
          netem_post(c, sh, ts, cl, &rec);
          c->stats.copies++;
          ++queued;
          if (rec.meta & TGSIM_F_STAGE_D) {
            if (rec.t < c->t_end && od_push(K, rec.t)) return TGSIM_ENOMEM;
          } else if (rec.t < c->t_end) {
            ou u = {rec.t, rec.seq, clone ? 0u : 1u, rec.size};
            if (ou_push(U, u)) return TGSIM_ENOMEM;
          }
          if (route_copy(c, &rec)) return TGSIM_ENOMEM;
        }
      } else {
        st |= TGSIM_ST_FLAG_CLONE_LOST;
      }
      if (clone == 1) st |= TGSIM_ST_FLAG_DUP;
      if (clone == 0) break;
    }
    if (!queued) { st = (uint8_t)((st & 0xF0u) | TGSIM_ST_OVERLIMIT); }
    c->status[i] = st;
  }
  return 0;
}

static int tcp_release(tgo_ctx* c, int64_t t_end);
int tgo_advance_begin(tgo_ctx* c, int64_t t_end) {
  if (c->in_window) return fail(c, TGSIM_ESTATE, "window already open");
  if (t_end < c->now) return fail(c, TGSIM_ECAUSALITY, "t_end before window start");
  if (react_owed(c)) return TGSIM_ESTATE;
  if (c->tcp_on) {
    if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tcp_react after every window");
    int rc = tcp_release(c, t_end);
    if (rc) return rc;
  }
  omsgs* s = &c->staged;
  for (size_t i = 0; i < s->n; ++i)
    if (s->t[i] >= t_end) return fail(c, TGSIM_ECAUSALITY, "staged message %zu sent at/after t_end", i);
  c->t_end = t_end;
  c->A.n = c->D.n = 0;
  for (uint32_t p = 0; p < c->S; ++p) c->outbox[p].n = 0;
  /* 1. due events from the pending set: netem-ready copies (token bucket now) and departures */
  oext* ext = NULL; size_t n_ext = 0, ext_cap = 0;
  while (c->heap.n && c->heap.v[0].t < t_end) {
    tgsim_record r = pend_pop(c);
    if (grow((void**)&ext, &ext_cap, n_ext + 1, sizeof(oext))) { free(ext); return TGSIM_ENOMEM; }
    ext[n_ext].src = r.src; ext[n_ext].r = r; ++n_ext;
    int rc = (r.meta & TGSIM_F_STAGE_D) ? route_record(c, &r) : recs_push(&c->A, &r);
    if (rc) { free(ext); return TGSIM_ENOMEM; }
  }
  if (n_ext) qsort(ext, n_ext, sizeof(oext), cmp_ext);
  /* 2. route + netem for every staged message; each sender's messages reach its qdisc in
   *    (t_send, seq) order, which its queue limit and crandom state follow */
  if (grow((void**)&c->status, &c->status_cap, s->n + 1, 1)) { free(ext); return fail(c, TGSIM_ENOMEM, "oom"); }
  c->n_status = s->n;
  size_t* order = (size_t*)malloc((s->n + 1) * sizeof(size_t));
  if (!order) { free(ext); return fail(c, TGSIM_ENOMEM, "oom"); }
  size_t nq = 0;  /* messages that reach a qdisc, in order[0..nq) */
  for (size_t i = 0; i < s->n; ++i) {
    uint32_t src = s->src[i], dst = s->dst[i], seq = s->seq[i], size = s->size[i];
    int64_t ts = s->t[i];
    c->stats.msgs_in++;
    if (dst == src) {
      tgsim_record r = {ts, src, dst, seq, size, TGSIM_F_LOCAL | TGSIM_F_STAGE_D, 0};
      c->status[i] = TGSIM_ST_LOCAL; c->stats.local++;
      if (route_record(c, &r)) { free(ext); free(order); return TGSIM_ENOMEM; }
      continue;
    }
    int ext_dst = dst == TGSIM_DST_EXTERNAL;
    int rt = route_lookup(c, src, ext_dst ? EXTERNAL_IP : c->ip[dst]);
    if (rt == R_DROP) { c->status[i] = TGSIM_ST_DROPPED; c->stats.dropped++; continue; }
    if (rt == R_REJECT) { c->status[i] = TGSIM_ST_REJECTED; c->stats.rejected++; continue; }
    if (rt == R_DEFAULT) {
      if (ext_dst) { c->status[i] = TGSIM_ST_EXTERNAL; c->stats.external++; }
      else { c->status[i] = TGSIM_ST_UNREACHABLE; c->stats.unreachable++; }
      continue;
    }
    if (rt == R_NONE) { c->status[i] = TGSIM_ST_UNREACHABLE; c->stats.unreachable++; continue; }
    if (!c->enabled[dst]) { c->status[i] = TGSIM_ST_DEST_DOWN; c->stats.dest_down++; continue; }
    order[nq++] = i;
  }
  g_sort_msgs = s;
  if (nq) qsort(order, nq, sizeof(size_t), cmp_msg_order);
  ouheap U = {0}; odheap K = {0};
  int rc = 0;
  size_t e0 = 0;
  for (size_t a = 0; a < nq && !rc;) {
    size_t b = a;
    const uint32_t src = s->src[order[a]];
    while (b < nq && s->src[order[b]] == src) ++b;
    while (e0 < n_ext && ext[e0].src < src) ++e0;
    size_t e1 = e0;
    while (e1 < n_ext && ext[e1].src == src) ++e1;
    rc = sender_window(c, order, a, b, ext + e0, e1 - e0, &U, &K);
    a = b;
  }
  free(U.v); free(K.v); free(order); free(ext);
  if (rc) return fail(c, rc, "oom");
  s->n = 0;
  /* 3. HTB token bucket (GCRA form): copies whose netem time is < t_end, per sender in
   *    (time_to_send, seq, clone-first) order; d = max(e, X); X = min(max(X, e - tau) + cost, 2^61). */
  if (c->A.n) qsort(c->A.v, c->A.n, sizeof(tgsim_record), cmp_tb);
  for (size_t i = 0; i < c->A.n; ++i) {
    tgsim_record r = c->A.v[i];
    uint32_t l = r.src - c->lo;
    const oshape* sh = &c->shape[l];
    int64_t X = c->X[l];
    int64_t d = r.t > X ? r.t : X;
    int64_t base = X > r.t - sh->tau ? X : r.t - sh->tau;
    int64_t nx = base + (int64_t)l2t_ns(sh, r.size);
    c->X[l] = nx > TB_CLAMP ? TB_CLAMP : nx;
    r.t = d;
    r.meta |= TGSIM_F_STAGE_D;
    if (route_record(c, &r)) return TGSIM_ENOMEM;
  }
  /* 4. pack the exchange (peer-major blocks, header record .t = count). The per-peer bound is the
   * device block's usable records: below 513 records one slice of xcap - 1, else 8 slices of
   * (xcap - 1) / 8 (include/tgsim.h exchange_cap), so both refuse the same windows. */
  memset(c->xsend, 0, (size_t)c->S * c->xcap * sizeof(tgsim_record));
  const size_t xslices = c->xcap - 1 >= 8 * 64 ? 8 : 1, xusable = (c->xcap - 1) / xslices * xslices;
  for (uint32_t p = 0; p < c->S; ++p) {
    orecs* o = &c->outbox[p];
    if (o->n > xusable) return fail(c, TGSIM_ECAPACITY, "exchange capacity exceeded (%zu records to peer %u)", o->n, p);
    c->xsend[(size_t)p * c->xcap].t = (int64_t)o->n;
    memcpy(&c->xsend[(size_t)p * c->xcap + 1], o->v, o->n * sizeof(tgsim_record));
  }
  c->in_window = 1;
  c->tcp_need_react = c->tcp_on;
  c->pr_need_react = c->pr != NULL;
  c->sm_need_react = c->sm != NULL;
  return TGSIM_OK;
}

int tgo_exchange_buffers(tgo_ctx* c, void** send, void** recv, size_t* bytes) {
  *send = c->xsend; *recv = c->xrecv;
  *bytes = (size_t)c->S * c->xcap * sizeof(tgsim_record);
  return TGSIM_OK;
}

int tgo_advance_end(tgo_ctx* c) {
  if (!c->in_window) return fail(c, TGSIM_ESTATE, "no open window");
  /* 5. received records (all due this window) join this shard's deliveries */
  if (c->S > 1) {
    for (uint32_t p = 0; p < c->S; ++p) {
      if (p == c->cfg.shard_id) continue;
      const tgsim_record* blk = &c->xrecv[(size_t)p * c->xcap];
      size_t n = (size_t)blk[0].t;
      if (n + 1 > c->xcap) return fail(c, TGSIM_ECAPACITY, "corrupt exchange header");
      for (size_t i = 0; i < n; ++i) {
        if (blk[1 + i].t >= c->t_end) return fail(c, TGSIM_ECAPACITY, "exchanged record not due");
        if (recs_push(&c->D, &blk[1 + i])) return TGSIM_ENOMEM;
      }
    }
  }
  /* 6. deliveries: inbox order (dst, t, src, seq, clone-first) */
  if (c->D.n) qsort(c->D.v, c->D.n, sizeof(tgsim_record), cmp_dl);
  c->out.n = 0;
  if (grow((void**)&c->out.v, &c->out.cap, c->D.n + 1, sizeof(tgsim_record))) return TGSIM_ENOMEM;
  memcpy(c->out.v, c->D.v, c->D.n * sizeof(tgsim_record));
  c->out.n = c->D.n;
  memset(c->inbox, 0, (c->nloc + 1) * sizeof(uint32_t));
  for (size_t i = 0; i < c->out.n; ++i) c->inbox[c->out.v[i].dst - c->lo + 1]++;
  for (uint32_t i = 0; i < c->nloc; ++i) c->inbox[i + 1] += c->inbox[i];
  c->stats.delivered += c->out.n;
  c->stats.windows++;
  c->stats.inflight = c->heap.n;
  c->horizon = c->now;
  c->now = c->t_end;
  c->in_window = 0;
  return TGSIM_OK;
}

/* A shard whose sharded call fails tells the others (tgsim_transport.abort): their pending and later
 * collectives fail instead of waiting for it; this context refuses sharded calls from then on. */
static int shard_failed(tgo_ctx* c, int rc) {
  if (rc && c->S > 1 && c->has_tr) {
    if (c->tr.abort) c->tr.abort(c->tr.user);
    c->has_tr = 0;
    c->tr_aborted = 1;
  }
  return rc;
}

int tgo_comm_abort(tgo_ctx* c) {
  (void)shard_failed(c, TGSIM_ESTATE);
  return TGSIM_OK;
}

int tgo_set_transport(tgo_ctx* c, const tgsim_transport* t) {
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (t && (!t->alltoall || !t->allreduce_max_i64 || !t->allgather)) return fail(c, TGSIM_EINVAL, "incomplete transport");
  c->has_tr = t != NULL;
  c->tr_aborted = 0;
  if (t) c->tr = *t; else memset(&c->tr, 0, sizeof(c->tr));
  return TGSIM_OK;
}

/* One window; sharded: collective, the exchange between the sender and receiver halves. */
static int advance_impl(tgo_ctx* c, int64_t t_end) {
  if (c->S != 1 && !c->has_tr)
    return fail(c, TGSIM_ESTATE, c->tr_aborted ? "the transport was aborted (a shard failed)"
                                               : "a sharded context needs a transport or begin/end");
  int rc = tgo_advance_begin(c, t_end);
  if (rc) return rc;
  if (c->S != 1 && c->tr.alltoall(c->tr.user, c->xsend, c->xrecv, c->xcap * sizeof(tgsim_record), NULL) != 0) {
    c->in_window = 0;
    return fail(c, TGSIM_EHIP, "transport all-to-all failed");
  }
  return tgo_advance_end(c);
}
int tgo_advance(tgo_ctx* c, int64_t t_end) { return shard_failed(c, advance_impl(c, t_end)); }

/* The CPU model has no stream: the same call as tgo_advance. */
int tgo_advance_async(tgo_ctx* c, int64_t t_end) { return tgo_advance(c, t_end); }

int tgo_delivery_count(tgo_ctx* c, size_t* n) { *n = c->out.n; return 0; }

int tgo_copy_deliveries(tgo_ctx* c, tgsim_delivery_soa* o, size_t cap, size_t* n) {
  *n = c->out.n;
  if (c->out.n > cap) return fail(c, TGSIM_ECAPACITY, "output capacity");
  for (size_t i = 0; i < c->out.n; ++i) {
    const tgsim_record* r = &c->out.v[i];
    o->t_deliver[i] = r->t; o->src[i] = r->src; o->dst[i] = r->dst; o->seq[i] = r->seq;
    o->size[i] = r->size; o->flags[i] = r->meta & ~(uint32_t)TGSIM_F_STAGE_D; o->corrupt_off[i] = r->corrupt_off;
  }
  return TGSIM_OK;
}

int tgo_copy_inbox_offsets(tgo_ctx* c, uint32_t* out, size_t cap) {
  if (cap < (size_t)c->nloc + 1) return TGSIM_ECAPACITY;
  memcpy(out, c->inbox, (c->nloc + 1) * sizeof(uint32_t));
  return 0;
}

int tgo_copy_status(tgo_ctx* c, uint8_t* out, size_t cap, size_t* n) {
  *n = c->n_status;
  if (c->n_status > cap) return TGSIM_ECAPACITY;
  memcpy(out, c->status, c->n_status);
  return 0;
}

int tgo_get_stats(tgo_ctx* c, tgsim_stats* out) { *out = c->stats; out->inflight = c->heap.n; return 0; }  /* tb_items/extracted/inserted stay 0: structure-specific */

/* ============================== sync service ================================================ */
/* sdk-go sync.Client [EXT]: SignalEntry increments the state's counter and returns the new value
 * (1-based seq); Barrier(state, target) fires once the counter reaches target. Simulated: a batch
 * is ordered by (t, instance); signal times per state never go backwards across batches. */

typedef struct { uint32_t state, inst; int64_t t; size_t idx; } osig;
static int cmp_sig(const void* a, const void* b) {
  const osig* x = (const osig*)a; const osig* y = (const osig*)b;
  if (x->state != y->state) return x->state < y->state ? -1 : 1;
  if (x->t != y->t) return x->t < y->t ? -1 : 1;
  if (x->inst != y->inst) return x->inst < y->inst ? -1 : 1;
  return x->idx < y->idx ? -1 : x->idx > y->idx;
}

static int ensure_state(tgo_ctx* c, uint32_t st) {
  if (st >= (1u << 24)) return fail(c, TGSIM_EINVAL, "state id too large");
  if (st < c->n_states) return 0;
  size_t nn = c->n_states ? c->n_states : 16;
  while (nn <= st) nn *= 2;
  otimes* v = (otimes*)realloc(c->sig, nn * sizeof(otimes));
  if (!v) return TGSIM_ENOMEM;
  memset(v + c->n_states, 0, (nn - c->n_states) * sizeof(otimes));
  c->sig = v; c->n_states = nn;
  return 0;
}

static int sync_signal_local(tgo_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                             size_t n, uint32_t* seq_out);

/* A sharded batch with a transport: every shard's signals in shard order, processed whole on every
 * shard (replicated sync state); seq_out = this shard's own sequence numbers. */
static int sync_signal_gathered(tgo_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                                size_t n, uint32_t* seq_out);
int tgo_sync_signal(tgo_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                    size_t n, uint32_t* seq_out) {
  if (c->S == 1 || !c->has_tr || c->replicated_batch) return sync_signal_local(c, states, inst, t, n, seq_out);
  return shard_failed(c, sync_signal_gathered(c, states, inst, t, n, seq_out));
}
static int sync_signal_gathered(tgo_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                                size_t n, uint32_t* seq_out) {
  typedef struct { uint32_t state, inst; int64_t t; } grec;
  uint64_t n64 = n;
  uint64_t* sizes = (uint64_t*)calloc(c->S, 8);
  if (!sizes) return TGSIM_ENOMEM;
  if (c->tr.allgather(c->tr.user, &n64, sizes, 8, NULL) != 0) { free(sizes); return fail(c, TGSIM_EHIP, "all-gather failed"); }
  uint64_t maxn = 0, total = 0, mine = 0;
  for (uint32_t k = 0; k < c->S; ++k) {
    if (k == c->cfg.shard_id) mine = total;
    if (sizes[k] > maxn) maxn = sizes[k];
    total += sizes[k];
  }
  int rc = TGSIM_OK;
  grec* loc = (grec*)calloc(maxn + 1, sizeof(grec));
  grec* all = (grec*)calloc(maxn * c->S + 1, sizeof(grec));
  uint32_t* gs = (uint32_t*)malloc((total + 1) * 4); uint32_t* gi = (uint32_t*)malloc((total + 1) * 4);
  uint32_t* gq = (uint32_t*)malloc((total + 1) * 4); int64_t* gt = (int64_t*)malloc((total + 1) * 8);
  if (!loc || !all || !gs || !gi || !gq || !gt) rc = TGSIM_ENOMEM;
  if (!rc && maxn) {
    for (size_t i = 0; i < n; ++i) { loc[i].state = states[i]; loc[i].inst = inst[i]; loc[i].t = t[i]; }
    if (c->tr.allgather(c->tr.user, loc, all, maxn * sizeof(grec), NULL) != 0) rc = fail(c, TGSIM_EHIP, "all-gather failed");
  }
  if (!rc) {
    size_t j = 0;
    for (uint32_t k = 0; k < c->S; ++k)
      for (uint64_t i = 0; i < sizes[k]; ++i, ++j) {
        const grec* r = &all[(size_t)k * maxn + i];
        gs[j] = r->state; gi[j] = r->inst; gt[j] = r->t;
      }
    rc = sync_signal_local(c, gs, gi, gt, total, gq);
    if (!rc && seq_out && n) memcpy(seq_out, gq + mine, n * 4);
  }
  free(sizes); free(loc); free(all); free(gs); free(gi); free(gq); free(gt);
  return rc;
}

static int sync_signal_local(tgo_ctx* c, const uint32_t* states, const uint32_t* inst, const int64_t* t,
                             size_t n, uint32_t* seq_out) {
  if (n == 0) return 0;
  osig* v = (osig*)malloc(n * sizeof(osig));
  if (!v) return TGSIM_ENOMEM;
  for (size_t i = 0; i < n; ++i) {
    int rc = ensure_state(c, states[i]);
    if (rc) { free(v); return rc; }
    otimes* ts = &c->sig[states[i]];
    if (t[i] < 0 || (ts->n && t[i] < ts->t[ts->n - 1])) { free(v); return fail(c, TGSIM_ECAUSALITY, "signal %zu goes back in time", i); }
    v[i].state = states[i]; v[i].inst = inst[i]; v[i].t = t[i]; v[i].idx = i;
  }
  qsort(v, n, sizeof(osig), cmp_sig);
  for (size_t i = 0; i < n; ++i) {
    otimes* ts = &c->sig[v[i].state];
    if (grow((void**)&ts->t, &ts->cap, ts->n + 1, sizeof(int64_t))) { free(v); return TGSIM_ENOMEM; }
    ts->t[ts->n++] = v[i].t;
    if (seq_out) seq_out[v[i].idx] = (uint32_t)ts->n;
  }
  free(v);
  return 0;
}

int tgo_sync_barrier(tgo_ctx* c, uint32_t state, uint32_t target, int64_t t_wait, uint32_t* w) {
  if (t_wait == TGSIM_T_NOW) t_wait = c->now;
  int rc = ensure_state(c, state);
  if (rc) return rc;
  if (grow((void**)&c->waiters, &c->waiters_cap, c->n_waiters + 1, sizeof(owaiter))) return TGSIM_ENOMEM;
  c->waiters[c->n_waiters].state = state; c->waiters[c->n_waiters].target = target;
  c->waiters[c->n_waiters].t_wait = t_wait;
  *w = (uint32_t)c->n_waiters++;
  return 0;
}

int tgo_sync_poll(tgo_ctx* c, uint32_t w, int64_t* rel) {
  if (w >= c->n_waiters) return fail(c, TGSIM_EINVAL, "bad waiter");
  owaiter* x = &c->waiters[w];
  const otimes* ts = &c->sig[x->state];
  if (x->target == 0) { *rel = x->t_wait; return 0; }
  if (ts->n < x->target) { *rel = -1; return 0; }
  int64_t tk = ts->t[x->target - 1];
  *rel = tk > x->t_wait ? tk : x->t_wait;
  return 0;
}

int tgo_sync_count(tgo_ctx* c, uint32_t state, uint32_t* count) {
  *count = state < c->n_states ? (uint32_t)c->sig[state].n : 0;
  return 0;
}

int tgo_advance_to_barrier(tgo_ctx* c, uint32_t w, int64_t offset) {
  int64_t rel;
  int rc = tgo_sync_poll(c, w, &rel);
  if (rc) return shard_failed(c, rc);
  if (rel < 0) return shard_failed(c, fail(c, TGSIM_ESTATE, "barrier not released"));
  return tgo_advance(c, rel + offset);
}

/* ============================== workload: gossip storm =============== */
/* Instance g picks `fanout` distinct peers != g by Philox (rejection on repeats), sends `size` bytes
 * to each at t0 + U[0, spread), and signals `state` at its last send (the SignalAndWait pattern of
 * plans/benchmarks/benchmarks.go:122-141 around a storm round, plans/benchmarks/storm.go:150-197). */
static int gen_storm_impl(tgo_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                          int64_t spread_ns, uint32_t state, int tcp);
int tgo_gen_storm_round(tgo_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                        int64_t spread_ns, uint32_t state) {
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode: tcp_gen_storm_round");
  if (react_owed(c)) return TGSIM_ESTATE;
  return gen_storm_impl(c, round, t0, fanout, size, spread_ns, state, 0);
}

/* The storm round as TCP writes (one segment each: size <= mss), staged like tgo_tcp_send. */
int tgo_tcp_gen_storm_round(tgo_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                            int64_t spread_ns, uint32_t state) {
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (size > c->tcp.mss) return fail(c, TGSIM_EINVAL, "a storm write must fit one segment");
  if (c->S != 1) {  /* the wire ids: every round of one fanout, and within the packets' 27/28 bits */
    if (c->tcp_F && c->tcp_F != fanout) return fail(c, TGSIM_ENOTSUP, "sharded TCP storms keep one fanout");
    const uint64_t rounds = (uint64_t)c->tsg_n / ((uint64_t)c->nloc * fanout) + 1;
    if (rounds * c->N * fanout > (c->tcp.acks ? (1ull << 27) : (1ull << 28)))
      return fail(c, TGSIM_ECAPACITY, "TCP segment ids beyond the packets' seq bits");
    c->tcp_F = fanout;
  }
  return gen_storm_impl(c, round, t0, fanout, size, spread_ns, state, 1);
}

static int tcp_send_impl(tgo_ctx* c, const tgsim_msg_soa* m, size_t n);
static int gen_storm_impl(tgo_ctx* c, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                          int64_t spread_ns, uint32_t state, int tcp) {
  if (fanout == 0 || fanout >= c->N || fanout > 32) return fail(c, TGSIM_EINVAL, "bad fanout");
  if (t0 == TGSIM_T_NOW) t0 = c->now;
  size_t n = (size_t)c->nloc * fanout;
  uint32_t* src = (uint32_t*)malloc(n * 4); uint32_t* dst = (uint32_t*)malloc(n * 4);
  uint32_t* seq = (uint32_t*)malloc(n * 4); uint32_t* sz = (uint32_t*)malloc(n * 4);
  int64_t* ts = (int64_t*)malloc(n * 8);
  uint32_t* sst = (uint32_t*)malloc(c->nloc * 4); uint32_t* sin = (uint32_t*)malloc(c->nloc * 4);
  int64_t* stt = (int64_t*)malloc(c->nloc * 8);
  int rc = TGSIM_ENOMEM;
  if (!src || !dst || !seq || !sz || !ts || !sst || !sin || !stt) goto out;
  uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
  for (uint32_t l = 0; l < c->nloc; ++l) {
    uint32_t g = c->lo + l;
    uint32_t chosen[64];
    int64_t tmax = t0;
    for (uint32_t k = 0; k < fanout; ++k) {
      uint32_t out[4], p;
      uint32_t ctr[4] = {g, round, k << 16, 0x53544F52u /* "STOR" */};
      tgo_philox4x32_10(ctr, key, out);
      uint64_t u = ((uint64_t)out[2] << 32) | out[1];
      int64_t t = t0 + (spread_ns > 0 ? (int64_t)(u % (uint64_t)spread_ns) : 0);
      for (uint32_t attempt = 0;; ++attempt) {
        if (attempt) { uint32_t ctr2[4] = {g, round, (k << 16) | attempt, 0x53544F52u}; tgo_philox4x32_10(ctr2, key, out); }
        p = out[0] % (c->N - 1);
        if (p >= g) ++p;
        int dupl = 0;
        for (uint32_t j = 0; j < k; ++j) dupl |= chosen[j] == p;
        if (!dupl) break;
      }
      chosen[k] = p;
      size_t i = (size_t)l * fanout + k;
      src[i] = g; dst[i] = p; seq[i] = round * fanout + k; sz[i] = size; ts[i] = t;
      if (t > tmax) tmax = t;
    }
    sst[l] = state; sin[l] = g; stt[l] = tmax;
  }
  tgsim_msg_soa m = {src, dst, seq, sz, ts};
  rc = tcp ? tcp_send_impl(c, &m, n) : enqueue_impl(c, &m, n);
  /* single shard, or sharded with a transport (the batch is gathered: replicated sync state) */
  if (!rc && (c->S == 1 || c->has_tr)) rc = tgo_sync_signal(c, sst, sin, stt, c->nloc, NULL);
  if (!rc && c->S > 1 && !c->has_tr) { /* sharded: the caller MAX-reduces the local release across shards */
    int64_t mx = INT64_MIN;
    for (uint32_t l = 0; l < c->nloc; ++l) mx = stt[l] > mx ? stt[l] : mx;
    c->storm_release = mx;
  }
out:
  free(src); free(dst); free(seq); free(sz); free(ts); free(sst); free(sin); free(stt);
  return rc;
}

int tgo_storm_release(tgo_ctx* c, int64_t* out) {
  if (c->S == 1) return fail(c, TGSIM_ESTATE, "single-shard storms commit their signals: use a barrier");
  *out = c->storm_release;
  return TGSIM_OK;
}

/* ============================== flood (config 5) ============================================
 * Workload of SURVEY.md 8(d) config 5 / BASELINE.json configs[4]: a publication floods a fixed
 * graph; an instance forwards it on first receipt to every neighbour except the one it came from
 * (the gossip/flood pattern pubsub plans run over their peers, cf. plans/benchmarks/storm.go:31-197
 * for the message fan-out and plans/network/pingpong.go:219-245 for the per-instance address
 * exchange that builds the peer lists). Message seq = pub * D + neighbour slot (D = max degree),
 * so (src, seq) is unique per run; a forward leaves at max(t_deliver, horizon). */

static int fl_seen_get(const tgo_ctx* c, uint32_t p, uint32_t l) {
  return (c->fl_seen[(size_t)p * c->fl_wpp + (l >> 5)] >> (l & 31)) & 1u;
}
static void fl_seen_set(tgo_ctx* c, uint32_t p, uint32_t l) {
  c->fl_seen[(size_t)p * c->fl_wpp + (l >> 5)] |= 1u << (l & 31);
}

int tgo_flood_set_graph(tgo_ctx* c, const uint32_t* off, const uint32_t* nbr, uint32_t max_pubs) {
  if (!off || (off[c->N] && !nbr) || max_pubs == 0) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->pr) return fail(c, TGSIM_ESTATE, "probes are set up: floods need the deliveries to themselves");
  if (c->sm) return fail(c, TGSIM_ESTATE, "a storm reactor is set up: floods need the deliveries to themselves");
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is on: flood workloads need message mode");
  uint32_t D = 1;
  for (uint32_t g = 0; g < c->N; ++g) {
    if (off[g + 1] < off[g]) return fail(c, TGSIM_EINVAL, "offsets not monotonic");
    uint32_t len = off[g + 1] - off[g];
    if (len > 64) return fail(c, TGSIM_EINVAL, "degree %u > 64", len);
    if (len > D) D = len;
    for (uint32_t k = off[g]; k < off[g + 1]; ++k)
      if (nbr[k] >= c->N || nbr[k] == g) return fail(c, TGSIM_EINVAL, "bad neighbour of %u", g);
  }
  if ((uint64_t)max_pubs * D > 0x100000000ull) return fail(c, TGSIM_EINVAL, "max_pubs * degree > 2^32");
  free(c->fl_off); free(c->fl_nbr); free(c->fl_seen);
  uint32_t base = off[c->lo], m = off[c->hi] - base;
  c->fl_off = (uint32_t*)malloc((c->nloc + 1) * 4);
  c->fl_nbr = (uint32_t*)malloc((m ? m : 1) * 4);
  c->fl_wpp = (c->nloc + 31) / 32;
  c->fl_seen = (uint32_t*)calloc((size_t)max_pubs * c->fl_wpp + 1, 4);
  if (!c->fl_off || !c->fl_nbr || !c->fl_seen) return fail(c, TGSIM_ENOMEM, "oom");
  for (uint32_t l = 0; l <= c->nloc; ++l) c->fl_off[l] = off[c->lo + l] - base;
  if (m) memcpy(c->fl_nbr, nbr + base, (size_t)m * 4);
  c->fl_D = D; c->fl_max_pubs = max_pubs;
  return TGSIM_OK;
}

/* forwards of local instance l for publication p (excluding neighbour `from`), appended to m */
static void fl_emit(const tgo_ctx* c, uint32_t l, uint32_t p, uint32_t from, int64_t t, uint32_t size,
                    uint32_t* src, uint32_t* dst, uint32_t* seq, uint32_t* sz, int64_t* ts, size_t* n) {
  for (uint32_t k = c->fl_off[l]; k < c->fl_off[l + 1]; ++k) {
    uint32_t v = c->fl_nbr[k];
    if (v == from) continue;
    src[*n] = c->lo + l; dst[*n] = v; seq[*n] = p * c->fl_D + (k - c->fl_off[l]); sz[*n] = size; ts[*n] = t;
    ++*n;
  }
}

static int fl_enqueue(tgo_ctx* c, size_t cap, uint32_t* src, uint32_t* dst, uint32_t* seq, uint32_t* sz,
                      int64_t* ts, size_t n) {
  (void)cap;
  tgsim_msg_soa m = {src, dst, seq, sz, ts};
  return tgo_enqueue(c, &m, n);
}

int tgo_flood_publish(tgo_ctx* c, const uint32_t* inst, const uint32_t* pubs, const int64_t* t, size_t n,
                      uint32_t size) {
  if (!c->fl_off) return fail(c, TGSIM_ESTATE, "no flood graph");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (n && (!inst || !pubs || !t)) return fail(c, TGSIM_EINVAL, "bad arguments");
  for (size_t i = 0; i < n; ++i)
    if (inst[i] >= c->N || pubs[i] >= c->fl_max_pubs) return fail(c, TGSIM_EINVAL, "bad publication %zu", i);
  size_t cap = n * c->fl_D + 1, k = 0;
  uint32_t* src = malloc(cap * 4); uint32_t* dst = malloc(cap * 4); uint32_t* seq = malloc(cap * 4);
  uint32_t* sz = malloc(cap * 4); int64_t* ts = malloc(cap * 8);
  int rc = TGSIM_ENOMEM;
  if (src && dst && seq && sz && ts) {
    for (size_t i = 0; i < n; ++i)
      if (inst[i] >= c->lo && inst[i] < c->hi) fl_emit(c, inst[i] - c->lo, pubs[i], UINT32_MAX, t[i], size, src, dst, seq, sz, ts, &k);
    rc = fl_enqueue(c, cap, src, dst, seq, sz, ts, k);
    if (!rc)
      for (size_t i = 0; i < n; ++i)
        if (inst[i] >= c->lo && inst[i] < c->hi) fl_seen_set(c, pubs[i], inst[i] - c->lo);
  }
  free(src); free(dst); free(seq); free(sz); free(ts);
  return rc;
}

int tgo_flood_react(tgo_ctx* c, uint32_t size, size_t* n_fwd) {
  if (!c->fl_off) return fail(c, TGSIM_ESTATE, "no flood graph");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is on: flood workloads need message mode");
  const orecs* o = &c->out;
  size_t cap = o->n * c->fl_D + 1, k = 0;
  uint32_t* src = malloc(cap * 4); uint32_t* dst = malloc(cap * 4); uint32_t* seq = malloc(cap * 4);
  uint32_t* sz = malloc(cap * 4); int64_t* ts = malloc(cap * 8);
  int rc = TGSIM_ENOMEM;
  if (src && dst && seq && sz && ts) {
    rc = TGSIM_OK;
    for (size_t i = 0; i < o->n; ++i) {   /* inbox order: (dst, t, src, seq, clone first) */
      const tgsim_record* r = &o->v[i];
      uint32_t p = r->seq / c->fl_D, l = r->dst - c->lo;
      if (p >= c->fl_max_pubs) { rc = fail(c, TGSIM_EINVAL, "delivery %zu is not a flood message", i); break; }
      if (fl_seen_get(c, p, l)) continue;
      fl_seen_set(c, p, l);
      fl_emit(c, l, p, r->src, r->t > c->horizon ? r->t : c->horizon, size, src, dst, seq, sz, ts, &k);
    }
    if (!rc) rc = fl_enqueue(c, cap, src, dst, seq, sz, ts, k);
  }
  free(src); free(dst); free(seq); free(sz); free(ts);
  if (n_fwd) *n_fwd = rc ? 0 : k;
  return rc;
}

/* ============================== sequential probes ===========================
 * plans/splitbrain/main.go:153-175: each node GETs its peers one at a time (http.Client{Timeout:
 * time.Minute}); the next GET starts when the previous one returned. A probe is a request and its
 * reply; it ends OK at the reply's first arrival before the deadline, REFUSED at once when the
 * prober's own route refuses the request (a local route error fails connect() immediately [EXT]),
 * TIMEOUT at the deadline otherwise. */

enum { PR_IDLE = 0, PR_WAIT = 1, PR_DONE = 2 };
#define PR_NONE INT64_MAX
#define PR_MASK 0x3FFFFFFFu
typedef struct oprobe {
  uint32_t pos, state, refused, replied;  /* replied: 0, 1, 2 = the peer's notice came in this reaction */
  int64_t t_req, t_rep, t_reparr, t_done;
} oprobe;

int tgo_probe_setup(tgo_ctx* c, const uint32_t* order, uint32_t n_order, const tgsim_probe_config* cfg) {
  if (!order || !cfg || n_order == 0 || n_order > PR_MASK) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (cfg->timeout_ns <= 0 || cfg->window_ns <= 0 || cfg->request_bytes >= 0x80000000u || cfg->reply_bytes >= 0x80000000u)
    return fail(c, TGSIM_EINVAL, "bad probe configuration");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->S != 1 && !c->has_tr) return fail(c, TGSIM_ESTATE, "a sharded context needs a transport for probes");
  if (c->N > PR_MASK) return fail(c, TGSIM_ENOTSUP, "too many instances for probe tags");
  if (c->tcp_on || c->fl_off) return fail(c, TGSIM_ESTATE, "probes run in message mode, without a flood graph");
  if (c->sm) return fail(c, TGSIM_ESTATE, "a storm reactor is set up: it owns the deliveries");
  for (uint32_t j = 0; j < n_order; ++j)
    if (order[j] >= c->N) return fail(c, TGSIM_EINVAL, "order[%u] is not an instance", j);
  oprobe* pr = (oprobe*)calloc(c->nloc ? c->nloc : 1, sizeof(oprobe));
  uint32_t* ord = (uint32_t*)malloc((size_t)n_order * 4);
  uint8_t* out = (uint8_t*)calloc((size_t)(c->nloc ? c->nloc : 1) * n_order, 1);
  if (!pr || !ord || !out) { free(pr); free(ord); free(out); return fail(c, TGSIM_ENOMEM, "oom"); }
  memcpy(ord, order, (size_t)n_order * 4);
  for (uint32_t l = 0; l < c->nloc; ++l) pr[l].t_done = INT64_MIN;
  free(c->pr); free(c->pr_order); free(c->pr_out);
  free(c->pr_ans); free(c->pr_cur); free(c->pr_list); free(c->pr_rqa);
  c->pr_ans = (uint32_t*)calloc(c->N, 4); c->pr_cur = (uint32_t*)calloc(c->N, 4);
  c->pr_list = (uint32_t*)calloc(c->N, 4); c->pr_rqa = (int64_t*)malloc((size_t)c->N * 8);
  if (!c->pr_ans || !c->pr_cur || !c->pr_list || !c->pr_rqa) return fail(c, TGSIM_ENOMEM, "oom");
  for (uint32_t g = 0; g < c->N; ++g) c->pr_rqa[g] = PR_NONE;
  c->pr = pr; c->pr_order = ord; c->pr_out = out; c->pr_n = n_order; c->pr_cfg = *cfg;
  c->pr_need_react = 0;
  return TGSIM_OK;
}

/* The next position after pos (or the first, pos = UINT32_MAX) that is not the prober itself. */
static uint32_t pr_next(const tgo_ctx* c, const oprobe* p, uint32_t pos) {
  uint32_t j = pos == UINT32_MAX ? 0 : pos + 1;
  while (j < c->pr_n && c->pr_order[j] == c->lo + (uint32_t)(p - c->pr)) ++j;
  return j;
}

typedef struct { uint32_t* src; uint32_t* dst; uint32_t* seq; uint32_t* size; int64_t* t; size_t n; } pbuf;
static void pr_stage(pbuf* b, uint32_t src, uint32_t dst, uint32_t seq, uint32_t size, int64_t t) {
  b->src[b->n] = src; b->dst[b->n] = dst; b->seq[b->n] = seq; b->size[b->n] = size; b->t[b->n] = t; ++b->n;
}
/* the previous probe of local l ended at te: probe pos leaves at max(te, H), or l is done at te */
static void pr_begin(tgo_ctx* c, uint32_t l, uint32_t pos, int64_t te, int64_t H, pbuf* b) {
  oprobe* p = &c->pr[l];
  if (pos >= c->pr_n) { p->state = PR_DONE; p->t_done = te; p->pos = c->pr_n; return; }
  const int64_t t = te > H ? te : H;
  p->state = PR_WAIT; p->pos = pos; p->t_req = t;
  p->refused = p->replied = 0; p->t_rep = p->t_reparr = PR_NONE;
  pr_stage(b, c->lo + l, c->pr_order[pos], TGSIM_PROBE_REQ | pos, c->pr_cfg.request_bytes, t);
}
static int pr_alloc(pbuf* b, size_t cap) {
  b->n = 0;
  b->src = malloc(cap * 4); b->dst = malloc(cap * 4); b->seq = malloc(cap * 4); b->size = malloc(cap * 4);
  b->t = malloc(cap * 8);
  return b->src && b->dst && b->seq && b->size && b->t ? 0 : TGSIM_ENOMEM;
}
static void pr_free(pbuf* b) { free(b->src); free(b->dst); free(b->seq); free(b->size); free(b->t); }
static int pr_flush(tgo_ctx* c, pbuf* b) {
  tgsim_msg_soa m = {b->src, b->dst, b->seq, b->size, b->t};
  int rc = b->n ? tgo_enqueue(c, &m, b->n) : TGSIM_OK;
  pr_free(b);
  return rc;
}

int tgo_probe_start(tgo_ctx* c, int64_t t0) {
  if (!c->pr) return fail(c, TGSIM_ESTATE, "no probes set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (react_owed(c)) return TGSIM_ESTATE;
  if (t0 < c->horizon) return fail(c, TGSIM_ECAUSALITY, "t0 before the reaction horizon");
  pbuf b;
  if (pr_alloc(&b, (size_t)c->nloc + 1)) { pr_free(&b); return fail(c, TGSIM_ENOMEM, "oom"); }
  for (uint32_t l = 0; l < c->nloc; ++l)
    if (c->pr[l].state == PR_IDLE) pr_begin(c, l, pr_next(c, &c->pr[l], UINT32_MAX), t0, t0, &b);
  return pr_flush(c, &b);
}

/* Notices to a prober's shard: its peer answered request `pos` with a reply sent at t (record: t,
 * src = prober, dst = position, seq = PRN_REPLY) */
enum { PRN_REPLY = 3u };
static void pr_notice_apply(tgo_ctx* c, uint32_t g, uint32_t pos, int64_t t) {
  if (g < c->lo || g >= c->hi) return;
  oprobe* p = &c->pr[g - c->lo];
  if (p->state != PR_WAIT || p->pos != pos) return;  /* a request the prober has moved past */
  p->replied = 2;                                       /* 2: answered in this reaction */
  p->t_rep = t;
}

static int probe_react_impl(tgo_ctx* c, int64_t* next_end, uint32_t* n_active) {
  if (!c->pr) return fail(c, TGSIM_ESTATE, "no probes set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (!c->pr_need_react) return fail(c, TGSIM_ESTATE, "probes: no window since the last reaction");
  if (c->S != 1 && !c->has_tr) return fail(c, TGSIM_ESTATE, "the transport was aborted (a shard failed)");
  c->pr_need_react = 0;  /* the window's staged rows are read exactly once */
  const omsgs* s = &c->staged;
  const int64_t H = c->horizon, t_end = c->now, timeout = c->pr_cfg.timeout_ns;
  for (uint32_t p = 0; p < c->S; ++p) c->outbox[p].n = 0;
  /* 1. the window's requests (local probers): a route that refused one ends the probe at once */
  for (size_t i = 0; i < c->n_status; ++i) {
    const uint32_t sq = s->seq[i];
    if ((sq >> 30) != 1u) continue;
    const uint32_t code = c->status[i] & 0x0Fu, l = s->src[i] - c->lo;
    oprobe* p = &c->pr[l];
    if ((code == TGSIM_ST_DROPPED || code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) && p->state == PR_WAIT &&
        p->pos == (sq & PR_MASK) && c->pr_order[p->pos] == s->dst[i])
      p->refused = 1;
  }
  /* 2. the window's deliveries (local receivers): a request at its peer - a position of the prober
   *    beyond the last one answered here (the highest such position; its copies' earliest arrival) -
   *    and a reply at its prober */
  c->pr_list_n = 0;
  for (size_t i = 0; i < c->out.n; ++i) {
    const tgsim_record* r = &c->out.v[i];
    const uint32_t tag = r->seq >> 30;
    if (tag == 1u) {
      const uint32_t g = r->src, j = r->seq & PR_MASK;
      if (g >= c->N || j >= c->pr_n || c->pr_order[j] != r->dst || j + 1 <= c->pr_ans[g]) continue;
      if (!c->pr_cur[g]) c->pr_list[c->pr_list_n++] = g;
      /* the reply answers the highest position, at the first arrival of THAT position's request: a
       * request delayed past its timeout and arriving in its successor's window does not stamp the
       * successor's reply before the successor arrived */
      if (j + 1 > c->pr_cur[g]) { c->pr_cur[g] = j + 1; c->pr_rqa[g] = r->t; }
      else if (j + 1 == c->pr_cur[g] && r->t < c->pr_rqa[g]) c->pr_rqa[g] = r->t;
    } else if (tag == 3u && (r->seq & PR_MASK) == r->dst) {
      oprobe* p = &c->pr[r->dst - c->lo];
      if (p->state == PR_WAIT && p->replied && c->pr_order[p->pos] == r->src && r->t < p->t_reparr) p->t_reparr = r->t;
    }
  }
  /* 3. the peers answer: the reply at max(first arrival, horizon), and its notice to the prober */
  pbuf b;
  if (pr_alloc(&b, 2 * (size_t)c->nloc + c->pr_list_n + 1)) { pr_free(&b); return fail(c, TGSIM_ENOMEM, "oom"); }
  for (size_t i = 0; i < c->pr_list_n; ++i) {
    const uint32_t g = c->pr_list[i], j = c->pr_cur[g] - 1;
    const int64_t trep = c->pr_rqa[g] > H ? c->pr_rqa[g] : H;
    pr_stage(&b, c->pr_order[j], g, TGSIM_PROBE_REP | g, c->pr_cfg.reply_bytes, trep);
    c->pr_ans[g] = j + 1;
    c->pr_cur[g] = 0;
    c->pr_rqa[g] = PR_NONE;
    const uint32_t k = shard_of(c, g);
    if (k == c->cfg.shard_id) { pr_notice_apply(c, g, j, trep); continue; }
    tgsim_record r;
    memset(&r, 0, sizeof(r));
    r.t = trep; r.src = g; r.dst = j; r.seq = PRN_REPLY;
    if (recs_push(&c->outbox[k], &r)) { pr_free(&b); return fail(c, TGSIM_ENOMEM, "oom"); }
  }
  /* sharded: the notices to the probers' shards */
  if (c->S > 1) {
    memset(c->xsend, 0, (size_t)c->S * c->xcap * sizeof(tgsim_record));
    for (uint32_t p = 0; p < c->S; ++p) {
      orecs* o = &c->outbox[p];
      if (p == c->cfg.shard_id) continue;
      if (o->n + 1 > c->xcap) { pr_free(&b); return fail(c, TGSIM_ECAPACITY, "probe notices exceed the exchange capacity"); }
      c->xsend[(size_t)p * c->xcap].t = (int64_t)o->n;
      memcpy(&c->xsend[(size_t)p * c->xcap + 1], o->v, o->n * sizeof(tgsim_record));
      o->n = 0;
    }
    if (c->tr.alltoall(c->tr.user, c->xsend, c->xrecv, c->xcap * sizeof(tgsim_record), NULL) != 0) {
      pr_free(&b);
      return fail(c, TGSIM_EHIP, "transport all-to-all failed");
    }
    for (uint32_t p = 0; p < c->S; ++p) {
      if (p == c->cfg.shard_id) continue;
      const tgsim_record* blk = &c->xrecv[(size_t)p * c->xcap];
      const size_t n = (size_t)blk[0].t;
      if (n + 1 > c->xcap) { pr_free(&b); return fail(c, TGSIM_ECAPACITY, "corrupt exchange header"); }
      for (size_t i = 0; i < n; ++i) pr_notice_apply(c, blk[1 + i].src, blk[1 + i].dst, blk[1 + i].t);
    }
  }
  /* 4. per local prober: the probe's end, then the next request */
  int64_t min_dl = INT64_MAX;
  uint32_t active = 0;
  for (uint32_t l = 0; l < c->nloc; ++l) {
    oprobe* p = &c->pr[l];
    if (p->state != PR_WAIT) continue;
    const int64_t dl = p->t_req + timeout;
    /* a reply staged now before the deadline can still beat it */
    const int reply_pending = p->replied == 2 && p->t_rep < dl;
    if (p->replied == 2) p->replied = 1;
    uint8_t outc = TGSIM_PROBE_NONE;
    int64_t te = 0;
    if (p->refused) { outc = TGSIM_PROBE_REFUSED; te = p->t_req; }
    else if (p->t_reparr != PR_NONE && p->t_reparr < dl) { outc = TGSIM_PROBE_OK; te = p->t_reparr; }
    else if (dl < t_end && !reply_pending) { outc = TGSIM_PROBE_TIMEOUT; te = dl; }
    if (outc != TGSIM_PROBE_NONE) {
      c->pr_out[(size_t)l * c->pr_n + p->pos] = outc;
      pr_begin(c, l, pr_next(c, p, p->pos), te, H, &b);
    }
    if (p->state == PR_WAIT) {
      ++active;
      const int64_t d = p->t_req + timeout;
      if (d < min_dl) min_dl = d;
    }
  }
  int rc = pr_flush(c, &b);
  if (rc) return rc;
  /* 5. the next window: one window_ns while anything is staged or in flight (on any shard), else
   *    up to the earliest deadline */
  int64_t busy = c->staged.n || c->heap.n, tot = active, m = min_dl;
  if (c->S > 1) {
    int64_t mine[3] = {busy, (int64_t)active, min_dl};
    int64_t* all = (int64_t*)malloc((size_t)c->S * 3 * 8);
    if (!all) return fail(c, TGSIM_ENOMEM, "oom");
    if (c->tr.allgather(c->tr.user, mine, all, sizeof(mine), NULL) != 0) {
      free(all);
      return fail(c, TGSIM_EHIP, "transport all-gather failed");
    }
    busy = 0; tot = 0; m = INT64_MAX;
    for (uint32_t k = 0; k < c->S; ++k) {
      busy |= all[3 * k];
      tot += all[3 * k + 1];
      if (all[3 * k + 2] < m) m = all[3 * k + 2];
    }
    free(all);
  }
  int64_t ne = t_end + c->pr_cfg.window_ns;
  if (!busy && tot && m != INT64_MAX && m + 1 > ne) ne = m + 1;
  if (next_end) *next_end = ne;
  if (n_active) *n_active = (uint32_t)tot;
  return TGSIM_OK;
}
int tgo_probe_react(tgo_ctx* c, int64_t* next_end, uint32_t* n_active) {
  return shard_failed(c, probe_react_impl(c, next_end, n_active));
}

int tgo_probe_results(tgo_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap) {
  if (!c->pr) return fail(c, TGSIM_ESTATE, "no probes set up");
  const size_t n = (size_t)c->nloc * c->pr_n;
  if (outcome) {
    if (cap < n) return fail(c, TGSIM_ECAPACITY, "outcome capacity %zu < %zu", cap, n);
    memcpy(outcome, c->pr_out, n);
  }
  if (t_done)
    for (uint32_t l = 0; l < c->nloc; ++l) t_done[l] = c->pr[l].t_done;
  return TGSIM_OK;
}

/* ============================== topics (sync.Client Publish / Subscribe) ===================
 * [EXT sdk-go]; call sites plans/network/pingpong.go:219-245, plans/benchmarks/storm.go:232-255,
 * plans/splitbrain/main.go:91-103. A topic is a sync state: tgo_sync_signal assigns the positions
 * ((t, instance) order inside the batch), then each entry is stored at its position. */

static int topic_put(tgo_ctx* c, uint32_t topic, uint32_t pos, uint32_t inst, int64_t t, uint64_t off, uint32_t len) {
  if (topic >= c->n_topics) {
    size_t nn = topic + 1;
    otopic* q = (otopic*)realloc(c->topics, nn * sizeof(otopic));
    if (!q) return TGSIM_ENOMEM;
    memset(q + c->n_topics, 0, (nn - c->n_topics) * sizeof(otopic));
    c->topics = q; c->n_topics = nn;
  }
  otopic* tp = &c->topics[topic];
  size_t need = pos;  /* 1-based */
  if (need > tp->cap) {
    size_t nc = tp->cap ? tp->cap : 16;
    while (nc < need) nc *= 2;
    uint32_t* a = realloc(tp->inst, nc * 4); if (!a) return TGSIM_ENOMEM; tp->inst = a;
    int64_t* b = realloc(tp->t, nc * 8); if (!b) return TGSIM_ENOMEM; tp->t = b;
    uint64_t* o = realloc(tp->off, nc * 8); if (!o) return TGSIM_ENOMEM; tp->off = o;
    uint32_t* l = realloc(tp->len, nc * 4); if (!l) return TGSIM_ENOMEM; tp->len = l;
    tp->cap = nc;
  }
  tp->inst[pos - 1] = inst; tp->t[pos - 1] = t; tp->off[pos - 1] = off; tp->len[pos - 1] = len;
  if (pos > tp->n) tp->n = pos;
  return TGSIM_OK;
}

int tgo_sync_publish(tgo_ctx* c, const uint32_t* topics, const uint32_t* inst, const int64_t* t,
                     const uint64_t* off, const uint8_t* payload, size_t n, uint32_t* pos_out) {
  if (n && (!topics || !inst || !t || !off || (off[n] && !payload))) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (n && off[0] != 0) return fail(c, TGSIM_EINVAL, "payload offsets must start at 0");
  for (size_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFu) return fail(c, TGSIM_EINVAL, "bad payload offsets");
  if (n == 0) return TGSIM_OK;
  uint32_t* pos = (uint32_t*)malloc(n * 4);
  if (!pos) return TGSIM_ENOMEM;
  c->replicated_batch = 1;  /* topics are replicated: every shard publishes the same batch */
  int rc = tgo_sync_signal(c, topics, inst, t, n, pos);
  c->replicated_batch = 0;
  if (!rc && grow((void**)&c->tp_bytes, &c->tp_cap, c->tp_nbytes + off[n] + 1, 1)) rc = TGSIM_ENOMEM;
  if (!rc) {
    if (off[n]) memcpy(c->tp_bytes + c->tp_nbytes, payload, off[n]);
    for (size_t i = 0; i < n && !rc; ++i)
      rc = topic_put(c, topics[i], pos[i], inst[i], t[i], c->tp_nbytes + off[i], (uint32_t)(off[i + 1] - off[i]));
    c->tp_nbytes += off[n];
  }
  if (!rc && pos_out) memcpy(pos_out, pos, n * 4);
  free(pos);
  return rc;
}

int tgo_sync_subscribe(tgo_ctx* c, uint32_t topic, uint32_t from, int64_t until_t, size_t cap,
                       uint32_t* inst_out, int64_t* t_out, uint64_t* off_out, uint8_t* payload_out,
                       size_t payload_cap, size_t* n_out, size_t* payload_bytes) {
  if (!n_out || !payload_bytes || from == 0) return fail(c, TGSIM_EINVAL, "bad arguments");
  *n_out = 0; *payload_bytes = 0;
  if (topic >= c->cfg.max_states) return fail(c, TGSIM_EINVAL, "bad topic");
  if (topic >= c->n_topics) return TGSIM_OK;
  const otopic* tp = &c->topics[topic];
  size_t k = 0, bytes = 0;
  for (size_t p = from - 1; p < tp->n && k < cap && tp->t[p] <= until_t; ++p, ++k) bytes += tp->len[p];
  *n_out = k; *payload_bytes = bytes;
  if (bytes > payload_cap) return fail(c, TGSIM_ECAPACITY, "payload capacity %zu < %zu", payload_cap, bytes);
  if (k && (!inst_out || !t_out || !off_out || (bytes && !payload_out))) return fail(c, TGSIM_EINVAL, "bad arguments");
  size_t b = 0;
  for (size_t j = 0; j < k; ++j) {
    size_t p = from - 1 + j;
    inst_out[j] = tp->inst[p]; t_out[j] = tp->t[p]; off_out[j] = b;
    if (tp->len[p]) memcpy(payload_out + b, c->tp_bytes + tp->off[p], tp->len[p]);
    b += tp->len[p];
  }
  if (off_out) off_out[k] = b;
  return TGSIM_OK;
}

/* ============================== TCP mode ==================================== */
/* Segmentation and loss recovery over the per-packet path: plans/benchmarks/storm.go:127-180 writes
 * `size` bytes over a dialled connection, plans/network/pingpong.go:73-104 times round trips on one.
 * A segment's attempt fails when no copy enters the egress queue (the status of its packet) or when
 * every queued copy arrives corrupted; the next attempt leaves at max(t_a + rto * 2^a, the time the
 * failure is known) [EXT Linux tcp_retransmit_timer: exponential backoff from TCP_RTO_MIN]. */

int tgo_tcp_enable(tgo_ctx* c, const tgsim_tcp_config* cfg) {
  if (!cfg) return fail(c, TGSIM_EINVAL, "bad arguments");
  if (c->S != 1 && !c->has_tr) return fail(c, TGSIM_ESTATE, "a sharded context needs a transport for TCP mode");
  if (c->in_window || c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode already on or inside a window");
  if (c->staged.n) return fail(c, TGSIM_ESTATE, "messages already staged");
  if (c->fl_off) return fail(c, TGSIM_ESTATE, "a flood graph is installed: TCP mode and floods exclude each other");
  if (c->pr) return fail(c, TGSIM_ESTATE, "probes are set up: probes run in message mode");
  if (c->sm) return fail(c, TGSIM_ESTATE, "a storm reactor is set up: it runs in message mode");
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
  c->tcp = t;
  c->tcp_on = 1;
  return TGSIM_OK;
}

/* Segment ids on the wire (packet seq = id * 16 + attempt, the Philox counter of its netem draws) must
 * not depend on the shard count. A shard numbers its own segments 0, 1, ... (its state arrays); a
 * sharded context carries generated storm rounds only, each round n * F writes of one segment in
 * (instance, k) order, so the single run's id of local segment `sid` is the round's base plus the
 * shard's offset in it - an affine map per round, the identity on one shard. */
static uint32_t tcp_wire(const tgo_ctx* c, uint32_t sid) {
  if (c->S == 1) return sid;
  const uint32_t per = c->nloc * c->tcp_F, r = sid / per;
  return r * c->N * c->tcp_F + c->lo * c->tcp_F + sid % per;
}
static uint32_t tcp_local(const tgo_ctx* c, uint32_t wid) {
  if (c->S == 1) return wid;
  const uint32_t per = c->N * c->tcp_F, r = wid / per;
  return r * c->nloc * c->tcp_F + (wid % per - c->lo * c->tcp_F);
}

static int tcp_send_impl(tgo_ctx* c, const tgsim_msg_soa* m, size_t n);
int tgo_tcp_send(tgo_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (c->S != 1) return fail(c, TGSIM_ENOTSUP, "sharded TCP mode carries generated storm rounds (tcp_gen_storm_round) only");
  return tcp_send_impl(c, m, n);
}
static int tcp_send_impl(tgo_ctx* c, const tgsim_msg_soa* m, size_t n) {
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->tc_n) return fail(c, TGSIM_ESTATE, "a context with connections writes through tcp_write");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tcp_react after every window");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  size_t nseg = 0;
  for (size_t i = 0; i < n; ++i) {
    if (m->src[i] >= c->N || m->dst[i] >= c->N) return fail(c, TGSIM_EINVAL, "write %zu: bad instance id", i);
    if (m->t_send[i] < c->horizon) return fail(c, TGSIM_ECAUSALITY, "write %zu: t_send before the horizon", i);
    if (m->size[i] >= 0x80000000u) return fail(c, TGSIM_EINVAL, "write %zu: size too large", i);
    nseg += m->size[i] ? (m->size[i] + c->tcp.mss - 1) / c->tcp.mss : 1;
  }
  if (c->tw_n + n > c->tcp.max_writes || c->tsg_n + nseg > c->tcp.max_segments)
    return fail(c, TGSIM_ECAPACITY, "TCP write / segment capacity");
  if (grow((void**)&c->tw, &c->tw_cap, c->tw_n + n + 1, sizeof(otcpw)) ||
      grow((void**)&c->tsg, &c->tsg_cap, c->tsg_n + nseg + 1, sizeof(otcps)))
    return fail(c, TGSIM_ENOMEM, "oom");
  uint32_t* src = malloc((nseg + 1) * 4); uint32_t* dst = malloc((nseg + 1) * 4);
  uint32_t* seq = malloc((nseg + 1) * 4); uint32_t* sz = malloc((nseg + 1) * 4);
  int64_t* ts = malloc((nseg + 1) * 8);
  if (!src || !dst || !seq || !sz || !ts) { free(src); free(dst); free(seq); free(sz); free(ts); return TGSIM_ENOMEM; }
  size_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t size = m->size[i], ns = size ? (size + c->tcp.mss - 1) / c->tcp.mss : 1;
    otcpw w = {m->src[i], m->dst[i], ns, TGSIM_TCP_PENDING, INT64_MIN, TCP_NOSEG};
    const uint32_t wi = (uint32_t)c->tw_n++;
    c->tw[wi] = w;
    for (uint32_t j = 0; j < ns; ++j, ++k) {
      const uint32_t pay = size ? (j + 1 < ns ? c->tcp.mss : size - j * c->tcp.mss) : 0;
      const uint32_t sid = (uint32_t)c->tsg_n++;
      otcps g = {wi, pay + c->tcp.header_bytes, 0, 0, 0, 0, m->t_send[i], INT64_MAX, INT64_MIN, 0, 0, TCP_NOSEG, 0, 0};
      c->tsg[sid] = g;
      src[k] = w.src; dst[k] = w.dst; seq[k] = tcp_wire(c, sid) << 4; sz[k] = g.wire; ts[k] = m->t_send[i];
    }
  }
  tgsim_msg_soa p = {src, dst, seq, sz, ts};
  int rc = enqueue_impl(c, &p, k);
  free(src); free(dst); free(seq); free(sz); free(ts);
  if (rc) return rc;
  c->tstats.writes += n;
  c->tstats.segments += k;
  c->tstats.packets += k;
  return TGSIM_OK;
}

/* ---- connections: congestion window and ACK clocking (acks = 1) ------------
 * Reno [EXT Linux tcp_cong.c, RFC 5681]: IW10, slow start below ssthresh, one segment per cwnd ACKs
 * above, ssthresh = max(cwnd / 2, 2) and cwnd = 1 at a window's first retransmission timeout. */

typedef struct { uint32_t* src; uint32_t* dst; uint32_t* seq; uint32_t* size; int64_t* t; size_t n, cap; } ostage;
static int ostage_push(ostage* b, uint32_t src, uint32_t dst, uint32_t seq, uint32_t size, int64_t t) {
  if (b->n == b->cap) {
    size_t nc = b->cap ? 2 * b->cap : 256;
    uint32_t* a = realloc(b->src, nc * 4); if (!a) return TGSIM_ENOMEM; b->src = a;
    a = realloc(b->dst, nc * 4); if (!a) return TGSIM_ENOMEM; b->dst = a;
    a = realloc(b->seq, nc * 4); if (!a) return TGSIM_ENOMEM; b->seq = a;
    a = realloc(b->size, nc * 4); if (!a) return TGSIM_ENOMEM; b->size = a;
    int64_t* q = realloc(b->t, nc * 8); if (!q) return TGSIM_ENOMEM; b->t = q;
    b->cap = nc;
  }
  b->src[b->n] = src; b->dst[b->n] = dst; b->seq[b->n] = seq; b->size[b->n] = size; b->t[b->n] = t; ++b->n;
  return TGSIM_OK;
}
static int ostage_flush(tgo_ctx* c, ostage* b) {
  int rc = TGSIM_OK;
  if (b->n) {
    tgsim_msg_soa m = {b->src, b->dst, b->seq, b->size, b->t};
    rc = enqueue_impl(c, &m, b->n);
    c->tstats.packets += b->n;
  }
  free(b->src); free(b->dst); free(b->seq); free(b->size); free(b->t);
  return rc;
}

static void tcp_finish(tgo_ctx* c, uint32_t wi, uint32_t state, int64_t t, size_t* done);

/* Connection k sends while its flight is below cwnd, each segment at max(written, t0): first the
 * segments a timeout marked lost (in order, the next attempt; settled ones are passed over, and one
 * of a failed write or out of attempts gives up), then new ones. */
static int conn_release(tgo_ctx* c, uint32_t k, int64_t t0, ostage* b, size_t* done) {
  otcpc* q = &c->tc[k];
  while (q->flight < q->cwnd && q->head != TCP_NOSEG) {
    const uint32_t sid = q->head;
    otcps* g = &c->tsg[sid];
    q->head = g->next;
    if (g->acked || g->gave_up) continue;
    const int64_t t = g->t_att > t0 ? g->t_att : t0;
    uint32_t seq = sid << 4;
    if (g->lost) {
      const uint32_t st = c->tw[g->w].state;
      g->lost = 0;
      if (st == TGSIM_TCP_TIMEOUT || st == TGSIM_TCP_REFUSED || g->attempt + 1 >= c->tcp.max_attempts) {
        g->gave_up = 1;
        tcp_finish(c, g->w, TGSIM_TCP_TIMEOUT, t, done);
        continue;
      }
      g->attempt++;
      seq |= g->attempt;
      c->tstats.retransmissions++;
    } else {
      g->unsent = 0;
      q->queued--;
    }
    g->t_att = t;
    q->flight++;
    if (ostage_push(b, q->src, q->dst, seq, g->wire, t)) return TGSIM_ENOMEM;
  }
  return TGSIM_OK;
}

int tgo_tcp_connect(tgo_ctx* c, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* conn_out) {
  if (!c->tcp_on || !c->tcp.acks) return fail(c, TGSIM_ESTATE, "connections need TCP mode with acks = 1");
  if (c->S != 1) return fail(c, TGSIM_ENOTSUP, "connections (their ACK clock) need a single-shard context");
  if (c->sm) return fail(c, TGSIM_ESTATE, "a storm reactor owns the connections");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->tw_n && !c->tc_n) return fail(c, TGSIM_ESTATE, "tcp_send writes exist: a context uses one or the other");
  if (n && (!src || !dst)) return fail(c, TGSIM_EINVAL, "bad arguments");
  for (size_t i = 0; i < n; ++i)
    if (src[i] >= c->N || dst[i] >= c->N) return fail(c, TGSIM_EINVAL, "connection %zu: bad instance id", i);
  if (c->tc_n + n > c->tcp.max_writes) return fail(c, TGSIM_ECAPACITY, "connection capacity");
  if (grow((void**)&c->tc, &c->tc_cap, c->tc_n + n + 1, sizeof(otcpc))) return fail(c, TGSIM_ENOMEM, "oom");
  for (size_t i = 0; i < n; ++i) {
    otcpc q = {src[i], dst[i], TCP_IW, 0x7FFFFFFFu, 0, 0, 0, TCP_NOSEG, TCP_NOSEG, 0, 0, 0, INT64_MAX, TCP_NOSEG, 0,
               INT64_MIN, TCP_NOSEG};
    if (conn_out) conn_out[i] = (uint32_t)c->tc_n;
    c->tc[c->tc_n++] = q;
  }
  return TGSIM_OK;
}

int tgo_tcp_write(tgo_ctx* c, const uint32_t* conn, const uint32_t* size, const int64_t* t, size_t n) {
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->sm) return fail(c, TGSIM_ESTATE, "a storm reactor owns the connections");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tcp_react after every window");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (n && (!conn || !size || !t)) return fail(c, TGSIM_EINVAL, "bad arguments");
  size_t nseg = 0;
  for (size_t i = 0; i < n; ++i) {
    if (conn[i] >= c->tc_n) return fail(c, TGSIM_EINVAL, "write %zu: no connection %u", i, conn[i]);
    if (conn[i] >= c->sm_conn_lo && conn[i] < c->sm_conn_hi)  /* its queue ends where the reactor left it */
      return fail(c, TGSIM_ESTATE, "write %zu: connection %u was a storm reactor's", i, conn[i]);
    if (t[i] < c->horizon) return fail(c, TGSIM_ECAUSALITY, "write %zu: t_send before the horizon", i);
    if (size[i] >= 0x80000000u) return fail(c, TGSIM_EINVAL, "write %zu: size too large", i);
    nseg += size[i] ? (size[i] + c->tcp.mss - 1) / c->tcp.mss : 1;
  }
  if (c->tw_n + n > c->tcp.max_writes || c->tsg_n + nseg > c->tcp.max_segments)
    return fail(c, TGSIM_ECAPACITY, "TCP write / segment capacity");
  if (grow((void**)&c->tw, &c->tw_cap, c->tw_n + n + 1, sizeof(otcpw)) ||
      grow((void**)&c->tsg, &c->tsg_cap, c->tsg_n + nseg + 1, sizeof(otcps)))
    return fail(c, TGSIM_ENOMEM, "oom");
  for (size_t i = 0; i < n; ++i) {
    otcpc* q = &c->tc[conn[i]];
    const uint32_t sz = size[i], ns = sz ? (sz + c->tcp.mss - 1) / c->tcp.mss : 1;
    const uint32_t wi = (uint32_t)c->tw_n++;
    otcpw w = {q->src, q->dst, ns, TGSIM_TCP_PENDING, INT64_MIN, conn[i]};
    c->tw[wi] = w;
    for (uint32_t j = 0; j < ns; ++j) {
      const uint32_t pay = sz ? (j + 1 < ns ? c->tcp.mss : sz - j * c->tcp.mss) : 0;
      const uint32_t sid = (uint32_t)c->tsg_n++;
      otcps g = {wi, pay + c->tcp.header_bytes, 0, 0, 0, 0, t[i], INT64_MAX, INT64_MIN, 0, 0, TCP_NOSEG, 1, 0};
      c->tsg[sid] = g;
      if (q->tail != TCP_NOSEG) c->tsg[q->tail].next = sid;
      if (q->head == TCP_NOSEG) q->head = sid;
      if (q->una == TCP_NOSEG) q->una = sid;
      q->tail = sid;
      q->queued++;
    }
  }
  c->tstats.writes += n;
  c->tstats.segments += nseg;
  /* what the windows have room for leaves now, at its write time */
  ostage b = {0};
  int rc = TGSIM_OK;
  size_t done = 0;
  for (uint32_t k = 0; k < c->tc_n && !rc; ++k)
    if (!c->tc[k].broken) rc = conn_release(c, k, INT64_MIN, &b, &done);
  const int rc2 = ostage_flush(c, &b);
  return rc ? fail(c, rc, "oom") : rc2;
}

int tgo_tcp_conns(tgo_ctx* c, uint32_t first, size_t n, uint64_t* acked, uint32_t* cwnd, uint32_t* flight,
                  uint32_t* queued) {
  if ((uint64_t)first + n > c->tc_n) return fail(c, TGSIM_EINVAL, "connections [%u, +%zu) out of range", first, n);
  for (size_t i = 0; i < n; ++i) {
    const otcpc* q = &c->tc[first + i];
    if (acked) acked[i] = q->acked;
    if (cwnd) cwnd[i] = q->cwnd;
    if (flight) flight[i] = q->flight;
    if (queued) queued[i] = q->queued;
  }
  return TGSIM_OK;
}

/* A write ends once: delivered (its last segment arrived) or failed. A failed write keeps its
 * earliest failure, refusal before timeout at equal times (key t * 2 + (timeout ? 1 : 0)), so the
 * outcome does not depend on the order the failures are found in. */
static void tcp_finish(tgo_ctx* c, uint32_t wi, uint32_t state, int64_t t, size_t* done) {
  otcpw* w = &c->tw[wi];
  if (w->state == TGSIM_TCP_DELIVERED) return;
  if (w->state != TGSIM_TCP_PENDING) {  /* already failed: keep the earlier failure */
    const int64_t k_old = w->t * 2 + (w->state == TGSIM_TCP_TIMEOUT), k_new = t * 2 + (state == TGSIM_TCP_TIMEOUT);
    if (state != TGSIM_TCP_DELIVERED && k_new < k_old) { w->state = state; w->t = t; }
    return;
  }
  w->state = state;
  w->t = t;
  ++*done;
  if (state == TGSIM_TCP_DELIVERED) c->tstats.delivered++; else c->tstats.failed++;
}

/* attempt g->attempt failed; the failure is known at t_known. A segment of a write that has
 * already failed is still scheduled (and dropped at release), so scheduling is order-independent. */
static int tcp_schedule(tgo_ctx* c, uint32_t sid, int64_t t_known, size_t* done) {
  otcps* g = &c->tsg[sid];
  int64_t t = g->t_att + (c->tcp.rto_ns << g->attempt);
  if (t < t_known) t = t_known;
  if (g->attempt + 1 >= c->tcp.max_attempts) { tcp_finish(c, g->w, TGSIM_TCP_TIMEOUT, t, done); return TGSIM_OK; }
  g->attempt++;
  g->t_att = t;
  g->t_last = INT64_MIN;
  if (grow((void**)&c->tpend, &c->tpend_cap, c->tpend_n + 1, 4)) return TGSIM_ENOMEM;
  c->tpend[c->tpend_n++] = sid;
  c->tstats.retransmissions++;
  return TGSIM_OK;
}

/* copies of a packet that entered its egress queue, from its status (tgsim.h status flags) */
static uint32_t tcp_copies(uint8_t st) {
  const uint8_t code = st & 0x0Fu;
  if (code == TGSIM_ST_LOCAL) return 1;
  if (code != TGSIM_ST_QUEUED) return 0;
  uint32_t q = (st & TGSIM_ST_FLAG_OVERLIMIT) ? 0u : 1u;
  if ((st & TGSIM_ST_FLAG_DUP) && !(st & TGSIM_ST_FLAG_CLONE_LOST)) ++q;
  return q;
}

static int tcp_react_acks(tgo_ctx* c, size_t* done);

/* Sharded TCP: a write's segments live on its writer's shard
 * (its packets were staged and shaped there: egress), while a data copy is delivered on its receiver's
 * shard. After each window every shard forwards the data copies it delivered for another shard's
 * writers to that shard as their delivery records (one all-to-all of the exchange blocks), and
 * collects those delivered elsewhere for its own writers into c->tcp_rx. ACKs (acks = 1) leave from
 * the receiver's shard and are delivered on the writer's: they need no forwarding. */
static int tcp_forward(tgo_ctx* c) {
  c->tcp_rx.n = 0;
  if (c->S == 1) return TGSIM_OK;
  if (!c->has_tr) return fail(c, TGSIM_ESTATE, "the transport was aborted (a shard failed)");
  const uint32_t me = c->cfg.shard_id;
  for (uint32_t p = 0; p < c->S; ++p) c->outbox[p].n = 0;
  for (size_t i = 0; i < c->out.n; ++i) {
    const tgsim_record* r = &c->out.v[i];
    if (c->tcp.acks && (r->seq & TGSIM_TCP_ACK_BIT)) continue;
    const uint32_t p = shard_of(c, r->src);
    if (p != me && recs_push(&c->outbox[p], r)) return fail(c, TGSIM_ENOMEM, "oom");
  }
  memset(c->xsend, 0, (size_t)c->S * c->xcap * sizeof(tgsim_record));
  for (uint32_t p = 0; p < c->S; ++p) {
    orecs* o = &c->outbox[p];
    if (p == me) continue;
    if (o->n + 1 > c->xcap) return fail(c, TGSIM_ECAPACITY, "TCP arrivals exceed the exchange capacity (%zu to peer %u)", o->n, p);
    c->xsend[(size_t)p * c->xcap].t = (int64_t)o->n;
    memcpy(&c->xsend[(size_t)p * c->xcap + 1], o->v, o->n * sizeof(tgsim_record));
    o->n = 0;
  }
  if (c->tr.alltoall(c->tr.user, c->xsend, c->xrecv, c->xcap * sizeof(tgsim_record), NULL) != 0)
    return fail(c, TGSIM_EHIP, "transport all-to-all failed");
  for (uint32_t p = 0; p < c->S; ++p) {
    if (p == me) continue;
    const tgsim_record* blk = &c->xrecv[(size_t)p * c->xcap];
    const size_t n = (size_t)blk[0].t;
    if (n + 1 > c->xcap) return fail(c, TGSIM_ECAPACITY, "corrupt exchange header");
    for (size_t i = 0; i < n; ++i)
      if (recs_push(&c->tcp_rx, &blk[1 + i])) return fail(c, TGSIM_ENOMEM, "oom");
  }
  return TGSIM_OK;
}

/* a data copy this shard settles: delivered here to a local writer's segment, or forwarded (tcp_rx) */
static int tcp_mine(const tgo_ctx* c, const tgsim_record* r) {
  return c->S == 1 || shard_of(c, r->src) == c->cfg.shard_id;
}

int tgo_tcp_react(tgo_ctx* c, size_t* n_done) {
  size_t done = 0;
  if (n_done) *n_done = 0;
  if (!c->tcp_on) return fail(c, TGSIM_ESTATE, "TCP mode is off");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (!c->tcp_need_react) return TGSIM_OK;
  {
    const int rc = tcp_forward(c);
    if (rc) return rc;
  }
  if (c->tcp.acks) {
    int rc = tcp_react_acks(c, &done);
    if (rc) return rc;
    c->tcp_need_react = 0;
    if (n_done) *n_done = done;
    return TGSIM_OK;
  }
  /* 1. the window's packets (staged arrays are intact until the next staging) */
  const omsgs* s = &c->staged;
  for (size_t i = 0; i < c->n_status; ++i) {
    const uint32_t sid = tcp_local(c, s->seq[i] >> 4);
    otcps* g = &c->tsg[sid];
    const uint32_t q = tcp_copies(c->status[i]);
    if (q) { g->outstanding += q; continue; }
    const uint8_t code = c->status[i] & 0x0Fu;
    if (code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) tcp_finish(c, g->w, TGSIM_TCP_REFUSED, g->t_att, &done);
    else if (tcp_schedule(c, sid, g->t_att, &done)) return fail(c, TGSIM_ENOMEM, "oom");
  }
  /* 2. the window's deliveries: first intact arrival, copies accounted - the copies of this shard's
   *    writers delivered here, then those forwarded from the receivers' shards */
  uint32_t* touched = (uint32_t*)malloc((c->out.n + c->tcp_rx.n + 1) * 4);
  if (!touched) return fail(c, TGSIM_ENOMEM, "oom");
  size_t nt = 0;
  for (size_t i = 0; i < c->out.n + c->tcp_rx.n; ++i) {
    const tgsim_record* r = i < c->out.n ? &c->out.v[i] : &c->tcp_rx.v[i - c->out.n];
    if (i < c->out.n && !tcp_mine(c, r)) continue;
    const uint32_t sid = tcp_local(c, r->seq >> 4);
    otcps* g = &c->tsg[sid];
    if (!(r->meta & TGSIM_F_CORRUPT) && r->t < g->arrival) g->arrival = r->t;
    if (r->t > g->t_last) g->t_last = r->t;
    g->outstanding--;
    if (!g->touched) { g->touched = 1; touched[nt++] = sid; }
  }
  int rc = 0;
  for (size_t k = 0; k < nt && !rc; ++k) {
    otcps* g = &c->tsg[touched[k]];
    g->touched = 0;
    if (g->arrived) continue;
    if (g->arrival != INT64_MAX) {
      g->arrived = 1;
      otcpw* w = &c->tw[g->w];
      if (g->arrival > w->t && w->state == TGSIM_TCP_PENDING) w->t = g->arrival;
      if (--w->remaining == 0) tcp_finish(c, g->w, TGSIM_TCP_DELIVERED, w->t, &done);
    } else if (g->outstanding == 0) {
      rc = tcp_schedule(c, touched[k], g->t_last, &done);
    }
  }
  free(touched);
  if (rc) return fail(c, TGSIM_ENOMEM, "oom");
  c->tcp_need_react = 0;
  c->tstats.pending_retx = c->tpend_n;
  if (n_done) *n_done = done;
  return TGSIM_OK;
}

/* acks = 1: the window's packets only refuse (a timer handles every other failure); its deliveries
 * are data (first intact arrival, and an ACK back for every intact copy at max(arrival, horizon):
 * when it arrived, a late send) or ACKs (an intact one acknowledges its segment). */
static int tcp_react_acks(tgo_ctx* c, size_t* done) {
  const omsgs* s = &c->staged;
  for (size_t i = 0; i < c->n_status; ++i) {
    if (s->seq[i] & TGSIM_TCP_ACK_BIT) continue;
    const uint8_t code = c->status[i] & 0x0Fu;
    otcps* g = &c->tsg[tcp_local(c, s->seq[i] >> 4)];
    if (code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) {
      tcp_finish(c, g->w, TGSIM_TCP_REFUSED, g->t_att, done);
      if (c->tw[g->w].conn != TCP_NOSEG) c->tc[c->tw[g->w].conn].broken = 1;  /* the connection is reset */
    }
  }
  uint32_t* touched = (uint32_t*)malloc((c->out.n + c->tcp_rx.n + 1) * 4);
  if (!touched || grow((void**)&c->tack, &c->tack_cap, c->tack_n + c->out.n + 1, sizeof(otack))) {
    free(touched);
    return fail(c, TGSIM_ENOMEM, "oom");
  }
  size_t nt = 0;
  /* the deliveries here (ACKs of this shard's writers' segments; data: answered from here, settled
   * here for a local writer), then the data copies of this shard's writers delivered elsewhere */
  for (size_t i = 0; i < c->out.n + c->tcp_rx.n; ++i) {
    const int rx = i >= c->out.n;
    const tgsim_record* r = rx ? &c->tcp_rx.v[i - c->out.n] : &c->out.v[i];
    const int intact = !(r->meta & TGSIM_F_CORRUPT);
    /* this shard's segment: an ACK's always, a data copy's once its writer is known to be local */
    const uint32_t sid = tcp_local(c, (r->seq & ~TGSIM_TCP_ACK_BIT) >> 4);
    if (r->seq & TGSIM_TCP_ACK_BIT) {
      otcps* g = &c->tsg[sid];  /* an ACK arrives at the writer: always this shard's */
      /* the first intact ACK of a segment that has not given up settles it (its flight slot); what
       * the window's ACKs release leaves at the latest intact one's arrival (duplicates included) */
      if (intact && !g->gave_up) {
        const uint32_t k = c->tw[g->w].conn;
        if (k != TCP_NOSEG && r->t > c->tc[k].tack) c->tc[k].tack = r->t;
        if (!g->acked) {
          g->acked = 1;
          if (k != TCP_NOSEG) {
            c->tc[k].acks++;
            if (!g->lost) c->tc[k].facks++;  /* a segment marked lost holds no flight slot */
          }
        }
      }
      continue;
    }
    if (!intact) continue;
    if (!rx) {  /* the receiver answers every intact data copy it got */
      otack a = {r->dst, r->src, TGSIM_TCP_ACK_BIT | r->seq, r->t > c->horizon ? r->t : c->horizon};
      c->tack[c->tack_n++] = a;
      if (!tcp_mine(c, r)) continue;  /* its writer's shard settles the segment */
    }
    otcps* g = &c->tsg[sid];
    if (r->t < g->arrival) g->arrival = r->t;
    if (!g->touched) { g->touched = 1; touched[nt++] = sid; }
  }
  for (size_t k = 0; k < nt; ++k) {
    otcps* g = &c->tsg[touched[k]];
    g->touched = 0;
    if (g->arrived) continue;
    g->arrived = 1;
    otcpw* w = &c->tw[g->w];
    if (w->state != TGSIM_TCP_PENDING) continue;  /* failed first: stays failed */
    if (g->arrival > w->t) w->t = g->arrival;
    if (--w->remaining == 0) tcp_finish(c, g->w, TGSIM_TCP_DELIVERED, w->t, done);
  }
  free(touched);
  /* connections: the window's first ACKs free flight and open cwnd, and what now fits leaves at
   * max(the latest of them's arrival, horizon) (the window's end without ACKs); fast retransmit
   * [EXT RFC 5681 3.2]: once three segments after the oldest outstanding one have been ACKed (three
   * duplicate ACKs in a cumulative-ACK stack) and it has not, it is resent then (its next attempt,
   * once per segment, keeping its flight slot), ssthresh = max(flight / 2, 2), cwnd = ssthresh; a
   * reset connection fails its queued writes at the window's end */
  ostage b = {0};
  int rc = TGSIM_OK;
  for (uint32_t k = 0; k < c->tc_n && !rc; ++k) {
    otcpc* q = &c->tc[k];
    int64_t t0 = c->t_end;
    q->flight -= q->facks;
    q->facks = 0;
    q->acked += q->acks;
    for (uint32_t a = 0; a < q->acks; ++a) {
      if (q->cwnd < q->ssthresh) ++q->cwnd;
      else if (++q->cnt >= q->cwnd) { ++q->cwnd; q->cnt = 0; }
      if (q->cwnd > TCP_CWND_CLAMP) q->cwnd = TCP_CWND_CLAMP;
    }
    if (q->acks) {
      t0 = q->tack > c->horizon ? q->tack : c->horizon;
      q->tack = INT64_MIN;
      uint32_t u = q->una;
      while (u != q->head && (c->tsg[u].acked || c->tsg[u].gave_up)) u = c->tsg[u].next;
      q->una = u;
      if (u != q->head && !q->broken && !c->tsg[u].lost && q->fr != u && c->tsg[u].attempt + 1 < c->tcp.max_attempts) {
        otcps* g = &c->tsg[u];
        const uint32_t st = c->tw[g->w].state;
        uint32_t dup = 0;
        for (uint32_t x = g->next; x != q->head && dup < 3; x = c->tsg[x].next) dup += c->tsg[x].acked;
        if (dup >= 3 && st != TGSIM_TCP_TIMEOUT && st != TGSIM_TCP_REFUSED) {
          q->fr = u;
          q->ssthresh = q->flight / 2 > 2 ? q->flight / 2 : 2;
          q->cwnd = q->ssthresh;
          q->cnt = 0;
          g->attempt++;
          g->t_att = t0;
          c->tstats.retransmissions++;
          if (ostage_push(&b, q->src, q->dst, (u << 4) | g->attempt, g->wire, t0)) rc = TGSIM_ENOMEM;
        }
      }
    }
    q->acks = 0;
    if (q->broken) {
      while (q->head != TCP_NOSEG) {
        otcps* g = &c->tsg[q->head];
        tcp_finish(c, g->w, TGSIM_TCP_REFUSED, g->t_att > c->t_end ? g->t_att : c->t_end, done);
        g->unsent = 0;
        g->gave_up = 1;
        q->head = g->next;
      }
      q->queued = 0;
      continue;
    }
    if (!rc) rc = conn_release(c, k, t0, &b, done);
  }
  const int rc2 = ostage_flush(c, &b);
  return rc ? fail(c, rc, "oom") : rc2;
}

typedef struct { int64_t t; uint32_t sid; } otx;
static int cmp_otx(const void* a, const void* b) {
  const otx* x = (const otx*)a; const otx* y = (const otx*)b;
  if (x->t != y->t) return x->t < y->t ? -1 : 1;
  return x->sid < y->sid ? -1 : (x->sid > y->sid);
}

/* Stage the retransmissions whose time falls before t_end, in (time, segment) order; those of a
 * failed write are dropped. */
static int tcp_release_acks(tgo_ctx* c, int64_t t_end);
static int tcp_release(tgo_ctx* c, int64_t t_end) {
  if (c->tcp.acks) return tcp_release_acks(c, t_end);
  if (!c->tpend_n) return TGSIM_OK;
  otx* due = (otx*)malloc(c->tpend_n * sizeof(otx));
  if (!due) return fail(c, TGSIM_ENOMEM, "oom");
  size_t nd = 0, keep = 0;
  for (size_t i = 0; i < c->tpend_n; ++i) {
    const uint32_t sid = c->tpend[i];
    const otcps* g = &c->tsg[sid];
    if (c->tw[g->w].state != TGSIM_TCP_PENDING) continue;
    if (g->t_att < t_end) { due[nd].t = g->t_att; due[nd].sid = sid; ++nd; }
    else c->tpend[keep++] = sid;
  }
  c->tpend_n = keep;
  c->tstats.pending_retx = keep;
  int rc = TGSIM_OK;
  if (nd) {
    qsort(due, nd, sizeof(otx), cmp_otx);
    uint32_t* src = malloc(nd * 4); uint32_t* dst = malloc(nd * 4); uint32_t* seq = malloc(nd * 4);
    uint32_t* sz = malloc(nd * 4); int64_t* ts = malloc(nd * 8);
    if (!src || !dst || !seq || !sz || !ts) rc = TGSIM_ENOMEM;
    for (size_t i = 0; i < nd && !rc; ++i) {
      const otcps* g = &c->tsg[due[i].sid];
      src[i] = c->tw[g->w].src; dst[i] = c->tw[g->w].dst; seq[i] = (tcp_wire(c, due[i].sid) << 4) | g->attempt;
      sz[i] = g->wire; ts[i] = g->t_att;
    }
    if (!rc) {
      tgsim_msg_soa p = {src, dst, seq, sz, ts};
      rc = enqueue_impl(c, &p, nd);
      c->tstats.packets += nd;
    }
    free(src); free(dst); free(seq); free(sz); free(ts);
  }
  free(due);
  return rc;
}

/* acks = 1, at the start of window [now, t_end): the ACKs of the last reaction, then every timer of
 * an attempt sent in an earlier window that falls before t_end and whose segment no ACK has reached:
 * the next attempt at max(timer, now), or the segment gives up (TIMEOUT at the timer for a write
 * that has not completed). Packets are staged in (time, segment) order, the ACKs first. */
static int tcp_release_acks(tgo_ctx* c, int64_t t_end) {
  const int64_t H = c->now;
  int rc = TGSIM_OK;
  if (c->tack_n) {
    const size_t na = c->tack_n;
    uint32_t* src = malloc(na * 4); uint32_t* dst = malloc(na * 4); uint32_t* seq = malloc(na * 4);
    uint32_t* sz = malloc(na * 4); int64_t* ts = malloc(na * 8);
    if (!src || !dst || !seq || !sz || !ts) rc = TGSIM_ENOMEM;
    for (size_t i = 0; i < na && !rc; ++i) {
      src[i] = c->tack[i].src; dst[i] = c->tack[i].dst; seq[i] = c->tack[i].seq; sz[i] = c->tcp.header_bytes;
      ts[i] = c->tack[i].t;
    }
    if (!rc) {
      tgsim_msg_soa p = {src, dst, seq, sz, ts};
      rc = enqueue_impl(c, &p, na);
    }
    free(src); free(dst); free(seq); free(sz); free(ts);
    c->tack_n = 0;
    if (rc) return rc;
  }
  otx* due = (otx*)malloc((c->tsg_n + 1) * sizeof(otx));
  if (!due) return fail(c, TGSIM_ENOMEM, "oom");
  size_t nd = 0, done = 0;
  for (size_t sid = 0; sid < c->tsg_n; ++sid) {
    otcps* g = &c->tsg[sid];
    /* settled, marked lost (no timer until resent), or its attempt not yet sent */
    if (g->acked || g->gave_up || g->unsent || g->lost || g->t_att >= H) continue;
    const uint32_t st = c->tw[g->w].state;
    if (st == TGSIM_TCP_TIMEOUT || st == TGSIM_TCP_REFUSED) continue;
    const int64_t T = g->t_att + (c->tcp.rto_ns << g->attempt);
    if (T >= t_end) continue;
    const uint32_t k = c->tw[g->w].conn;
    if (g->attempt + 1 >= c->tcp.max_attempts) {
      g->gave_up = 1;
      if (k != TCP_NOSEG) c->tc[k].flight--;
      tcp_finish(c, g->w, TGSIM_TCP_TIMEOUT, T, &done);
      continue;
    }
    if (k != TCP_NOSEG) {  /* a connection's timeout: its loss episode below resends under cwnd */
      if (T < c->tc[k].tloss) c->tc[k].tloss = T;
      continue;
    }
    g->attempt++;
    g->t_att = T > H ? T : H;
    c->tstats.retransmissions++;
    due[nd].t = g->t_att; due[nd].sid = (uint32_t)sid; ++nd;
  }
  if (nd) {
    qsort(due, nd, sizeof(otx), cmp_otx);
    uint32_t* src = malloc(nd * 4); uint32_t* dst = malloc(nd * 4); uint32_t* seq = malloc(nd * 4);
    uint32_t* sz = malloc(nd * 4); int64_t* ts = malloc(nd * 8);
    if (!src || !dst || !seq || !sz || !ts) rc = TGSIM_ENOMEM;
    for (size_t i = 0; i < nd && !rc; ++i) {
      const otcps* g = &c->tsg[due[i].sid];
      src[i] = c->tw[g->w].src; dst[i] = c->tw[g->w].dst; seq[i] = (tcp_wire(c, due[i].sid) << 4) | g->attempt;
      sz[i] = g->wire; ts[i] = g->t_att;
    }
    if (!rc) {
      tgsim_msg_soa p = {src, dst, seq, sz, ts};
      rc = enqueue_impl(c, &p, nd);
      c->tstats.packets += nd;
    }
    free(src); free(dst); free(seq); free(sz); free(ts);
  }
  free(due);
  /* loss episodes [EXT Linux tcp_enter_loss, RFC 5681 3.1 / RFC 6298 5.4]: a connection whose timer
   * expired in this window, at its earliest expiry T: ssthresh = max(cwnd / 2, 2) unless cwnd is
   * already 1 (the same episode), cwnd = 1; every outstanding segment is marked lost and the send
   * queue restarts at the oldest, which leaves at max(T, H); the rest follow as ACKs open cwnd. */
  ostage b = {0};
  for (uint32_t k = 0; k < c->tc_n && !rc; ++k) {
    otcpc* q = &c->tc[k];
    if (q->tloss == INT64_MAX) continue;
    const int64_t tl = q->tloss;
    q->tloss = INT64_MAX;
    if (q->cwnd > 1) q->ssthresh = q->cwnd / 2 > 2 ? q->cwnd / 2 : 2;
    q->cwnd = 1;
    q->cnt = 0;
    uint32_t u = q->una;
    while (u != q->head && (c->tsg[u].acked || c->tsg[u].gave_up)) u = c->tsg[u].next;
    q->una = u;
    for (uint32_t x = u; x != q->head; x = c->tsg[x].next)
      if (!c->tsg[x].acked && !c->tsg[x].gave_up) c->tsg[x].lost = 1;
    q->head = u;
    q->flight = 0;
    if (!q->broken) rc = conn_release(c, k, tl > H ? tl : H, &b, &done);
  }
  const int rc2 = ostage_flush(c, &b);
  c->tstats.pending_retx = 0;
  return rc ? rc : rc2;
}

int tgo_tcp_writes(tgo_ctx* c, uint8_t* state, int64_t* t, size_t cap, size_t* n) {
  if (!n) return TGSIM_EINVAL;
  *n = c->tw_n;
  if (c->tw_n > cap) return fail(c, TGSIM_ECAPACITY, "write capacity");
  for (size_t i = 0; i < c->tw_n; ++i) {
    if (state) state[i] = (uint8_t)c->tw[i].state;
    if (t) t[i] = c->tw[i].state == TGSIM_TCP_PENDING ? INT64_MIN : c->tw[i].t;
  }
  return TGSIM_OK;
}

int tgo_tcp_writes_range(tgo_ctx* c, uint64_t first, size_t n, uint8_t* state, int64_t* t) {
  if (first + n > c->tw_n) return fail(c, TGSIM_EINVAL, "writes [%llu, +%zu) out of range", (unsigned long long)first, n);
  for (size_t i = 0; i < n; ++i) {
    const otcpw* w = &c->tw[first + i];
    if (state) state[i] = (uint8_t)w->state;
    if (t) t[i] = w->state == TGSIM_TCP_PENDING ? INT64_MIN : w->t;
  }
  return TGSIM_OK;
}

int tgo_tcp_get_stats(tgo_ctx* c, tgsim_tcp_stats* out) {
  if (!out) return TGSIM_EINVAL;
  *out = c->tstats;
  /* packets = every segment once + the retransmissions released (the device's definition: a
   * reserved segment counts whether or not its write was reached, e.g. a storm whose dials failed) */
  out->packets = c->tstats.segments + c->tstats.retransmissions - c->tstats.pending_retx;
  return TGSIM_OK;
}

/* ============================== storm plan reactor ==========================
 * plans/benchmarks/storm.go:117-190 per instance: `outgoing` goroutines sleep until t_ready, take
 * the dial semaphore `sem` (FIFO, concurrent slots), DialTimeout 30 s (:141-152); after
 * "outgoing-dials-done" each writes data_size in 4 KiB chunks, every conn.Write under `writesem`
 * (:158-183) and blocking its goroutine (holding the slot) while the send buffer is full. A dial is a
 * SYN answered by a SYN-ACK, a probe of DESIGN.md 2.12; a chunk stays in its connection's buffer until
 * its first copy arrives or it fails. Straight loops over instances and connections. */

enum { SM_SLEEP = 0, SM_WAIT = 1, SM_DONE = 2 };
#define SM_NONE INT64_MAX
#define SM_BUSY INT64_MAX
typedef struct ostorm_conn {
  uint32_t dst, slot, emit, rem, infl;
  uint8_t state, flags, res, pad;
  int64_t t_ready, t_start, t_synarr, t_ackarr, t_done, t_rep;
} ostorm_conn;
typedef struct ostorm ostorm;
struct ostorm {
  tgsim_storm_config cfg;
  uint32_t O, C, nchunks, phase;
  uint64_t n_conn;
  ostorm_conn* conn;
  uint32_t* order;  /* per instance its connections in (t_ready, k) order */
  uint8_t* claim;   /* per chunk: first arrival seen */
  uint32_t *dq, *qh, *ql, *nh, *ring, *hold;
  int64_t* slot_t;
  uint8_t* failed;
  int64_t* t_last;
  uint64_t written, delivered, failed_chunks, bytes;
  /* TCP mode: connection h is TCP connection h; write W0 + h * (nchunks + 1) + j
   * (j = 0 the SYN) and segments from S0 + h * spcon (the SYN's, then spc per full chunk) are
   * reserved at setup and linked onto the connection's queue when written */
  int tcp;
  uint32_t W0, S0, spc, spcon;
  uint32_t *settled, *wsegs;
  /* the listener's side of connection h (its shard is dst[h]'s): SYN answered, the SYN's first
   * arrival, and the connections answered in this reaction (sharded reactor) */
  uint8_t* ans;
  int64_t* lsyn;
  uint64_t* alist;
  size_t alist_n;
};
/* Notices from the listener's shard to the dialer's (records: t = value, src = connection, seq = kind):
 * the SYN-ACK the listener staged (value: its send time) and a chunk's arrival (value: chunk j). On
 * one shard they are applied in place; sharded, they cross in the exchange blocks (tgsim_transport). */
enum { SMN_SYNACK = 1u, SMN_CHUNK = 2u };

static void sm_free(tgo_ctx* c) {
  ostorm* s = c->sm;
  if (!s) return;
  free(s->conn); free(s->order); free(s->claim); free(s->dq); free(s->qh); free(s->ql); free(s->nh);
  free(s->ring); free(s->hold); free(s->slot_t); free(s->failed); free(s->t_last); free(s->settled); free(s->wsegs);
  free(s->ans); free(s->lsyn); free(s->alist);
  free(s);
  c->sm = NULL;
  c->sm_need_react = 0;
}

/* per instance, its connections in (t_ready, k) order: a stable insertion sort (no comparator state
 * shared between contexts - shards may be set up on several threads at once) */
static void sm_sort_order(uint32_t* o, const int64_t* tr, uint32_t O) {
  for (uint32_t k = 0; k < O; ++k) o[k] = k;
  for (uint32_t i = 1; i < O; ++i) {
    const uint32_t v = o[i];
    uint32_t j = i;
    while (j > 0 && tr[o[j - 1]] > tr[v]) { o[j] = o[j - 1]; --j; }
    o[j] = v;
  }
}

int tgo_storm_setup(tgo_ctx* c, const uint32_t* dst, const int64_t* t_ready, const tgsim_storm_config* cfg) {
  if (!cfg) return TGSIM_EINVAL;
  if (cfg->outgoing == 0 || cfg->concurrent == 0 || cfg->chunk_bytes == 0 || cfg->msg_window == 0 ||
      cfg->dial_timeout_ns <= 0 || cfg->window_ns <= 0 || cfg->syn_bytes >= 0x80000000u ||
      (uint64_t)cfg->chunk_bytes + cfg->header_bytes >= 0x80000000ull)
    return fail(c, TGSIM_EINVAL, "bad storm configuration");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (c->S != 1 && (c->tcp_on || !c->has_tr))
    return fail(c, TGSIM_ENOTSUP, "a sharded storm reactor needs message mode and a transport");
  if (c->fl_off || c->pr) return fail(c, TGSIM_ESTATE, "the storm reactor runs without a flood graph or probes");
  if (c->tcp_on && (!c->tcp.acks || c->tc_n || c->tw_n))
    return fail(c, TGSIM_ESTATE, "a TCP storm needs acks = 1 and a context without connections or writes yet");
  const uint64_t n_conn = (uint64_t)c->N * cfg->outgoing;
  const uint64_t nchunks = (cfg->data_bytes + cfg->chunk_bytes - 1) / cfg->chunk_bytes;
  if (n_conn > 0x3FFFFFFFull || nchunks * cfg->outgoing > 0x3FFFFFFFull)
    return fail(c, TGSIM_ENOTSUP, "too many connections or chunks for the storm's packet tags");
  if (n_conn && (!dst || !t_ready)) return fail(c, TGSIM_EINVAL, "bad arguments");
  for (uint64_t h = 0; h < n_conn; ++h) {
    if (dst[h] >= c->N) return fail(c, TGSIM_EINVAL, "connection %llu: bad peer", (unsigned long long)h);
    if (t_ready[h] < c->now) return fail(c, TGSIM_ECAUSALITY, "connection %llu: t_ready before now", (unsigned long long)h);
  }
  uint64_t spc = 0, spcon = 0, tot_w = 0, tot_s = 0;
  if (c->tcp_on) {
    const uint64_t mss = c->tcp.mss, last = nchunks ? cfg->data_bytes - (nchunks - 1) * cfg->chunk_bytes : 0;
    spc = (cfg->chunk_bytes + mss - 1) / mss;
    spcon = 1 + (nchunks ? (nchunks - 1) * spc + (last + mss - 1) / mss : 0);
    tot_w = n_conn * (nchunks + 1);
    tot_s = n_conn * spcon;
    if (n_conn > c->tcp.max_writes || tot_w > c->tcp.max_writes || tot_s > c->tcp.max_segments)
      return fail(c, TGSIM_ECAPACITY, "TCP storm: writes / segments exceed the TCP capacities");
  }
  sm_free(c);
  const uint32_t O = cfg->outgoing, C = cfg->concurrent, Hc = C < O ? C : O;
  const size_t nl = c->nloc ? c->nloc : 1, nc = n_conn ? n_conn : 1;
  ostorm* s = (ostorm*)calloc(1, sizeof(ostorm));
  if (!s) return fail(c, TGSIM_ENOMEM, "oom");
  c->sm = s;
  s->conn = (ostorm_conn*)calloc(nc, sizeof(ostorm_conn));
  s->order = (uint32_t*)malloc(nc * 4);
  s->claim = (uint8_t*)calloc(n_conn * nchunks + 1, 1);
  s->dq = (uint32_t*)calloc(nl, 4); s->qh = (uint32_t*)calloc(nl, 4); s->ql = (uint32_t*)calloc(nl, 4);
  s->nh = (uint32_t*)calloc(nl, 4); s->ring = (uint32_t*)calloc(nc, 4); s->hold = (uint32_t*)calloc(nl * Hc, 4);
  s->slot_t = (int64_t*)malloc(nl * C * 8); s->failed = (uint8_t*)calloc(nl, 1); s->t_last = (int64_t*)malloc(nl * 8);
  s->ans = (uint8_t*)calloc(nc, 1); s->lsyn = (int64_t*)malloc(nc * 8); s->alist = (uint64_t*)malloc(nc * 8);
  if (!s->conn || !s->order || !s->claim || !s->dq || !s->qh || !s->ql || !s->nh || !s->ring || !s->hold ||
      !s->slot_t || !s->failed || !s->t_last || !s->ans || !s->lsyn || !s->alist) { sm_free(c); return fail(c, TGSIM_ENOMEM, "oom"); }
  for (size_t i = 0; i < nc; ++i) s->lsyn[i] = SM_NONE;
  for (size_t i = 0; i < nl * C; ++i) s->slot_t[i] = INT64_MIN;
  for (size_t i = 0; i < nl; ++i) s->t_last[i] = INT64_MIN;
  for (uint64_t h = 0; h < n_conn; ++h) {
    s->conn[h].dst = dst[h];
    s->conn[h].t_ready = t_ready[h];
    s->conn[h].t_done = INT64_MIN;
  }
  for (uint32_t g = 0; g < c->N; ++g) sm_sort_order(s->order + (size_t)g * O, t_ready + (size_t)g * O, O);
  s->cfg = *cfg; s->O = O; s->C = C; s->nchunks = (uint32_t)nchunks; s->n_conn = n_conn; s->phase = 0;
  if (c->tcp_on) {  /* the connections, then the reserved writes and segments as tgo_tcp_write builds them */
    uint32_t* src = (uint32_t*)malloc(nc * 4);
    s->settled = (uint32_t*)calloc(nc, 4);
    s->wsegs = (uint32_t*)calloc(nc, 4);
    if (!src || !s->settled || !s->wsegs) { free(src); sm_free(c); return fail(c, TGSIM_ENOMEM, "oom"); }
    for (uint64_t h = 0; h < n_conn; ++h) src[h] = (uint32_t)(h / O);
    ostorm* keep = c->sm;
    c->sm = NULL;  /* tgo_tcp_connect refuses while a reactor owns the connections */
    const uint64_t lo = c->tc_n;
    int rc = tgo_tcp_connect(c, src, dst, n_conn, NULL);
    c->sm = keep;
    if (!rc) { c->sm_conn_lo = lo; c->sm_conn_hi = c->tc_n; }
    free(src);
    if (rc) { sm_free(c); return rc; }
    if (grow((void**)&c->tw, &c->tw_cap, c->tw_n + tot_w + 1, sizeof(otcpw)) ||
        grow((void**)&c->tsg, &c->tsg_cap, c->tsg_n + tot_s + 1, sizeof(otcps))) { sm_free(c); return fail(c, TGSIM_ENOMEM, "oom"); }
    s->tcp = 1; s->spc = (uint32_t)spc; s->spcon = (uint32_t)spcon;
    s->W0 = (uint32_t)c->tw_n; s->S0 = (uint32_t)c->tsg_n;
    const uint32_t mss = c->tcp.mss, hdr = c->tcp.header_bytes;
    for (uint64_t h = 0; h < n_conn; ++h) {
      for (uint32_t j = 0; j <= s->nchunks; ++j) {
        const uint32_t pay = j ? (j < s->nchunks ? cfg->chunk_bytes
                                                 : (uint32_t)(cfg->data_bytes - (uint64_t)(j - 1) * cfg->chunk_bytes)) : 0;
        const uint32_t ns = pay ? (pay + mss - 1) / mss : 1;
        const uint32_t wi = s->W0 + (uint32_t)h * (s->nchunks + 1) + j;
        const uint32_t first = s->S0 + (uint32_t)h * s->spcon + (j ? 1 + (j - 1) * s->spc : 0);
        otcpw w = {(uint32_t)(h / O), dst[h], ns, TGSIM_TCP_PENDING, INT64_MIN, (uint32_t)h};
        c->tw[wi] = w;
        for (uint32_t i = 0; i < ns; ++i) {
          otcps g = {wi, (pay ? (i + 1 < ns ? mss : pay - i * mss) : 0) + hdr, 0, 0, 0, 0, 0, INT64_MAX, INT64_MIN, 0, 0,
                     TCP_NOSEG, 1, 0};
          c->tsg[first + i] = g;
        }
      }
    }
    c->tw_n += tot_w; c->tsg_n += tot_s;
    c->tstats.writes += tot_w; c->tstats.segments += tot_s;
  }
  return TGSIM_OK;
}

/* TCP mode: a write's segments join connection h's send queue at time t (tgo_tcp_write's loop) */
static void sm_link(tgo_ctx* c, uint64_t h, uint32_t first, uint32_t n, int64_t t) {
  otcpc* q = &c->tc[h];
  for (uint32_t sid = first; sid < first + n; ++sid) {
    c->tsg[sid].t_att = t;
    if (q->tail != TCP_NOSEG) c->tsg[q->tail].next = sid;
    if (q->head == TCP_NOSEG) q->head = sid;
    if (q->una == TCP_NOSEG) q->una = sid;
    q->tail = sid;
    q->queued++;
  }
}
static uint32_t sm_wid(const ostorm* s, uint64_t h, uint32_t j) { return s->W0 + (uint32_t)h * (s->nchunks + 1) + j; }

static int sm_failed_code(uint8_t st) {
  const uint32_t code = st & 0x0Fu;
  return code != TGSIM_ST_QUEUED && code != TGSIM_ST_LOCAL;
}

/* Dial phase of instance g (frame: horizon H, window end t_end): resolve its waiting dials, then the
 * semaphore admits dials in FIFO order into free slots, each at max(t_ready, slot free, H), while
 * that is before the next window's end. */
static void sm_dials(tgo_ctx* c, uint32_t g, int resolve, int64_t H, int64_t t_end, pbuf* b, int64_t* dl_min,
                     int64_t* ns_min, uint32_t* act, uint32_t* waiting) {
  ostorm* s = c->sm;
  const uint32_t O = s->O, C = s->C, l = g - c->lo;
  const int64_t timeout = s->cfg.dial_timeout_ns;
  ostorm_conn* cn = s->conn + (size_t)g * O;
  for (uint32_t k = 0; k < O && resolve; ++k) {
    ostorm_conn* x = &cn[k];
    if (x->state != SM_WAIT) continue;
    if (s->tcp) {  /* the SYN write: ACKed (connect() returned, seen at the window's end) or failed */
      const uint64_t h = (uint64_t)g * O + k;
      const uint32_t ws = c->tw[sm_wid(s, h, 0)].state;
      uint8_t out = c->tc[h].acked >= 1 ? TGSIM_PROBE_OK
                  : ws == TGSIM_TCP_TIMEOUT ? TGSIM_PROBE_TIMEOUT : ws == TGSIM_TCP_REFUSED ? TGSIM_PROBE_REFUSED : TGSIM_PROBE_NONE;
      int64_t te = t_end;
      if (out == TGSIM_PROBE_NONE && x->t_start + timeout < t_end) {  /* net.DialTimeout (storm.go:144): */
        size_t unused = 0;                                             /* the SYN write fails at the deadline */
        te = x->t_start + timeout;
        out = TGSIM_PROBE_TIMEOUT;
        tcp_finish(c, sm_wid(s, h, 0), TGSIM_TCP_TIMEOUT, te, &unused);
      }
      if (out != TGSIM_PROBE_NONE) {
        x->state = SM_DONE; x->res = out; x->t_done = te;
        s->slot_t[(size_t)l * C + x->slot] = te;
      } else {
        ++*act; ++*waiting;
      }
      continue;
    }
    const int64_t dl = x->t_start + timeout;
    /* the listener answered the SYN's first arrival in this reaction (its notice): the SYN-ACK may
     * still beat the deadline, so a timeout waits one more window */
    const int reply_pending = (x->flags & 8u) && x->t_rep < dl;
    x->flags &= ~8u;
    uint8_t out = TGSIM_PROBE_NONE;
    int64_t te = 0;
    if (x->flags & 1u) { out = TGSIM_PROBE_REFUSED; te = x->t_start; }
    else if (x->t_ackarr != SM_NONE && x->t_ackarr < dl) { out = TGSIM_PROBE_OK; te = x->t_ackarr; }
    else if (dl < t_end && !reply_pending) { out = TGSIM_PROBE_TIMEOUT; te = dl; }
    if (out != TGSIM_PROBE_NONE) {
      x->state = SM_DONE; x->res = out; x->t_done = te;
      s->slot_t[(size_t)l * C + x->slot] = te;
    } else {
      ++*act; ++*waiting;
      if (dl < *dl_min) *dl_min = dl;
    }
  }
  if (s->tcp && t_end > H) H = t_end;  /* TCP: the reaction saw the previous dial end at the window's end */
  uint32_t q = s->dq[l];
  while (q < O) {
    uint32_t best = C;
    int64_t bt = SM_BUSY;
    for (uint32_t j = 0; j < C; ++j)
      if (s->slot_t[(size_t)l * C + j] < bt) { bt = s->slot_t[(size_t)l * C + j]; best = j; }
    if (best == C) break;
    const uint32_t k = s->order[(size_t)g * O + q];
    ostorm_conn* x = &cn[k];
    int64_t t0 = x->t_ready;
    if (bt > t0) t0 = bt;
    if (H > t0) t0 = H;
    if (t0 >= t_end + s->cfg.window_ns) { if (t0 < *ns_min) *ns_min = t0; break; }
    s->slot_t[(size_t)l * C + best] = SM_BUSY;
    x->slot = best; x->state = SM_WAIT; x->t_start = t0; x->flags = 0;
    ++*act; ++*waiting;
    ++q;
    if (s->tcp) {  /* the SYN: a bare segment written on the connection */
      const uint64_t h = (uint64_t)g * O + k;
      sm_link(c, h, s->S0 + (uint32_t)h * s->spcon, 1, t0);
      s->wsegs[h] = 1;
      continue;
    }
    x->t_ackarr = SM_NONE;
    pr_stage(b, g, x->dst, TGSIM_STORM_SYN | k, s->cfg.syn_bytes, t0);
    if (t0 + timeout < *dl_min) *dl_min = t0 + timeout;
  }
  s->dq[l] = q;
  *act += O - q;
}

static uint32_t sm_payload(const ostorm* s, uint32_t j) {
  return j + 1 < s->nchunks ? s->cfg.chunk_bytes : (uint32_t)(s->cfg.data_bytes - (uint64_t)j * s->cfg.chunk_bytes);
}
/* conn.Write of the connection's next chunk at t (the buffer had room) */
static uint32_t sm_nseg(const tgo_ctx* c, const ostorm* s, uint32_t j) {
  return (sm_payload(s, j) + c->tcp.mss - 1) / c->tcp.mss;
}
static void sm_write(tgo_ctx* c, uint32_t g, uint32_t k, int64_t t, pbuf* b) {
  ostorm* s = c->sm;
  const uint64_t h = (uint64_t)g * s->O + k;
  ostorm_conn* x = &s->conn[h];
  const uint32_t j = s->nchunks - x->rem;
  if (s->tcp) {  /* its segments after the previous write's last one */
    const uint32_t first = s->S0 + (uint32_t)h * s->spcon + 1 + j * s->spc, n = sm_nseg(c, s, j);
    sm_link(c, h, first, n, t);
    s->wsegs[h] += n;
  } else {
    pr_stage(b, g, x->dst, TGSIM_STORM_DATA | (k * s->nchunks + j), sm_payload(s, j) + s->cfg.header_bytes, t);
    x->infl++;
  }
  x->rem--;
  s->written++; s->bytes += sm_payload(s, j);
}
/* conn.Write of connection (g, k)'s next chunk fits: message mode, the buffer's `msg_window` chunks;
 * TCP, 2 x cwnd segments minus those written and not ACKed, one chunk per reaction */
static int sm_room(tgo_ctx* c, const ostorm* s, uint64_t h, uint32_t wrote_now) {
  const ostorm_conn* x = &s->conn[h];
  if (!s->tcp) return x->infl < s->cfg.msg_window;
  if (wrote_now) return 0;
  const int64_t buffered = (int64_t)s->wsegs[h] - (int64_t)c->tc[h].acked;
  return 2 * (int64_t)c->tc[h].cwnd - buffered >= (int64_t)sm_nseg(c, s, s->nchunks - x->rem);
}
/* Write phase of instance g at t: one writesem round (storm.go:158-183). */
static void sm_writes(tgo_ctx* c, uint32_t g, int64_t t, pbuf* b, uint32_t* act) {
  ostorm* s = c->sm;
  const uint32_t O = s->O, C = s->C, Hc = C < O ? C : O, win = s->cfg.msg_window, l = g - c->lo;
  ostorm_conn* cn = s->conn + (size_t)g * O;
  uint32_t* ring = s->ring + (size_t)g * O;
  uint32_t* hold = s->hold + (size_t)l * Hc;
  uint32_t qh = s->qh[l], ql = s->ql[l], nh = s->nh[l], wrote = 0;
  uint8_t now_[1024];  /* TCP: connections written in this round (one chunk per reaction) */
  uint8_t* now = O <= sizeof(now_) ? now_ : (uint8_t*)malloc(O);
  memset(now, 0, O);
  (void)win;
  if (s->tcp) {  /* settle the written chunks in order from their write states */
    for (uint32_t k = 0; k < O; ++k) {
      const uint64_t h = (uint64_t)g * O + k;
      const uint32_t written = s->nchunks - cn[k].rem;
      while (s->settled[h] < written) {
        const uint32_t st = c->tw[sm_wid(s, h, 1 + s->settled[h])].state;
        if (st == TGSIM_TCP_PENDING) break;
        if (st == TGSIM_TCP_DELIVERED) s->delivered++;
        else { s->failed_chunks++; s->failed[l] = 1; }
        s->settled[h]++;
      }
    }
  }
  int progress = 1;
  while (progress) {
    progress = 0;
    uint32_t keep = 0;
    for (uint32_t i = 0; i < nh; ++i) {  /* blocked writers whose buffer drained */
      const uint32_t k = hold[i];
      if (sm_room(c, s, (uint64_t)g * O + k, now[k])) {
        sm_write(c, g, k, t, b); now[k] = 1; ++wrote; progress = 1;
        if (cn[k].rem) { ring[(qh + ql) % O] = k; ++ql; }
      } else {
        hold[keep++] = k;
      }
    }
    nh = keep;
    while (nh < C && ql > 0) {  /* free slots go to the queue's head */
      const uint32_t k = ring[qh];
      qh = (qh + 1) % O; --ql;
      if (sm_room(c, s, (uint64_t)g * O + k, now[k])) {
        sm_write(c, g, k, t, b); now[k] = 1; ++wrote; progress = 1;
        if (cn[k].rem) { ring[(qh + ql) % O] = k; ++ql; }
      } else {
        hold[nh++] = k;
      }
    }
  }
  s->qh[l] = qh; s->ql[l] = ql; s->nh[l] = nh;
  if (wrote) s->t_last[l] = t;
  for (uint32_t k = 0; k < O; ++k) {
    const uint64_t h = (uint64_t)g * O + k;
    *act += (cn[k].rem || (s->tcp ? s->settled[h] < s->nchunks - cn[k].rem : cn[k].infl != 0)) ? 1u : 0u;
  }
  if (now != now_) free(now);
}

/* one reaction frame (H, t_end): every instance's step, then the proposal of the next window's end */
/* one reaction frame (H, t_end): every local instance's step, then the proposal of the next window's
 * end. propose: sharded, the proposal is collective (every shard's busy flag, active count and
 * earliest deadline / dial start gathered over the transport; the one-shard rule over the whole). */
static int sm_step(tgo_ctx* c, int resolve, int64_t H, int64_t t_end, int64_t* next_end, uint32_t* n_active,
                   int propose) {
  ostorm* s = c->sm;
  pbuf b;
  const size_t cap = s->phase ? (size_t)s->n_conn * s->cfg.msg_window + 1 : 2 * (size_t)s->n_conn + 1;
  if (pr_alloc(&b, cap)) { pr_free(&b); return fail(c, TGSIM_ENOMEM, "oom"); }
  int64_t dl = SM_NONE, ns = SM_NONE;
  uint32_t act = 0, waiting = 0;
  for (uint32_t g = c->lo; g < c->hi; ++g) {
    if (s->phase) sm_writes(c, g, t_end, &b, &act);
    else sm_dials(c, g, resolve, H, t_end, &b, &dl, &ns, &act, &waiting);
  }
  int rc = pr_flush(c, &b);
  if (rc) return rc;
  /* TCP: the windows' room goes at the write times (tgo_tcp_write's release); the proposal looks
   * at the staged packets before it, as the device does (its release runs after the reaction) */
  const int staged_before = c->staged.n != 0;
  if (s->tcp) {
    ostage q = {0};
    size_t done = 0;
    for (uint32_t k = 0; k < c->tc_n && !rc; ++k)
      if (!c->tc[k].broken) rc = conn_release(c, k, INT64_MIN, &q, &done);
    const int rc2 = ostage_flush(c, &q);
    if (rc || rc2) return rc ? fail(c, rc, "oom") : rc2;
  }
  int64_t cand = dl != SM_NONE ? dl + 1 : SM_NONE;
  if (ns < cand) cand = ns;
  int64_t busy = staged_before || c->heap.n || (s->tcp && waiting), tot = act;
  if (propose && c->S > 1) {
    int64_t mine[3] = {busy, (int64_t)act, cand};
    int64_t* all = (int64_t*)malloc((size_t)c->S * 3 * 8);
    if (!all) return fail(c, TGSIM_ENOMEM, "oom");
    if (c->tr.allgather(c->tr.user, mine, all, sizeof(mine), NULL) != 0) {
      free(all);
      return fail(c, TGSIM_EHIP, "transport all-gather failed");
    }
    busy = 0; tot = 0; cand = SM_NONE;
    for (uint32_t k = 0; k < c->S; ++k) {
      busy |= all[3 * k];
      tot += all[3 * k + 1];
      if (all[3 * k + 2] < cand) cand = all[3 * k + 2];
    }
    free(all);
  }
  int64_t ne = t_end + s->cfg.window_ns;
  if (!busy && tot && cand != SM_NONE && cand > ne) ne = cand;  /* idle: jump to the next deadline or dial */
  if (next_end) *next_end = ne;
  if (n_active) *n_active = (uint32_t)tot;
  return TGSIM_OK;
}

int tgo_storm_start(tgo_ctx* c) {
  if (!c->sm) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->sm->phase != 0) return fail(c, TGSIM_ESTATE, "the storm's dials have started");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (react_owed(c)) return TGSIM_ESTATE;
  return sm_step(c, 0, c->now, c->now, NULL, NULL, 0);
}

/* The connection of a chunk packet (src -> dst, chunk id cj = k * nchunks + j) on its dialer's shard,
 * or -1 when no chunk the storm has written matches it (a message the host staged beside the
 * reactor: ADVICE r4). */
static int64_t sm_chunk_conn(const ostorm* s, uint32_t src, uint32_t dst, uint32_t cj) {
  if (s->nchunks == 0) return -1;
  const uint32_t k = cj / s->nchunks, j = cj - k * s->nchunks;
  const uint64_t h = (uint64_t)src * s->O + k;
  if (k >= s->O || h >= s->n_conn || s->conn[h].dst != dst || j >= s->nchunks - s->conn[h].rem) return -1;
  return (int64_t)h;
}

/* A notice on the dialer's shard: the SYN-ACK its listener staged (sent at v), or the arrival of
 * chunk j = v (the first copy of a written chunk frees its buffer slot) */
static void sm_notice_apply(tgo_ctx* c, uint64_t h, uint32_t kind, int64_t v) {
  ostorm* s = c->sm;
  if (h >= s->n_conn) return;
  ostorm_conn* x = &s->conn[h];
  if (kind == SMN_SYNACK) {
    x->flags |= 2u | 8u;
    x->t_rep = v;
  } else if (kind == SMN_CHUNK) {
    const int64_t hh = sm_chunk_conn(s, (uint32_t)(h / s->O), x->dst, (uint32_t)((h % s->O) * s->nchunks + v));
    if (hh < 0 || v < 0 || (uint64_t)v >= s->nchunks) return;
    const uint64_t bit = h * s->nchunks + (uint64_t)v;
    if (!s->claim[bit]) { s->claim[bit] = 1; x->infl--; s->delivered++; }
  }
}
static int sm_notice(tgo_ctx* c, uint64_t h, uint32_t kind, int64_t v) {
  const uint32_t p = shard_of(c, (uint32_t)(h / c->sm->O));
  if (p == c->cfg.shard_id) { sm_notice_apply(c, h, kind, v); return TGSIM_OK; }
  tgsim_record r;
  memset(&r, 0, sizeof(r));
  r.t = v; r.src = (uint32_t)h; r.seq = kind;
  return recs_push(&c->outbox[p], &r) ? fail(c, TGSIM_ENOMEM, "oom") : TGSIM_OK;
}

/* Sharded: the notices cross in the exchange blocks (peer-major, header .t = count), then apply */
static int sm_notice_exchange(tgo_ctx* c) {
  memset(c->xsend, 0, (size_t)c->S * c->xcap * sizeof(tgsim_record));
  for (uint32_t p = 0; p < c->S; ++p) {
    orecs* o = &c->outbox[p];
    if (p == c->cfg.shard_id) continue;
    if (o->n + 1 > c->xcap) return fail(c, TGSIM_ECAPACITY, "storm notices exceed the exchange capacity (%zu to peer %u)", o->n, p);
    c->xsend[(size_t)p * c->xcap].t = (int64_t)o->n;
    memcpy(&c->xsend[(size_t)p * c->xcap + 1], o->v, o->n * sizeof(tgsim_record));
    o->n = 0;
  }
  if (c->tr.alltoall(c->tr.user, c->xsend, c->xrecv, c->xcap * sizeof(tgsim_record), NULL) != 0)
    return fail(c, TGSIM_EHIP, "transport all-to-all failed");
  for (uint32_t p = 0; p < c->S; ++p) {
    if (p == c->cfg.shard_id) continue;
    const tgsim_record* blk = &c->xrecv[(size_t)p * c->xcap];
    const size_t n = (size_t)blk[0].t;
    if (n + 1 > c->xcap) return fail(c, TGSIM_ECAPACITY, "corrupt exchange header");
    for (size_t i = 0; i < n; ++i) sm_notice_apply(c, blk[1 + i].src, blk[1 + i].seq, blk[1 + i].t);
  }
  return TGSIM_OK;
}

static int storm_react_impl(tgo_ctx* c, int64_t* next_end, uint32_t* n_active) {
  ostorm* s = c->sm;
  if (!s) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (!c->sm_need_react) return fail(c, TGSIM_ESTATE, "storm: no window since the last reaction");
  if (c->tcp_need_react) return fail(c, TGSIM_ESTATE, "TCP mode: tcp_react before storm_react");
  if (c->S != 1 && !c->has_tr) return fail(c, TGSIM_ESTATE, "the transport was aborted (a shard failed)");
  c->sm_need_react = 0;
  if (s->tcp) return sm_step(c, 1, c->horizon, c->now, next_end, n_active, 1);  /* the TCP reaction settled the window */
  const omsgs* st = &c->staged;
  const uint32_t O = s->O;
  int rc = TGSIM_OK;
  for (uint32_t p = 0; p < c->S; ++p) c->outbox[p].n = 0;
  /* 1. the window's packets (local dialers): refused SYNs, chunks no copy of entered the egress queue */
  for (size_t i = 0; i < c->n_status; ++i) {
    const uint32_t sq = st->seq[i], tag = sq >> 30, code = c->status[i] & 0x0Fu;
    if (tag == 1u) {
      const size_t h = (size_t)st->src[i] * O + (sq & PR_MASK);
      if ((sq & PR_MASK) >= O || h >= s->n_conn) continue;
      ostorm_conn* x = &s->conn[h];
      if ((code == TGSIM_ST_DROPPED || code == TGSIM_ST_REJECTED || code == TGSIM_ST_UNREACHABLE) &&
          x->state == SM_WAIT && x->dst == st->dst[i])
        x->flags |= 1u;
    } else if (tag == 2u && sm_failed_code(c->status[i])) {
      const int64_t h = sm_chunk_conn(s, st->src[i], st->dst[i], sq & PR_MASK);
      if (h < 0) continue;
      s->conn[h].infl--;
      s->failed[st->src[i] - c->lo] = 1;
      s->failed_chunks++;
    }
  }
  /* 2. the window's deliveries (local receivers): a SYN at its listener (first arrival of the
   *    connection's SYN: answered in this reaction), a SYN-ACK at its dialer, a chunk at its listener
   *    (the dialer's shard claims its first copy) */
  s->alist_n = 0;
  for (size_t i = 0; i < c->out.n && !rc; ++i) {
    const tgsim_record* r = &c->out.v[i];
    const uint32_t tag = r->seq >> 30;
    if (tag == 1u) {
      const uint64_t h = (uint64_t)r->src * O + (r->seq & PR_MASK);
      if ((r->seq & PR_MASK) >= O || h >= s->n_conn || s->conn[h].dst != r->dst || s->ans[h] == 1) continue;
      if (s->ans[h] == 0) { s->ans[h] = 2; s->alist[s->alist_n++] = h; }  /* 2: answered in this reaction */
      if (r->t < s->lsyn[h]) s->lsyn[h] = r->t;
    } else if (tag == 3u) {
      const size_t h = r->seq & PR_MASK;
      if (h < s->n_conn && h / O == r->dst) {
        ostorm_conn* x = &s->conn[h];
        if (x->dst == r->src && x->state == SM_WAIT && r->t < x->t_ackarr) x->t_ackarr = r->t;
      }
    } else if (tag == 2u && s->nchunks) {
      const uint32_t cj = r->seq & PR_MASK, k = cj / s->nchunks;
      const uint64_t h = (uint64_t)r->src * O + k;
      if (k >= O || h >= s->n_conn || s->conn[h].dst != r->dst) continue;
      rc = sm_notice(c, h, SMN_CHUNK, cj - k * s->nchunks);
    }
  }
  /* 3. the listeners answer: a SYN-ACK at max(first arrival, horizon) per connection answered now */
  pbuf b;
  if (!rc && pr_alloc(&b, s->alist_n + 1)) { pr_free(&b); rc = fail(c, TGSIM_ENOMEM, "oom"); }
  if (rc) return rc;
  for (size_t i = 0; i < s->alist_n && !rc; ++i) {
    const uint64_t h = s->alist[i];
    const int64_t trep = s->lsyn[h] > c->horizon ? s->lsyn[h] : c->horizon;
    s->ans[h] = 1;
    pr_stage(&b, s->conn[h].dst, (uint32_t)(h / O), TGSIM_STORM_SYNACK | (uint32_t)h, s->cfg.syn_bytes, trep);
    rc = sm_notice(c, h, SMN_SYNACK, trep);
  }
  if (rc) { pr_free(&b); return rc; }
  rc = pr_flush(c, &b);
  if (rc) return rc;
  /* 4. sharded: the notices to the dialers' shards */
  if (c->S > 1 && (rc = sm_notice_exchange(c))) return rc;
  /* 5. per local instance: dials or writes, then the proposal */
  return sm_step(c, 1, c->horizon, c->now, next_end, n_active, 1);
}
int tgo_storm_react(tgo_ctx* c, int64_t* next_end, uint32_t* n_active) {
  return shard_failed(c, storm_react_impl(c, next_end, n_active));
}

/* the local instances' connections: [lo * O, hi * O) */
int tgo_storm_dials(tgo_ctx* c, uint8_t* outcome, int64_t* t_done, size_t cap) {
  ostorm* s = c->sm;
  if (!s) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  const uint64_t h0 = (uint64_t)c->lo * s->O, n = (uint64_t)c->nloc * s->O;
  if ((outcome || t_done) && cap < n) return fail(c, TGSIM_ECAPACITY, "dial capacity");
  for (uint64_t i = 0; i < n; ++i) {
    if (outcome) outcome[i] = s->conn[h0 + i].res;
    if (t_done) t_done[i] = s->conn[h0 + i].t_done;
  }
  return TGSIM_OK;
}

int tgo_storm_write_start(tgo_ctx* c, int64_t t0) {
  ostorm* s = c->sm;
  if (!s) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (s->phase != 0) return fail(c, TGSIM_ESTATE, "the write phase has started");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  if (react_owed(c)) return TGSIM_ESTATE;
  if (t0 < c->horizon) return fail(c, TGSIM_ECAUSALITY, "t0 before the reaction horizon");
  /* storm.go:156: every dial of every instance OK (sharded: agreed over the transport) */
  int64_t bad = -1;
  for (uint64_t h = (uint64_t)c->lo * s->O; h < (uint64_t)c->hi * s->O && bad < 0; ++h)
    if (s->conn[h].res != TGSIM_PROBE_OK) bad = (int64_t)h;
  if (c->S > 1) {
    if (!c->has_tr) return fail(c, TGSIM_ESTATE, "the transport was aborted (a shard failed)");
    if (c->tr.allreduce_max_i64(c->tr.user, &bad, 1, NULL) != 0) return shard_failed(c, fail(c, TGSIM_EHIP, "transport all-reduce failed"));
  }
  if (bad >= 0) return fail(c, TGSIM_ESTATE, "connection %lld has not dialled successfully", (long long)bad);
  s->phase = 1;
  for (uint32_t g = c->lo; g < c->hi; ++g) {
    uint32_t n = 0;
    for (uint32_t k = 0; k < s->O; ++k) {
      ostorm_conn* x = &s->conn[(size_t)g * s->O + k];
      x->rem = s->nchunks; x->infl = 0;
      if (s->nchunks) s->ring[(size_t)g * s->O + n++] = k;
    }
    s->qh[g - c->lo] = 0; s->ql[g - c->lo] = n; s->nh[g - c->lo] = 0;
  }
  return sm_step(c, 0, t0, t0, NULL, NULL, 0);
}

int tgo_storm_results(tgo_ctx* c, uint8_t* failed, int64_t* t_last, size_t cap, tgsim_storm_totals* tot) {
  ostorm* s = c->sm;
  if (!s) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if ((failed || t_last) && cap < c->nloc) return fail(c, TGSIM_ECAPACITY, "result capacity");
  for (uint32_t g = 0; g < c->nloc; ++g) {
    uint8_t f = s->failed[g];
    for (uint32_t k = 0; k < s->O; ++k) {
      const uint64_t h = (uint64_t)(c->lo + g) * s->O + k;
      const ostorm_conn* x = &s->conn[h];
      f |= (s->phase == 1 && x->rem) ? 1 : 0;
      f |= (s->tcp ? (s->phase == 1 && s->settled[h] < s->nchunks - x->rem) : x->infl != 0) ? 1 : 0;
    }
    if (failed) failed[g] = f;
    if (t_last) t_last[g] = s->t_last[g];
  }
  if (tot) {
    memset(tot, 0, sizeof(*tot));
    tot->chunks_written = s->written; tot->chunks_delivered = s->delivered;
    tot->chunks_failed = s->failed_chunks; tot->bytes_written = s->bytes;
    for (uint64_t h = (uint64_t)c->lo * s->O; h < (uint64_t)c->hi * s->O; ++h) {  /* the local connections */
      const ostorm_conn* x = &s->conn[h];
      tot->dials_ok += x->res == TGSIM_PROBE_OK;
      tot->dials_failed += x->res == TGSIM_PROBE_REFUSED || x->res == TGSIM_PROBE_TIMEOUT;
      tot->dials_pending += x->res == TGSIM_PROBE_NONE;
      tot->conns_writing += s->phase == 1 && (x->rem || (s->tcp ? s->settled[h] < s->nchunks - x->rem : x->infl != 0));
    }
  }
  return TGSIM_OK;
}

int tgo_storm_end(tgo_ctx* c) {
  if (!c->sm) return fail(c, TGSIM_ESTATE, "no storm reactor set up");
  if (c->in_window) return fail(c, TGSIM_ESTATE, "inside a window");
  sm_free(c);
  return TGSIM_OK;
}

