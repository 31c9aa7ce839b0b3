/*
 * tgsim_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement (single-threaded, plain C) of the
 * Testground sidecar data path that the HIP simulator (testground_amd/csrc) implements.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline. The product path never calls it.
 *
 * Parity status: the reference's path is Go + host-kernel netem/HTB/FIB +
 * un-vendored sdk-go/netlink/sync-service; none is buildable or importable here (no Go toolchain).
 * This oracle therefore restates the algorithm from the reference call sites (file:line in each
 * function) and from the recalled upstream algorithms marked [EXT]. It is pinned by:
 *   - Philox4x32-10 known-answer vectors (Random123 published KATs + rocRAND's host Philox),
 *   - the reference plans' known answers: ping-pong RTT windows (plans/network/pingpong.go:185,195),
 *     splitbrain reachability truth table (plans/splitbrain/main.go:50-58), routing-policy
 *     allowed/blocked (plans/network/traffic.go:46-52), sidecar config pass-through/errors
 *     (pkg/sidecar/sidecar_test.go:58-59,88-92), data-subnet table (pkg/runner/common_test.go:14-20).
 * Loss/jitter/duplicate/corrupt/bandwidth distributions are "parity unpinned" against real netem.
 *
 * The API mirrors include/tgsim.h one-for-one (tgo_* for tgsim_*), so tests can drive both with
 * identical inputs and compare outputs bit for bit.
 */
#ifndef TGSIM_ORACLE_H
#define TGSIM_ORACLE_H
#include "../include/tgsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tgo_ctx tgo_ctx;

/* primitives exposed for known-answer tests */
void tgo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t tgo_percentage2u32(float pct);
uint32_t tgo_time2tick(uint32_t us);
uint32_t tgo_to_microseconds(int64_t ns);
void tgo_ratecfg(uint64_t rate_Bps, uint32_t* mult, uint32_t* shift);
/* derived netem/htb parameters of a LinkShape: out[0]=mu_ns out[1]=sigma out[2]=loss_t out[3]=dup_t
 * out[4]=corrupt_t out[5]=reorder_t out[6]=tb_mult out[7]=tb_shift out[8]=tau_ns out[9]=limited */
int tgo_derive_shape(const tgsim_link_shape* s, int64_t out[10]);
int tgo_next_data_network(int len_networks, uint32_t* subnet, uint32_t* prefix_len, uint32_t* gw);

int tgo_create(const tgsim_config* cfg, tgo_ctx** out);
void tgo_destroy(tgo_ctx* ctx);
const char* tgo_last_error(const tgo_ctx* ctx);
int64_t tgo_now(const tgo_ctx* ctx);
int64_t tgo_horizon(const tgo_ctx* ctx);
int tgo_configure_network(tgo_ctx* ctx, uint32_t instance, const tgsim_network_config* cfg);
int tgo_configure_network_order(tgo_ctx* ctx, uint32_t instance, const tgsim_network_config* cfg, int32_t order);
int tgo_set_shape(tgo_ctx* ctx, uint32_t instance, const tgsim_link_shape* shape);
int tgo_set_shapes(tgo_ctx* ctx, const uint32_t* instances, const tgsim_link_shape* shapes, size_t n);
int tgo_add_rules(tgo_ctx* ctx, uint32_t instance, const tgsim_link_rule* rules, size_t n);
int tgo_set_policy(tgo_ctx* ctx, uint32_t instance, int32_t policy);
int tgo_set_enabled(tgo_ctx* ctx, uint32_t instance, int32_t enabled, int32_t has_ip, uint32_t ip);
int tgo_get_ip(const tgo_ctx* ctx, uint32_t instance, uint32_t* ip);

int tgo_enqueue(tgo_ctx* ctx, const tgsim_msg_soa* msgs, size_t n);
int tgo_advance(tgo_ctx* ctx, int64_t t_end);
int tgo_advance_async(tgo_ctx* ctx, int64_t t_end);
int tgo_tcp_enable(tgo_ctx* ctx, const tgsim_tcp_config* cfg);
int tgo_tcp_send(tgo_ctx* ctx, const tgsim_msg_soa* writes, size_t n);
int tgo_tcp_react(tgo_ctx* ctx, size_t* n_completed);
int tgo_tcp_writes(tgo_ctx* ctx, uint8_t* state_out, int64_t* t_out, size_t cap, size_t* n);
int tgo_tcp_get_stats(tgo_ctx* ctx, tgsim_tcp_stats* out);
int tgo_tcp_writes_range(tgo_ctx* ctx, uint64_t first, size_t n, uint8_t* state_out, int64_t* t_out);
int tgo_tcp_connect(tgo_ctx* ctx, const uint32_t* src, const uint32_t* dst, size_t n, uint32_t* conn_out);
int tgo_tcp_write(tgo_ctx* ctx, const uint32_t* conn, const uint32_t* size, const int64_t* t_send, size_t n);
int tgo_tcp_conns(tgo_ctx* ctx, uint32_t first, size_t n, uint64_t* acked, uint32_t* cwnd, uint32_t* flight,
                  uint32_t* queued);
int tgo_tcp_gen_storm_round(tgo_ctx* ctx, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                            int64_t spread_ns, uint32_t state);
int tgo_advance_begin(tgo_ctx* ctx, int64_t t_end);
/* host buffers, same layout as tgsim_exchange_buffers (peer-major, header record per peer) */
int tgo_exchange_buffers(tgo_ctx* ctx, void** send, void** recv, size_t* bytes);
int tgo_advance_end(tgo_ctx* ctx);
int tgo_set_transport(tgo_ctx* ctx, const tgsim_transport* transport); /* host buffers, stream NULL */
int tgo_comm_abort(tgo_ctx* ctx);
int tgo_delivery_count(tgo_ctx* ctx, size_t* n);
int tgo_copy_deliveries(tgo_ctx* ctx, tgsim_delivery_soa* out, size_t cap, size_t* n);
int tgo_copy_inbox_offsets(tgo_ctx* ctx, uint32_t* out, size_t cap);
int tgo_copy_status(tgo_ctx* ctx, uint8_t* out, size_t cap, size_t* n);
int tgo_get_stats(tgo_ctx* ctx, tgsim_stats* out);

int tgo_sync_signal(tgo_ctx* ctx, const uint32_t* states, const uint32_t* instances,
                    const int64_t* t, size_t n, uint32_t* seq_out);
int tgo_sync_barrier(tgo_ctx* ctx, uint32_t state, uint32_t target, int64_t t_wait, uint32_t* waiter_out);
int tgo_sync_poll(tgo_ctx* ctx, uint32_t waiter, int64_t* release_out);
int tgo_sync_count(tgo_ctx* ctx, uint32_t state, uint32_t* count_out);
int tgo_sync_publish(tgo_ctx* ctx, const uint32_t* topics, const uint32_t* instances, const int64_t* t,
                     const uint64_t* payload_off, const uint8_t* payload, size_t n, uint32_t* pos_out);
int tgo_sync_subscribe(tgo_ctx* ctx, uint32_t topic, uint32_t from, int64_t until_t, size_t cap,
                       uint32_t* instances_out, int64_t* t_out, uint64_t* payload_off_out,
                       uint8_t* payload_out, size_t payload_cap, size_t* n_out, size_t* payload_bytes);
int tgo_advance_to_barrier(tgo_ctx* ctx, uint32_t waiter, int64_t offset_ns);

int tgo_gen_storm_round(tgo_ctx* ctx, uint32_t round, int64_t t0, uint32_t fanout, uint32_t size,
                        int64_t spread_ns, uint32_t state);
int tgo_storm_release(tgo_ctx* ctx, int64_t* out); /* host-side twin of tgsim_storm_release_device */

/* Flood with first-receipt dedup over a fixed graph (tgsim.h). */
int tgo_flood_set_graph(tgo_ctx* ctx, const uint32_t* offsets, const uint32_t* neighbors, uint32_t max_pubs);
int tgo_flood_publish(tgo_ctx* ctx, const uint32_t* instances, const uint32_t* pubs, const int64_t* t, size_t n,
                      uint32_t size);
int tgo_flood_react(tgo_ctx* ctx, uint32_t size, size_t* n_forwarded);
int tgo_probe_setup(tgo_ctx* ctx, const uint32_t* order, uint32_t n_order, const tgsim_probe_config* cfg);
int tgo_probe_start(tgo_ctx* ctx, int64_t t0);
int tgo_probe_react(tgo_ctx* ctx, int64_t* next_end, uint32_t* n_active);
int tgo_probe_results(tgo_ctx* ctx, uint8_t* outcome, int64_t* t_done, size_t cap_outcome);
int tgo_storm_setup(tgo_ctx* ctx, const uint32_t* dst, const int64_t* t_ready, const tgsim_storm_config* cfg);
int tgo_storm_start(tgo_ctx* ctx);
int tgo_storm_react(tgo_ctx* ctx, int64_t* next_end, uint32_t* n_active);
int tgo_storm_dials(tgo_ctx* ctx, uint8_t* outcome, int64_t* t_done, size_t cap);
int tgo_storm_write_start(tgo_ctx* ctx, int64_t t0);
int tgo_storm_results(tgo_ctx* ctx, uint8_t* failed, int64_t* t_last, size_t cap, tgsim_storm_totals* totals);
int tgo_storm_end(tgo_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
