/*
 * scion_hfv.h -- C ABI of libscionhfv.so: SCION border-router hop-field (HF) AES-CMAC
 * verification on AMD MI355X (gfx950).
 *
 * What it replaces in the reference (netsys-lab/scion-xdp-br):
 *   - the per-packet data-plane call  int verify_hop_field(struct macinput*, u64 expected)
 *     (br/src/bpf/xdp.c:77-91) together with the macinput assembly and beta/SegID rule of
 *     defer_verify_hop_field / scion_as_ingress (br/src/bpf/path_processing.h:39-81),
 *     now executed for a whole batch per kernel launch;
 *   - the control-plane key table  mac_key_map  (br/src/bpf/maps.h:60-67) and its writers
 *     `br-loader key add|remove` (br/src/br_loader.cpp:182-261).
 *
 * Conventions
 *   - Status: 0 on success, a negative errno on failure (-EINVAL bad argument, -ENODEV no
 *     usable GPU, -ENOMEM allocation, -EIO HIP runtime error).  hfv_last_error() returns a
 *     human-readable message for the calling thread.  No C++ exception crosses the ABI.
 *   - Batch buffers (records, macinputs, tags, pass bitmaps) are DEVICE pointers (hipMalloc,
 *     hipMallocManaged or a framework allocation on the ctx's GPU) unless a function says
 *     otherwise.  `stream` is a hipStream_t passed as void*; NULL is HIP's default
 *     stream (hfv_ctx_stream() returns a private non-blocking stream of the ctx).  Calls enqueue work and return; completion is stream-ordered.
 *   - Verdict output: bit (i % 64) of pass_bits[i / 64] is 1 iff packet i's hop field
 *     verifies; bits for i >= n in the last word are 0.  A missing key fails closed
 *     (xdp.c:83-84).
 *   - Threading: one ctx per GPU, used by one host thread at a time (or externally
 *     serialised), like one XDP program instance per CPU queue.
 */
#ifndef SCION_HFV_H
#define SCION_HFV_H

#include <stddef.h>
#include <stdint.h>

#include "hfv_aes.h"

#ifdef __cplusplus
extern "C" {
#endif

#define HFV_ABI_VERSION 3
#define HFV_MAX_KEYS 256          /* key slots; the reference map holds 8 (maps.h:60-67) */
#define HFV_REC_INF_OFF 40        /* default 64 B record layout, DESIGN.md section 3 */
#define HFV_REC_HF_OFF 48

/* struct macinput (include/bpf/scion.h:122-132): 16 B, wire byte order */
struct macinput {
    uint16_t null0;
    uint16_t beta;
    uint32_t ts;
    uint8_t null1;
    uint8_t exp;
    uint16_t ingress;
    uint16_t egress;
    uint16_t null2;
} __attribute__((packed));

/* struct hop_key (br/src/bpf/common.h:87-91): expanded key + CMAC subkey K1, 192 B */
struct hop_key {
    struct aes_key_schedule key;
    struct aes_block subkey;
};

/* Per-packet key selection (SURVEY.md 8b iii) */
enum hfv_keysel {
    HFV_KEYSEL_ZERO = 0,  /* mac_key_map[0] for every packet: the reference rule, xdp.c:82 */
    HFV_KEYSEL_IFID = 1,  /* slot = AS-ingress IFID & 0xff, IFID = Cons ? HF.ingress : HF.egress
                             (the hf_ingress rule of xdp.c:151-157) */
};

typedef struct hfv_ctx hfv_ctx;

/* ---- lifetime ----------------------------------------------------------------------
 * Replaces the mac_key_map creation/pinning part of attachBr (br_loader.cpp:88-151). */
int hfv_ctx_create(int device, hfv_ctx **out);
int hfv_ctx_destroy(hfv_ctx *ctx);
int hfv_ctx_device(const hfv_ctx *ctx);
/* NUMA node of the ctx's GPU (its PCIe root port), -1 if unknown.  The library's host worker
 * threads (staging copies of the host-memory paths) run on that node's CPUs (HFV_NUMA_PIN=0:
 * unpinned); a host feeder thread per GPU should be placed there too. */
int hfv_ctx_numa_node(const hfv_ctx *ctx);
void *hfv_ctx_stream(hfv_ctx *ctx);
int hfv_ctx_set_keysel(hfv_ctx *ctx, int keysel);
/* Offsets of the current InfoField / HopField inside each record (multiples of 8). */
int hfv_ctx_set_record_layout(hfv_ctx *ctx, uint32_t inf_off, uint32_t hf_off);
/* Wait for all work the ctx enqueued on its own stream. */
int hfv_ctx_synchronize(hfv_ctx *ctx);

/* ---- key table (mac_key_map) -------------------------------------------------------
 * Updates are made on a host shadow table and published to the GPU at the next batch
 * boundary (stream-ordered, double-buffered): batches already enqueued keep the table
 * they were launched with, like RCU readers of the BPF hash map. */
/* br-loader key add: decodeKey -> aes_key_expansion -> aes_cmac_subkeys -> keep K1
 * -> map update (br_loader.cpp:182-229). */
int hfv_key_add(hfv_ctx *ctx, uint32_t index, const struct aes_key *key);
/* Same, from the 24-character base64 form the CLI takes (decodeKey, br_loader.cpp:65-73). */
int hfv_key_add_b64(hfv_ctx *ctx, uint32_t index, const char *base64);
/* Map::update with a ready hop_key (what br-loader writes to the map). */
int hfv_key_set_hop_key(hfv_ctx *ctx, uint32_t index, const struct hop_key *hk);
/* br-loader key remove: Map::erase (br_loader.cpp:231-261); the slot then fails closed.
 * Returns -ENOENT if the slot was empty (the BPF map erase fails the same way). */
int hfv_key_remove(hfv_ctx *ctx, uint32_t index);
/* Map lookup: copies the slot's hop_key, -ENOENT if empty. */
int hfv_key_get(hfv_ctx *ctx, uint32_t index, struct hop_key *out);

/* ---- pinned key map ------------------------------------------------------------------
 * A file-backed mac_key_map that other processes update while the data plane runs, the
 * analogue of the bpffs-pinned map /sys/fs/bpf/<br>/mac_key_map (br_loader.cpp:119-126,
 * 191, 221-222).  Path: $HFV_PIN_DIR/<br>/mac_key_map, HFV_PIN_DIR defaults to /dev/shm/hfv.
 * Writers serialise with flock; readers see whole updates (seqlock). */
int hfv_keymap_path(const char *br, char *out, size_t len);
/* Map modes, fixed when the map is created:
 *   HFV_KEYMAP_SLOTS  256 direct slots, index 0..255 (per-interface keys, config 3);
 *   HFV_KEYMAP_HASH8  the reference map's semantics (maps.h:60-67: BPF_MAP_TYPE_HASH, u32
 *                     index, max_entries 8): any u32 index, a 9th new index fails with -E2BIG
 *                     as bpf_map_update_elem does.  The data plane reads indices < 256 (slot 0
 *                     in the reference's single-key mode, xdp.c:82); larger ones are kept and
 *                     listed but never looked up.  `hfv-loader` creates this mode. */
#define HFV_KEYMAP_SLOTS 0
#define HFV_KEYMAP_HASH8 1
/* Map::update (BPF_ANY) of one index, creating a SLOTS map file if needed. */
int hfv_keymap_update(const char *path, uint32_t index, const struct hop_key *hk);
/* An empty map (no slot written) if the file does not exist yet; an existing map is kept. */
int hfv_keymap_create(const char *path);
/* The same with the mode; an existing map without keys takes the mode, one with keys keeps its own. */
int hfv_keymap_create_mode(const char *path, int mode);
/* The map's mode (>= 0) or a negative errno. */
int hfv_keymap_mode(const char *path);
/* Map::erase of one index; -ENOENT if it was empty. */
int hfv_keymap_erase(const char *path, uint32_t index);
/* Every entry (index ascending) into indices[]/keys[] up to cap; *count = number of entries. */
int hfv_keymap_list(const char *path, uint32_t *indices, struct hop_key *keys, size_t cap, size_t *count);
/* Consistent snapshot of all HFV_MAX_KEYS slots and the 256-bit valid mask. */
int hfv_keymap_read(const char *path, struct hop_key *slots, uint32_t *valid);
/* reusePinnedMap: the ctx reloads its key table from the pinned map whenever the map
 * changed, at the next batch boundary; hfv_key_add/remove on the ctx then write through
 * to the map.  The map is created empty if it does not exist. */
int hfv_ctx_attach_keymap(hfv_ctx *ctx, const char *path);

/* ---- data path ----------------------------------------------------------------------
 * Fused per-packet verify over fixed-layout records: build macinput from the record's
 * InfoField/HopField with the AS-ingress beta rule (path_processing.h:39-81), select the
 * key (keysel), one-block CMAC (aes.h:129-141), 48-bit compare (xdp.c:89-90).
 * recs: n records of `stride` bytes (8-byte aligned, stride % 8 == 0). */
int hfv_verify_records(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits,
                       void *stream);
/* One batch of records for the multi-batch calls (hfv_verify_batches, hfv_service_submitv,
 * hfv_service_run): n records of `stride` bytes at recs, verdicts into pass_bits. */
struct hfv_batch {
    const void *recs;
    size_t stride;
    size_t n;
    uint64_t *pass_bits;
};
/* hfv_verify_records over `count` batches in ONE stream-ordered launch (up to 64 batches per
 * launch; more are split): the round tables are written into LDS once for all of them, and
 * the batches' tiles are dealt to the CUs as one contiguous range.  Records written by earlier
 * work on `stream` are read, the bitmaps are complete for later work on it -- the fast path
 * for callers whose batches come from a copy or a parse kernel on a stream (one
 * hfv_verify_records launch per batch pays the table fill and the grid's ramp and tail per
 * batch).  Each batch is checked as hfv_verify_records checks one; empty batches are skipped. */
int hfv_verify_batches(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, void *stream);
/* Same, then waits and stores the launches' execution time (dispatch start of the first to
 * dispatch end of the last) in *kernel_ms.  For benchmarks. */
int hfv_verify_batches_timed(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, void *stream,
                             float *kernel_ms);
/* Verdict counts for the verify-only paths, modelled on record_verdict (xdp.c:54-70) but NOT
 * its layout: counters[slot][0] += packets that verified, counters[slot][1] += packets dropped
 * as VERDICT_INVALID_HF, where slot is the packet's AS-ingress interface (IFID & 0xff,
 * Cons ? HF.ingress : HF.egress, xdp.c:151-157) -- an IFID-keyed approximation with packet
 * counts only; the reference's port_stats_map is keyed by the receiving ifindex and also counts
 * bytes, so these do not compare with it (hfv_br_process's counters do).
 * From the records and the verdict bitmap hfv_verify_records or the service wrote for them.
 * counters: device u64[256][2], added to.  Stream-ordered like hfv_verify_records. */
int hfv_verdict_counters(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, const uint64_t *pass_bits,
                         uint64_t *counters, void *stream);
/* verify_hop_field (xdp.c:77-91) for n prepared inputs: macinput[i] against the 48-bit
 * expected[i] (low 48 bits of the LE u64, as defer_verify_hop_field stores it).
 * key_index: per-packet slot (device u8 array) or NULL for slot 0. */
int hfv_verify_macinputs(hfv_ctx *ctx, const struct macinput *mi, const uint64_t *expected,
                         const uint8_t *key_index, size_t n, uint64_t *pass_bits, void *stream);
/* Parity mode: full 16-byte AES-CMAC tags of n one-block messages (aes_cmac_16bytes).
 * A missing key yields an all-zero tag. */
int hfv_cmac_tags(hfv_ctx *ctx, const struct macinput *mi, const uint8_t *key_index, size_t n,
                  struct aes_cmac *tags, void *stream);
/* Same as hfv_verify_records, then waits for it and stores the kernel's own execution
 * time (start/stop timestamps of the dispatch, hipExtLaunchKernel events) in *kernel_ms.
 * Used by the benchmark to price the kernel against its roofline. */
int hfv_verify_records_timed(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits,
                             void *stream, float *kernel_ms);
/* Host-memory batch (config 5 path): records and bitmap in HOST memory; returns when
 * pass_bits is complete.  From pageable records, host threads (HFV_HOST_THREADS, default
 * min(8, cores)) gather each record's InfoField and HopField (the 20 bytes the verifier
 * reads) into 24-byte pinned staging records, chunk by chunk, with gather / H2D / kernel /
 * D2H overlapped over chunks on two streams; records inside a buffer registered with
 * hfv_host_register (an RX ring) are read by the kernel in place over PCIe (zero-copy),
 * and a registered pass_bits is written in place. */
int hfv_verify_records_host(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits);

/* ---- resident verify service -----------------------------------------------------------
 * The GPU counterpart of the XDP program staying attached to the interface
 * (border_router, xdp.c:250-284, runs for every packet without a per-packet load): one
 * persistent grid per ctx keeps the AES tables (and, for KEYSEL_IFID, the key image)
 * resident in LDS and verifies batches as the host posts them, with the same verdict
 * semantics as hfv_verify_records.  Batches are posted into a 128-entry descriptor ring in
 * pinned host memory; no kernel launch or table fill per batch, and a batch's tail
 * overlaps the next batch's start.  Batches posted before the grid starts (hfv_service_run /
 * run_async, submitv on a stopped service) travel in the launch's kernel arguments (up to 64),
 * so those batches involve no PCIe round trip at all; batches posted to a running grid are
 * fetched by one relay wave, up to 64 per host read, and their completions are forwarded to
 * the ring by the same wave -- the verifying waves never access host memory.
 *   - Key-table, keysel or record-layout changes take effect at the next submit (the
 *     service is restarted there, after the batches already posted: a batch boundary).
 *   - Any other data-path call on the ctx (hfv_verify_records, hfv_br_process, ...) first
 *     stops the service after its posted batches; the next submit starts it again.
 *   - The grid exits by itself after idle_ms without a new batch (default 1000 ms), so a
 *     host that disappears never leaves it running; a later submit restarts it.
 *   - While the service runs it holds every CU's LDS: other kernels on this GPU wait for it
 *     to stop. */
/* Launch the service grid (no-op if running).  idle_ms 0: 1000 ms. */
int hfv_service_start(hfv_ctx *ctx, uint32_t idle_ms);
/* Post one batch (device pointers, as hfv_verify_records; starts the service if needed).
 * Returns its ticket (1, 2, ...) in *ticket.  Blocks only while 128 batches are in flight.
 * Host-ordered, not stream-ordered: the records must be in place and the bitmap must no
 * longer be written by other work when the call is made (synchronize their producers). */
int hfv_service_submit(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits,
                       uint64_t *ticket);
/* Post `count` batches in one call (tickets *first_ticket .. *first_ticket + count - 1), the
 * many-descriptor form of hfv_service_submit (recvmmsg-style: one call per burst of RX
 * batches).  All batches are checked before any is posted. */
int hfv_service_submitv(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket);
/* One-shot run: the batches on a fresh grid (a running service is stopped first), with the
 * stop descriptor posted right behind them, so the grid exits as soon as the last batch is
 * verified; returns when it has (every ticket done) with the grid's lifetime in *kernel_ms
 * (nullable).  For a known set of batches it saves posting and relaying a stop afterwards. */
int hfv_service_run(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket,
                    float *kernel_ms);
/* The same without the wait: returns once the grid is launched with the batches and the stop
 * behind them, so a caller that synchronizes the device (or the tickets) anyway does not wait
 * twice.  The grid exits by itself after the last batch; hfv_service_stop (or any later data-path
 * call) reaps it and reports its lifetime. */
int hfv_service_run_async(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket);
/* Tickets are monotonic over the ctx's life, across service restarts (key changes, idle
 * exits): a ticket of a stopped grid reports done, or -EIO if that grid exited on its idle
 * timeout without verifying it. */
/* 1 if the ticket's verdicts are complete in pass_bits (visible to any stream and to
 * copies), 0 if not yet.  A grid that has exited on the stop a run / run_async posted has
 * verified every batch before it (its completions need not have been forwarded). */
int hfv_service_poll(hfv_ctx *ctx, uint64_t ticket);
/* Wait until the ticket is complete; timeout_ms < 0 waits indefinitely.  -ETIMEDOUT on
 * timeout, -EIO if the service stopped before completing it. */
int hfv_service_wait(hfv_ctx *ctx, uint64_t ticket, int timeout_ms);
/* Finish the posted batches and stop the grid; *kernel_ms (nullable) receives the grid's
 * lifetime (dispatch start/stop events).  -ETIMEDOUT if it had exited on its idle timeout. */
int hfv_service_stop(hfv_ctx *ctx, float *kernel_ms);
int hfv_service_running(const hfv_ctx *ctx);
/* Grids started from now on carry the dispatch start/stop events that hfv_service_stop /
 * hfv_service_run report as the lifetime (1, the default) or not (0: the lifetime reads 0).
 * The events cost the runtime ~12 us per launch-to-synchronize round trip on MI355X (7.5 us of
 * host time in the launch call, profiles/r03/launch_cost/), which a short run can leave out. */
int hfv_service_set_timing(hfv_ctx *ctx, int enable);
/* Service grids started from now on use `blocks` blocks (one per CU at most; 0 = one per CU,
 * the default).  For several processes sharing one GPU, each with its own service: every grid
 * holds the LDS of the CUs it runs on, so grids of cus/ranks blocks run side by side.  Stops
 * a running grid after its posted batches. */
int hfv_service_set_grid(hfv_ctx *ctx, int blocks);

/* ---- key-schedule kernels ------------------------------------------------------------
 * AES-128 key expansion + CMAC K1 on the GPU, one key per lane: device raw keys[n] ->
 * device hop_keys[n] (same bytes as aes_key_expansion + aes_cmac_subkeys). */
int hfv_expand_keys(hfv_ctx *ctx, const struct aes_key *keys, size_t n, struct hop_key *out, void *stream);
/* Bulk install: n raw host keys into slots first..first+n-1, expanded on the GPU. */
int hfv_key_add_batch(hfv_ctx *ctx, uint32_t first, const struct aes_key *keys, size_t n);

/* ---- synthetic traffic ---------------------------------------------------------------
 * Writes n synthetic 64 B SCION records with valid MACs under the
 * ctx's CURRENT key table and keysel (1/16 corrupted), records first_index.. of `seed`'s
 * stream.  stride >= 64, 16-byte aligned. */
int hfv_gen_records(hfv_ctx *ctx, void *recs, size_t stride, size_t n, uint64_t seed, uint64_t first_index,
                    void *stream);

/* ---- full BR per-packet path (config 4) -------------------------------------------------
 * border_router / process_packet (br/src/bpf/xdp.c:54-284) over a batch of Ethernet frames:
 * parse Eth/IPv4|IPv6/UDP/SCION (parser.h), AS ingress/egress processing with deferred HF
 * verification (path_processing.h), next-hop resolution, rewrite with incremental IP/UDP
 * checksums (rewrite.h), HF MAC verification (slot 0 of the ctx key table, xdp.c:259-274),
 * redirect decision and per-ingress-interface verdict counters (record_verdict).
 *
 * The BPF maps become one configuration struct.  bpf_fib_lookup (a kernel helper) is
 * replaced by a static next-hop table with longest-prefix match; an address with no route
 * behaves like BPF_FIB_LKUP_RET_NOT_FWDED.  Addresses and ports are in wire byte order. */
#define HFV_AF_INET 2
#define HFV_AF_INET6 10
#define HFV_BR_MAX_IFACES 16
#define HFV_BR_MAX_ROUTES 64
#define HFV_BR_MAX_TXPORTS 128
#define HFV_BR_COUNTERS 11         /* enum counter (common.h:40-53) */
#define HFV_BR_STATS_IFINDEX 64    /* counters kept for ingress ifindex < 64 */
#define HFV_BR_ACTION_RETRY 0xff   /* internal to the windowed host path; never returned */

struct hfv_br_int_iface {          /* int_iface_map: ifindex -> internal address (common.h:116-128) */
    uint32_t ifindex;
    uint32_t family;
    uint8_t addr[16];              /* IPv4 in addr[0..3] */
    uint8_t port[2];
    uint8_t pad[2];
};
struct hfv_br_ingress {            /* ingress_map: {dst addr, dst port, ifindex} -> AS interface id (common.h:73-84) */
    uint32_t ifindex;
    uint32_t family;
    uint8_t addr[16];
    uint8_t port[2];
    uint8_t pad[2];
    uint32_t ifid;
};
struct hfv_br_egress {             /* egress_map: ifid -> fwd_info (common.h:131-145) */
    uint32_t ifid;
    uint32_t fwd_external;         /* 1: ext_link {remote, local}, 0: sibling BR {remote = its internal address} */
    uint32_t family;
    uint8_t remote[16];
    uint8_t local[16];
    uint8_t remote_port[2];
    uint8_t local_port[2];
};
struct hfv_br_route {              /* replaces bpf_fib_lookup (fib_lookup.h:74-261) */
    uint32_t family;
    uint8_t prefix[16];
    uint32_t prefix_len;
    int32_t ret;                   /* BPF_FIB_LKUP_RET_*: 0 success, 1-3 drop, 4-8 pass */
    uint32_t ifindex;
    uint8_t smac[6];
    uint8_t dmac[6];
};
struct hfv_br_config {
    uint32_t n_int_ifaces, n_ingress, n_egress, n_routes, n_tx_ports;
    struct hfv_br_int_iface int_ifaces[HFV_BR_MAX_IFACES];
    struct hfv_br_ingress ingress[HFV_BR_MAX_IFACES];
    struct hfv_br_egress egress[HFV_BR_MAX_IFACES];
    struct hfv_br_route routes[HFV_BR_MAX_ROUTES];
    uint32_t tx_ports[HFV_BR_MAX_TXPORTS];   /* tx_port_map: ifindices a redirect may target */
};

/* Install the router tables (copied; takes effect for batches enqueued afterwards).  Detaches
 * a pinned config attached with hfv_ctx_attach_brconfig. */
int hfv_br_set_config(hfv_ctx *ctx, const struct hfv_br_config *cfg);
/* The reference's ENABLE_HF_CHECK build switch (br/CMakeLists.txt:8,48-64) as a runtime
 * setting: enable = 0 skips the hop-field MAC check (defer_verify_hop_field and the MAC block
 * of border_router, path_processing.h:43-57 / xdp.c:259-274); default on.  Takes effect
 * for batches enqueued afterwards; survives hfv_br_set_config. */
int hfv_br_set_hf_check(hfv_ctx *ctx, int enable);
/* The reference's other build options (br/CMakeLists.txt:5-7, common.h:31-33), as a runtime
 * switch of the router: HFV_BR_NO_IPV4 / HFV_BR_NO_IPV6 compile that case of parse_underlay out
 * (parser.h:60,81: such frames fall to `default`, VERDICT_NOT_SCION, XDP_PASS), HFV_BR_NO_SCION_PATH
 * the standard SCION path type (parser.h:140: VERDICT_NOT_IMPLEMENTED).  Default 0: all built.
 * -EINVAL (tables unchanged) if the installed tables hold an address of a switched-off family,
 * which br-loader rejects (maps.cpp:68-80 "Border router configuration contains IPv4 address,
 * but IPv4 support is deactivated."); hfv_br_set_config checks the same against the options.
 * "Installed tables" are the ones last set by hfv_br_set_config or last loaded from an attached
 * pinned config (hfv_ctx_attach_brconfig); a republished pinned config carries the options
 * `hfv-loader attach` was given, and those replace the ones set here when it is reloaded. */
#define HFV_BR_NO_IPV4 1u
#define HFV_BR_NO_IPV6 2u
#define HFV_BR_NO_SCION_PATH 4u
int hfv_br_set_build_options(hfv_ctx *ctx, uint32_t disabled);
/* That check alone (for a loader): 0, or -EINVAL with br-loader's message in hfv_last_error(). */
int hfv_br_config_check_options(const struct hfv_br_config *cfg, uint32_t disabled);
/* ---- control plane: br-loader's configuration path ---------------------------------------
 * loadConfig + initializeMaps (br/src/config.cpp:212-262, maps.cpp:91-200, called by attachBr,
 * br_loader.cpp:88-151) for C hosts: the br-loader TOML file (`self`, `topology`,
 * `internal_interfaces`, br/README.md) and the SCION topology.json it names are parsed, each
 * local underlay address is resolved to the interface holding it, and the router tables are
 * built.  The next-hop table replaces bpf_fib_lookup (no kernel FIB on the GPU). */
struct hfv_br_ifaddr {             /* one address of the getifaddrs view (config.cpp:168-204) */
    char ifname[16];
    uint32_t ifindex;
    uint32_t family;               /* HFV_AF_INET / HFV_AF_INET6 */
    uint8_t addr[16];
};
struct hfv_br_next_hop {           /* one static FIB entry */
    uint32_t family;
    uint8_t prefix[16];
    uint32_t prefix_len;
    char ifname[16];
    uint8_t smac[6];
    uint8_t dmac[6];
    int32_t ret;                   /* BPF_FIB_LKUP_RET_*, 0 = forward */
};
/* ifaddrs NULL: this network namespace (getifaddrs + if_nametoindex).  self, listing and diag
 * (each nullable, NUL-terminated, truncated to their length) receive the BR name, the
 * "XDP Border Router ..." listing br-loader prints and br-loader's stderr messages (the error,
 * or the "WARNING: No interface has IP ..." lines).  Returns 0, -EINVAL for a configuration
 * br-loader rejects, -ENOSPC if the tables exceed the fixed capacity. */
int hfv_br_config_load(const char *toml_path, const struct hfv_br_ifaddr *ifaddrs, size_t n_ifaddrs,
                       const struct hfv_br_next_hop *hops, size_t n_hops, struct hfv_br_config *out,
                       char *self, size_t self_len, char *listing, size_t listing_len, char *diag, size_t diag_len);
/* The same with this namespace's interfaces, installed into ctx (hfv_br_set_config). */
int hfv_br_load_config(hfv_ctx *ctx, const char *toml_path, const struct hfv_br_next_hop *hops, size_t n_hops);
/* Pinned router tables, $HFV_PIN_DIR/<br>/br_config: `hfv-loader attach` publishes them (the
 * maps attachBr fills and pins), a data plane attached with hfv_ctx_attach_brconfig reloads
 * them whenever they are republished, at the next batch boundary.  Writers flock; readers see
 * whole tables (seqlock). */
int hfv_brconfig_path(const char *br, char *out, size_t len);
int hfv_brconfig_publish(const char *path, const struct hfv_br_config *cfg);
/* The same with the router's build options (HFV_BR_NO_*), which an attached ctx adopts. */
int hfv_brconfig_publish_opts(const char *path, const struct hfv_br_config *cfg, uint32_t disabled);
int hfv_brconfig_read(const char *path, struct hfv_br_config *cfg);
/* `hfv-loader detach`: marks the pinned tables detached (the file stays, so data planes that
 * attached it see the change): from their next batch an attached ctx passes every frame
 * (action XDP_PASS, verdict 0, egress -1, nothing counted), as the interface does once
 * detachBr removed the XDP program (br_loader.cpp:153-162); a later hfv_brconfig_publish
 * re-attaches.  -ENOENT if the file is missing or already detached.  Publish and read reject
 * tables whose counts exceed the fixed capacity (-EINVAL), and an attached ctx keeps its
 * previous tables (and fails that call) when it finds such a snapshot. */
int hfv_brconfig_detach(const char *path);
int hfv_ctx_attach_brconfig(hfv_ctx *ctx, const char *path);
/* Process n frames in place.  pkts: frame i at pkts + i*slot (slot % 8 == 0, >= 64);
 * len[i] its length (<= slot); ingress_ifindex[i] the receiving interface.  Outputs per
 * frame: action[i] = the XDP action returned (0 aborted, 1 drop, 2 pass, 4 redirect),
 * verdict[i] = the last enum verdict recorded, egress_ifindex[i] = redirect target or -1.
 * stats (nullable): u64 [HFV_BR_STATS_IFINDEX][2][HFV_BR_COUNTERS] (bytes, packets) to which
 * the batch's record_verdict calls are added.  All pointers are device pointers. */
int hfv_br_process(hfv_ctx *ctx, uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex,
                   size_t n, uint8_t *action, uint8_t *verdict, int32_t *egress_ifindex, uint64_t *stats,
                   void *stream);
/* Config 5: frames in HOST memory (an RX ring of `slot`-byte slots).  Chunk by chunk, only
 * the first `window` bytes of each slot cross PCIe (host threads pack them into pinned
 * staging for one linear DMA each way and write the rewritten windows back; a ring
 * registered with hfv_host_register is instead read and written in place by the kernel over
 * PCIe), are processed
 * exactly as hfv_br_process does, and the rewritten window is copied back in place.  Frames
 * whose headers reach past the window are run again with the whole slot, so the result is
 * identical to hfv_br_process on the full frames.  len, ingress_ifindex, action, verdict,
 * egress_ifindex and stats (nullable, added to) are host arrays.  window: multiple of 8 with
 * 64 <= window <= slot, or 0 for 256 (capped at slot).  Synchronous: on return every output
 * is in host memory. */
int hfv_br_process_host(hfv_ctx *ctx, uint8_t *frames, size_t slot, const uint16_t *len,
                        const uint32_t *ingress_ifindex, size_t n, size_t window, uint8_t *action,
                        uint8_t *verdict, int32_t *egress_ifindex, uint64_t *stats);
/* ---- pinned verdict counters ----------------------------------------------------------
 * A file-backed port_stats_map (maps.h; pinned by br_loader.cpp:136-140, read by
 * `br-loader watch`, stats.cpp): $HFV_PIN_DIR/<br>/port_stats_map, same counter layout as the
 * `stats` buffer of hfv_br_process.  The data path adds its counters after a batch;
 * `hfv-loader watch <br> <iface>` prints them with per-second rates. */
int hfv_statsmap_path(const char *br, char *out, size_t len);
int hfv_statsmap_add(const char *path, const uint64_t *stats);   /* creates the map if needed */
int hfv_statsmap_read(const char *path, uint64_t *stats);

/* Page-lock and map an existing host buffer (e.g. the RX ring) for this ctx's GPU (at most 16
 * per ctx).  hfv_br_process_host on frames inside a registered buffer runs zero-copy: the
 * kernel reads the header windows across PCIe itself and writes back only rewritten rows
 * (`window` is then unused); registered len/ifindex/output arrays are used in place. */
int hfv_host_register(hfv_ctx *ctx, void *ptr, size_t bytes);
int hfv_host_unregister(hfv_ctx *ctx, void *ptr);

/* ---- config 5 in one process (br/evaluation/README.md:131-139) --------------------------
 * The reference measures its router with tcpreplay pushing gen_packets.py's frames into a veth
 * pair, the XDP program on the other end, and count_and_drop.py on the TX side.  hfv_loop_run
 * is that loop without the kernel's network stack: producer threads copy the frame list
 * (cycling, like `tcpreplay --loop`) into a registered RX ring of `chunks` x `chunk` slots,
 * the calling thread runs the router over each filled chunk (zero-copy like hfv_br_process_host,
 * or through HBM by DMA), `inflight` chunks at once on their own streams, and consumer
 * threads "transmit" redirected frames (count, bytes, optional digest) and drop the rest.
 * Producers and consumers run on the GPU's NUMA node. */
struct hfv_loop_config {
    const uint8_t *frames;       /* n_frames frames, frame_stride bytes apart */
    const uint16_t *lens;
    size_t n_frames, frame_stride;
    uint32_t rx_ifindex;         /* ingress interface of every frame */
    uint32_t slot;               /* ring slot bytes (multiple of 16, >= 128 and >= every len) */
    size_t chunk, chunks;        /* frames per chunk, chunks in the ring (>= 2) */
    uint64_t total;              /* frames to push through */
    int producers, consumers;    /* threads per side (0: 1) */
    int digest;                  /* 1: sum a 64-bit digest of every transmitted frame + egress */
    int inflight;                /* chunks on the GPU at once, each on its own stream (0: 2) */
    int dma;                     /* 0: the kernel reads/writes the ring over PCIe (zero-copy);
                                    1: each chunk is copied to HBM and back by the DMA engines;
                                    2: copied to HBM by DMA, the kernel writes the bytes it changes
                                       and its outputs straight back into the ring */
    uint64_t *stats;             /* nullable: per-ifindex verdict counters (added to), as hfv_br_process_host */
    /* Packet-socket I/O, the evaluation's veth loop (br/evaluation/veth_setup.bash,
     * README.md:131-139) -- NULL: the in-process frame list above.
     * rx_ifname: producers receive the frames tcpreplay pushes into the peer from an AF_PACKET
     *            socket on this interface (frames/lens/n_frames unused); `total` bounds them,
     *            and after idle_ms (0: 1000) without a frame the loop drains and returns.
     * tx_ifname: consumers send every redirected frame out of an AF_PACKET socket on this
     *            interface (count_and_drop.py counts them on the peer).
     * Needs CAP_NET_RAW; -EPERM (or the socket's errno) otherwise. */
    const char *rx_ifname, *tx_ifname;
    int idle_ms;
};
struct hfv_loop_stats {
    uint64_t rx_pkts, tx_pkts, tx_bytes, drop_pkts;
    uint64_t tx_digest;                         /* sum over transmitted frames (order-free) */
    uint64_t verdict_pkts[HFV_BR_COUNTERS];     /* frames per final verdict counter (verdict >> 3) */
    double seconds;                             /* wall time of the whole loop */
    double gpu_busy_s, gpu_wait_s;              /* router stage: inside hfv_br_process_host / waiting for RX */
    double producer_busy_s, consumer_busy_s;    /* summed over the threads of each side */
    uint64_t rx_truncated, tx_errors;           /* packet I/O: frames longer than a slot (dropped),
                                                   sends that failed after retries */
    int32_t numa_node;                          /* the GPU's NUMA node the threads were pinned to (-1: unknown) */
    uint32_t threads;                           /* producer + consumer threads */
    uint32_t threads_on_node;                   /* ... of which ended their work on a CPU of that node */
    uint32_t pad_;
};
int hfv_loop_run(hfv_ctx *ctx, const struct hfv_loop_config *cfg, struct hfv_loop_stats *out);

/* Same, then waits for the launch and returns its execution time (start/stop of the kernel
 * dispatch itself) in *kernel_ms.  For benchmarks. */
int hfv_br_process_timed(hfv_ctx *ctx, uint8_t *pkts, size_t slot, const uint16_t *len,
                         const uint32_t *ingress_ifindex, size_t n, uint8_t *action, uint8_t *verdict,
                         int32_t *egress_ifindex, uint64_t *stats, void *stream, float *kernel_ms);

/* ---- host helpers ---------------------------------------------------------------------- */
/* Scalar verify_hop_field on the host (SURVEY.md 8b v) for control-plane checks. */
int hfv_verify_macinput(const struct macinput *mi, uint64_t expected, const struct hop_key *key);
/* Base64 key decode with the reference's rules (exactly 24 chars, last two dropped). */
int hfv_decode_key_b64(const char *base64, struct aes_key *key);
/* Device memory helpers for C hosts without a framework allocator. */
int hfv_dev_alloc(hfv_ctx *ctx, size_t bytes, void **ptr);
int hfv_dev_free(hfv_ctx *ctx, void *ptr);
int hfv_memcpy_h2d(hfv_ctx *ctx, void *dst, const void *src, size_t bytes);
int hfv_memcpy_d2h(hfv_ctx *ctx, void *dst, const void *src, size_t bytes);
/* Writes a one-line description of the kernel variants the ctx launches. */
int hfv_ctx_describe(const hfv_ctx *ctx, char *buf, size_t len);
const char *hfv_last_error(void);
int hfv_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
