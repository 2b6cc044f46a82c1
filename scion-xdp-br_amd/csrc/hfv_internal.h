// hfv_internal.h -- shared between the host API (hfv_api.cpp, hfv_aes_host.cpp) and the
// kernel launchers (hfv_kernels.hip).  Not installed.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/scion_hfv.h"
#include "hfv_tables.h"

namespace hfv {

// error reporting (thread-local message, negative errno return)
int fail(int code, const char *fmt, ...);

// host AES (hfv_aes_host.cpp)
void expand_key(const uint8_t key[16], uint32_t w[44]);
void encrypt_block(const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]);
void hop_key_from_key(const uint8_t key[16], hop_key *hk);
void compile_dev_key(const hop_key *hk, uint32_t dk[4 * kDevKeyRows]);

// Device key table as the kernels see it: dev keys in round-major order
// [kDevKeyRows][HFV_MAX_KEYS] x 16 B, the 256-bit valid bitmap, then the key-schedule words of
// rounds 3..10 per slot for the per-interface-key kernels (config 3): sched[0][k] = t3..t6,
// sched[1][k] = t7..t10, t_r = SubWord(RotWord(w_{4r-1})) ^ Rcon_r = w_{4r} ^ w_{4r-4}
// (aes.c:120-137), so that round key r follows from round key r - 1 by XOR alone.
struct DevKeyTable {
    uint32_t rows[kDevKeyRows][HFV_MAX_KEYS][4];
    uint32_t valid[8];
    uint32_t pad_[24];
    uint32_t sched[2][HFV_MAX_KEYS][4];
};
static_assert(offsetof(DevKeyTable, sched) % 128 == 0, "schedule rows on 128 B boundaries");
// the schedule words of a hop_key (host side of DevKeyTable::sched)
void compile_dev_sched(const hop_key *hk, uint32_t t[8]);

// Router tables as the config-4 kernel sees them (compiled from struct hfv_br_config by
// hfv_br_set_config).  Addresses/ports keep the BPF code's little-endian view of wire bytes
// ("l32"/"l16" of the raw field) so they drop straight into the rewrite arithmetic; route
// prefixes are big-endian words with a precomputed mask for the longest-prefix match.
struct DevBrIntIface {
    uint32_t ifindex, family;
    uint32_t addr[4];   // l32 of addr[4i..4i+3]
    uint32_t port;      // l16 of port
};
struct DevBrIngress {        // ingress_map key {ipv4, ipv6[4], port, u16 ifindex} (common.h:73-84)
    uint32_t v4, v6[4];      // family INET: v4 = l32(addr), v6 = 0; otherwise v4 = 0, v6 = l32 words
    uint32_t port;           // l16
    uint32_t ifindex16;      // ifindex & 0xffff
    uint32_t ifid;
};
struct DevBrEgress {
    uint32_t ifid, fwd_external, family;
    uint32_t remote[4], local[4];   // l32 words
    uint32_t remote_port, local_port;   // l16
    // resolved at compile time from the static tables (the per-frame lookups' results depend
    // only on the entry): the next-hop route of `remote` (-1: none) and, for a sibling, the
    // internal interface on that route's ifindex (-1: none)
    int32_t route, sib_iface;
};
struct DevBrRoute {
    uint32_t family;    // 0: never matches (prefix length beyond the family's width)
    uint32_t plen;
    uint32_t pfx[4], mask[4];   // big-endian words, pfx pre-masked
    int32_t ret;
    uint32_t ifindex;
    uint32_t dmac_lo, dmac_hi, smac_lo, smac_hi;   // MAC bytes 0-3 / 4-5 as LE words
};
struct DevBrConfig {
    uint32_t n_int, n_ing, n_egr, n_routes;
    uint32_t hf_check_off;   // 1: the ENABLE_HF_CHECK=OFF router (hfv_br_set_hf_check)
    uint32_t detached;       // 1: the attached pinned config was detached -- every frame passes
    uint32_t feat_off;       // HFV_BR_NO_*: the reference build options switched off
    uint32_t pad_[1];
    uint32_t tx_bits[HFV_BR_MAX_TXPORTS / 32];
    DevBrIntIface int_ifaces[HFV_BR_MAX_IFACES];
    DevBrIngress ingress[HFV_BR_MAX_IFACES];
    DevBrEgress egress[HFV_BR_MAX_IFACES];
    DevBrRoute routes[HFV_BR_MAX_ROUTES];
    // direct maps for the common small keys (first match, -1: none): int_iface_map for ingress
    // ifindex < 64, egress_map for IFID < 256; larger keys use the linear searches
    int8_t int_of_ifindex[64];
    int8_t egr_of_ifid[256];
    // ingress_map candidates by ifindex < 64: the one entry on that ifindex (-1: none, -2: several)
    int8_t ing_of_ifindex[64];
};
static_assert(sizeof(DevBrConfig) % 16 == 0, "copied to LDS in 16 B pieces");

// Everything a launch reads from the published device state: the key table (first, so a
// DevState* is also the DevKeyTable* the verify kernels take) and the router tables.
struct DevState {
    DevKeyTable keys;
    DevBrConfig br;
};
void compile_br_config(const hfv_br_config *in, DevBrConfig *out);

enum KernelMode { kModeRecords = 0, kModeMacinputs = 1, kModeTags = 2 };

// Resident verify service (hfv_service_*).  The host posts batch descriptors into a ring in
// pinned, coherent host memory (SvcShared).  Batches posted before the grid starts (every
// hfv_service_run / run_async batch up to kSvcInline, and submitv's first ones) travel in the
// kernel arguments (SvcArgs::inl) and every block caches them in LDS at its start: no PCIe
// round trip stands between the grid and those batches.  Batches posted later are fetched by
// one relay wave of block 0, up to 64 descriptors per host read (read-ahead), into a device
// mirror (SvcDev::mir) that the blocks poll.  Blocks report the completion of their share of
// a batch into device memory (SvcDev::done); the relay forwards a batch's completion to the
// host ring (SvcShared::done) once every block has reported it.  So the compute waves never
// touch host memory, and no wave waits on a PCIe round trip per batch (round 3's relay did a
// seq poll, a field read and a host store per batch on the blocks' critical path: ~42 us per
// batch on a box whose host round trips were slow).  Batch b (0-based, ticket
// b+1) uses ring slot b % kSvcRing; the host posts ticket t only once ticket t - kSvcRing is
// complete, which is what lets each block cache kSvcRing descriptors in LDS without any reuse
// check (hfv_kernels.hip, k_verify_service).  A grid that exits on its stop descriptor has
// verified every batch before it, so the host needs no forwarded completion for those.
constexpr uint32_t kSvcRing = 128;   // batches in flight (a host hiccup of ~1.5 ms at 2^20 records does not starve the grid;
                                     // 128 x 64 B of descriptor cache per block leaves LDS room for config 3's key rows)
constexpr uint32_t kSvcMaxBlocks = 1024;
constexpr uint32_t kSvcInline = 64;  // descriptors in the kernel arguments
constexpr uint64_t kSvcStopN = ~0ull;   // descriptor n: the service exits
struct SvcDesc {
    uint64_t recs, bits, n, stride;   // device pointers / counts of the batch
    uint64_t seq;                     // generation tag | ticket; stored last, with release
    uint64_t pad[3];
};
struct SvcShared {   // pinned host memory
    SvcDesc desc[kSvcRing];
    uint64_t status;                 // nonzero: the grid stopped on its own (kSvcIdleTimeout, kSvcWatchdog)
    uint64_t pad[7];
    uint64_t done[kSvcRing];         // done[(t-1) % kSvcRing] = tag | t: batch t verified (forwarded by the relay)
};
// Relay diagnostics (SvcDev::relay), one grid's worth: how the host link behaved for it.
enum SvcRelayStat {
    kRelayProbeTicks = 0,   // one host-memory read round trip at grid start (100 MHz ticks)
    kRelayReads = 1,        // host ring reads (each covers up to 64 descriptors)
    kRelayReadTicks = 2,    // ... their summed round trips
    kRelayReadMax = 3,      // ... the longest
    kRelayDescs = 4,        // descriptors relayed (batches beyond the inline ones)
    kRelayForwarded = 5,    // batch completions forwarded to the host
    kRelayBlockWaits = 6,   // times a wave waited for a descriptor the relay had not published (SvcArea)
    kRelayInline = 7,       // descriptors the grid got in its kernel arguments
};
// Per-grid scratch that must start at zero: grid number L (launch count) uses area[L & 1] and
// zeroes area[(L + 1) & 1] for the next grid on the same stream, so no memset op has to run
// between the host's post and the grid.
struct SvcArea {
    uint64_t block_waits;         // kRelayBlockWaits
    uint64_t pad[7];
};
struct SvcDev {   // device memory: written by the grid; the host copies what it needs after it
    SvcDesc mir[kSvcRing];           // relayed descriptors
    uint64_t run_clock[4];           // block 0 wave 0 s_memtime/s_memrealtime at loop start, at exit
    uint64_t relay[8];               // SvcRelayStat
    uint64_t load_clock[kSvcRing];   // s_memrealtime when block 0 loaded the slot
    uint64_t relay_clock[kSvcRing];  // s_memrealtime when the relay published the slot
    // work balance (SvcWeights): s_memrealtime when block k finished its table fill, and when it
    // last completed its share of a batch
    uint64_t blk_start[kSvcMaxBlocks];
    uint64_t blk_fin[kSvcMaxBlocks];
    // s_memtime (shader clock) at the same two points: each block's clock over its loop
    uint64_t blk_clk0[kSvcMaxBlocks];
    uint64_t blk_clk1[kSvcMaxBlocks];
    SvcArea area[2];
    uint64_t done[kSvcRing][kSvcMaxBlocks];   // done[(t-1) % kSvcRing][k] = tag | t: block k's share of t is verified
};
constexpr uint64_t kSvcIdleTimeout = 2;
constexpr uint64_t kSvcWatchdog = 3;    // a wave gave up waiting for its block's loader

// Launch geometry of the one-launch-per-batch verify kernels: a persistent grid of one
// 1024-thread block per CU (LDS: the four 32x-replicated round tables, 128 KiB, plus config 3's
// 20 KiB of key rows), fixed at build time; the resident service takes the same shape.
struct LaunchGeom {
    int num_cus;
    int svc_blocks;   // blocks of a service grid: num_cus, or fewer (hfv_service_set_grid)
    // test-only overrides of the router launch (the test build's hfv_debug_br_grid / br_split;
    // always 0 in the product library): blocks per k_br_process launch, frames per split launch
    unsigned br_grid_cap = 0;
    uint64_t br_split_cap = 0;
};

// kernel launchers (hfv_kernels.hip); return hipError_t as int
// interleaved: grid-stride tile order (wave w takes tiles w, w + W, ...) instead of one
// contiguous tile range per block -- for records in host memory, where the 256 ranges far
// apart thrash the GPU's translation of 4 KiB host pages (zero-copy 2^20: 1.60 -> 1.27 ms)
// One-launch-per-batch record verify: the slot-0 key rows and T0 travel in the kernel arguments
// too (RecArgs), so a block's prologue is one memory hop (SvcArgs has the same fields).
struct RecArgs {
    uint32_t key0[kDevKeyRows * 4];
    uint32_t key0_ok, pad_[3];
    uint32_t t0[256];
};
// host_keys: the key table as last published (the host staging image), for RecArgs
int launch_verify_records(const LaunchGeom &g, const DevKeyTable *tab, const DevKeyTable *host_keys, int keysel,
                          const uint8_t *recs,
                          size_t stride, size_t n, uint32_t inf_off, uint32_t hf_off, uint64_t *bits,
                          void *stream, void *ev_start = nullptr, void *ev_stop = nullptr,
                          bool interleaved = false);
int launch_verify_macinputs(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint64_t *expected,
                            const uint8_t *kidx, size_t n, uint64_t *bits, void *stream);
int launch_cmac_tags(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint8_t *kidx, size_t n,
                     void *tags, void *stream);
int launch_expand_keys(const uint8_t *raw, size_t n, hop_key *out, DevKeyTable *tab, uint32_t first_slot,
                       void *stream);
int launch_count_verdicts(const LaunchGeom &g, const uint8_t *recs, size_t stride, size_t n, uint32_t inf_off,
                          uint32_t hf_off, const uint64_t *bits, uint64_t *counters, void *stream);
int launch_gen_records(const LaunchGeom &g, const DevKeyTable *tab, int keysel, uint8_t *recs, size_t stride,
                       size_t n, uint64_t seed, uint64_t first_index, void *stream);
int query_geometry(int device, LaunchGeom *g);
int launch_verify_stamped(const LaunchGeom &g, const DevKeyTable *tab, const DevKeyTable *host_keys, const uint8_t *recs,
                          size_t n,
                          uint64_t *bits, uint64_t *stamps, void *stream);
// persistent verify service (one block of 1024 threads per CU); idle_ticks: 100 MHz ticks a
// block waits for the next descriptor before it exits with status kSvcIdleTimeout
// returns the grid size in *grid
struct SvcDescLite {
    uint64_t recs, bits, n, stride;
};
// Work balance of the resident grid.  The XCDs of one MI355X do not verify at the same rate
// (per-XCD means of the blocks' finish times differ by up to ~12 us over a 0.24 ms grid,
// profiles/r03/svc_span_*.log), and the grid ends with its slowest block.  Block k's share of a
// batch of T tiles is [T*cum(k)/W, T*cum(k+1)/W), W = cum(G), where cum(k) sums the weights of
// blocks 0..k-1: block j weighs w[j % 8] (workgroups go round the 8 XCDs in order), block 0
// (which also runs the relay wave) w0.  Equal weights give the plain T*k/G split.  The host
// re-derives the weights from each block's measured rate after every hfv_service_run grid.
struct SvcWeights {
    uint32_t w[8];
    uint32_t w0;
    uint32_t pad[3];
};
constexpr uint32_t kSvcWeightUnit = 1024;
constexpr uint64_t svc_cum(const SvcWeights &sw, uint64_t k)
{
    if (k == 0) return 0;
    uint64_t all = 0, part = 0;
    for (uint64_t x = 0; x < 8; ++x) {
        all += sw.w[x];
        if (x < k % 8) part += sw.w[x];
    }
    return (k / 8) * all + part - sw.w[0] + sw.w0;
}
// Everything a service grid takes, passed as ONE kernel argument (so the kernel reads the
// inline descriptors straight from the kernarg segment, indexed by batch).
struct SvcArgs {
    const DevKeyTable *tab;
    SvcShared *host;   // device view of the pinned ring
    SvcDev *dev;
    uint32_t inf_off, hf_off;
    uint64_t idle_ticks, tag;
    SvcWeights weights;
    uint32_t n_inline;        // descriptors in inl[] (batches 0 .. n_inline - 1; may end with a stop)
    uint32_t relay_delay_us;  // test hook (hfv_debug_relay_delay): the relay spins this long after each host read
    uint32_t launch;          // grid number (SvcArea parity)
    uint32_t pad_[3];
    // What every block reads before its first tile, in the kernel arguments so that the block
    // prologue is one memory hop (the kernarg segment) instead of two (kernarg -> key table /
    // table image): the slot-0 device key rows (KEYSEL_ZERO, as published for this grid) and T0.
    uint32_t key0[kDevKeyRows * 4];
    uint32_t key0_ok, pad2_[3];
    uint32_t t0[256];
    SvcDescLite inl[kSvcInline];
};
// both travel as one by-value kernel argument: the kernarg segment holds at most 4 KiB
static_assert(sizeof(SvcArgs) <= 4096, "SvcArgs exceeds the 4 KiB kernel-argument segment");
static_assert(sizeof(RecArgs) + 128 <= 4096, "RecArgs and the launch's other arguments exceed 4 KiB");
int launch_verify_service(const LaunchGeom &g, int keysel, const SvcArgs &args, void *stream, void *ev_start,
                          void *ev_stop, unsigned *grid);
// Stream-ordered batch list (hfv_verify_batches): up to kBatchMax batches per launch, their
// descriptors and the running tile count cum[] (batch j = global tiles [cum[j], cum[j+1]),
// cum[nb] = total) in the one by-value kernel argument, beside T0 and the slot-0 key rows.
constexpr uint32_t kBatchMax = 64;
constexpr uint32_t kBatchStampBlocks = 1024;
constexpr size_t kBatchClkWords = 4 + 2 * kBatchStampBlocks;
struct BatchArgs {
    const DevKeyTable *tab;
    uint32_t inf_off, hf_off;
    uint32_t nb, total;       // batches; tiles over all of them (< 2^32: 288 GB of records at stride 8 is 2^29 tiles)
    // nullable (diagnostics): [0..3] block 0's s_memtime / s_memrealtime at its start and at its end
    // (wave 0); [4 + k] block k's s_memrealtime at its entry, [4 + kBatchStampBlocks + k] when its
    // last wave left (atomic max: the host zeroes it before a timed launch)
    uint64_t *clk;
    uint32_t key0[kDevKeyRows * 4];
    uint32_t key0_ok, pad_[3];
    uint32_t t0[256];
    SvcDescLite d[kBatchMax];
    uint32_t cum[kBatchMax + 1];
};
static_assert(sizeof(BatchArgs) <= 4096, "BatchArgs exceeds the 4 KiB kernel-argument segment");
int launch_verify_batches(const LaunchGeom &g, int keysel, const BatchArgs &args, void *stream, void *ev_start,
                          void *ev_stop);
// diagnostic streaming read (hfv_debug_stream_read): nb device buffers, read densely
struct StreamArgs {
    uint32_t nb, pad_;
    uint32_t *sink;
    const void *buf[kBatchMax];
    uint64_t bytes[kBatchMax];
};
int launch_stream_read(const LaunchGeom &g, const StreamArgs &args, void *stream, void *ev_start, void *ev_stop);
// full border-router path (hfv_br_kernel.hip)
// slot: bytes between frames in `pkts`; maxlen: lengths are clamped to it (the caller's
// slot); window: bytes of each frame present (frames needing more get HFV_BR_ACTION_RETRY).
// Diagnostics: one wave spinning for `us` microseconds (s_memrealtime) on `stream`.
int launch_debug_spin(void *stream, uint32_t us);
int launch_br_process(const LaunchGeom &g, const DevState *st, uint8_t *pkts, size_t slot, uint32_t maxlen,
                      uint32_t window, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                      uint8_t *action, uint8_t *verdict, int32_t *egress_ifindex, uint64_t *stats, void *stream,
                      void *ev_start = nullptr, void *ev_stop = nullptr, uint8_t *out = nullptr);

// pinned key map (hfv_keymap.cpp)
int keymap_open_ro(const char *path, const void **mapping);
int keymap_create(const char *path, uint32_t mode);   // empty map (header only) if the file does not exist
// pinned router tables (hfv_config.cpp)
int brcfg_open_ro(const char *path, const void **mapping);
void brcfg_close(const void *mapping);
uint32_t brcfg_seq(const void *mapping);
uint32_t brcfg_snapshot(const void *mapping, hfv_br_config *out, uint32_t *detached, uint32_t *feat_off = nullptr);
int br_config_check(const hfv_br_config *cfg);
void keymap_close(const void *mapping);
uint32_t keymap_seq(const void *mapping);
uint32_t keymap_snapshot(const void *mapping, hop_key *slots, uint32_t valid[8]);

// Router stage for in-library pipelines (hfv_loop.cpp): br_zc_prepare stops a running service
// and makes the ctx's device current; br_dev_launch enqueues hfv_br_process on `stream` (any
// stream of the ctx's device) without waiting, over device-addressable frames and metadata
// (HBM, or the device view of mapped host memory), adding the verdict counters to the device
// array dstats (nullable).  dout (nullable: in place) receives the changed bytes of each frame
// and must already hold the rest of it (the host ring a DMA copy came from).
int br_zc_prepare(hfv_ctx *ctx);
// Test-only host router stage for hfv_loop_run (hfv_debug_loop_host_stage, not in the public
// header): frames of one chunk in place, outputs as the kernel writes them; 0 = ok.
typedef int (*hfv_loop_host_stage_fn)(void *user, uint8_t *frames, size_t slot, const uint16_t *len,
                                      const uint32_t *ingress_ifindex, size_t n, uint8_t *action, uint8_t *verdict,
                                      int32_t *egress_ifindex);
int br_dev_launch(hfv_ctx *ctx, void *stream, uint8_t *dframes, size_t slot, const uint16_t *dlen, const uint32_t *difx,
                  size_t n, uint8_t *dact, uint8_t *dver, int32_t *degr, uint64_t *dstats, uint8_t *dout = nullptr);
// Before destroying a stream that launched with the ctx's tables (after synchronizing it):
// drop it from the table readers the next publish would fence on.
void forget_stream(hfv_ctx *ctx, void *stream);

}  // namespace hfv
