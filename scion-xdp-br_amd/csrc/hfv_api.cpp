// hfv_api.cpp -- the C ABI of libscionhfv.so (include/scion_hfv.h): per-GPU context,
// the mac_key_map-equivalent key table, and the batch entry points.
//
// Key table publication (replaces map updates under RCU, br_loader.cpp:221-222): key
// add/remove edit a host shadow; the next data-path call on any stream copies the shadow
// into the inactive one of two device tables (through a pinned staging image), then
// launches with it.  A device table is rewritten only after the work that last read it
// has completed (tracked with one event per table), so in-flight batches keep a stable
// table.
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "hfv_internal.h"

namespace hfv {

static thread_local char g_err[256];

int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

static int hip_fail(hipError_t e, const char *what)
{
    return fail(-EIO, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_TRY(expr)                                          \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) return hip_fail(e_, #expr);      \
    } while (0)

// Restores the caller's current device on scope exit.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ---- router tables (hfv_br_set_config) -------------------------------------------------
static uint32_t le32(const uint8_t *q) { return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24; }
static uint32_t be32(const uint8_t *q) { return (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | (uint32_t)q[3]; }
static uint32_t le16(const uint8_t *q) { return (uint32_t)q[0] | (uint32_t)q[1] << 8; }

void compile_br_config(const hfv_br_config *in, DevBrConfig *out)
{
    memset(out, 0, sizeof *out);
    out->n_int = in->n_int_ifaces;
    out->n_ing = in->n_ingress;
    out->n_egr = in->n_egress;
    out->n_routes = in->n_routes;
    for (uint32_t i = 0; i < in->n_int_ifaces; ++i) {
        const hfv_br_int_iface &a = in->int_ifaces[i];
        DevBrIntIface &d = out->int_ifaces[i];
        d.ifindex = a.ifindex;
        d.family = a.family;
        for (int w = 0; w < 4; ++w) d.addr[w] = le32(a.addr + 4 * w);
        d.port = le16(a.port);
    }
    for (uint32_t i = 0; i < in->n_ingress; ++i) {   // struct ingress_addr key layout, common.h:73-84
        const hfv_br_ingress &a = in->ingress[i];
        DevBrIngress &d = out->ingress[i];
        if (a.family == HFV_AF_INET) d.v4 = le32(a.addr);
        else
            for (int w = 0; w < 4; ++w) d.v6[w] = le32(a.addr + 4 * w);
        d.port = le16(a.port);
        d.ifindex16 = a.ifindex & 0xffffu;
        d.ifid = a.ifid;
    }
    for (uint32_t i = 0; i < in->n_egress; ++i) {
        const hfv_br_egress &a = in->egress[i];
        DevBrEgress &d = out->egress[i];
        d.ifid = a.ifid;
        d.fwd_external = a.fwd_external;
        d.family = a.family;
        for (int w = 0; w < 4; ++w) {
            d.remote[w] = le32(a.remote + 4 * w);
            d.local[w] = le32(a.local + 4 * w);
        }
        d.remote_port = le16(a.remote_port);
        d.local_port = le16(a.local_port);
    }
    for (uint32_t i = 0; i < in->n_routes; ++i) {
        const hfv_br_route &a = in->routes[i];
        DevBrRoute &d = out->routes[i];
        uint32_t width = a.family == HFV_AF_INET ? 32 : a.family == HFV_AF_INET6 ? 128 : 0;
        d.family = (width && a.prefix_len <= width) ? a.family : 0;
        d.plen = a.prefix_len;
        for (int w = 0; w < 4; ++w) {
            uint32_t lo = 32u * (uint32_t)w, bits = a.prefix_len > lo ? a.prefix_len - lo : 0;
            d.mask[w] = bits >= 32 ? 0xffffffffu : bits ? ~0u << (32 - bits) : 0u;
            d.pfx[w] = be32(a.prefix + 4 * w) & d.mask[w];
        }
        d.ret = a.ret;
        d.ifindex = a.ifindex;
        d.dmac_lo = le32(a.dmac);
        d.dmac_hi = le16(a.dmac + 4);
        d.smac_lo = le32(a.smac);
        d.smac_hi = le16(a.smac + 4);
    }
    for (uint32_t i = 0; i < in->n_tx_ports; ++i)
        if (in->tx_ports[i] < HFV_BR_MAX_TXPORTS) out->tx_bits[in->tx_ports[i] >> 5] |= 1u << (in->tx_ports[i] & 31);
    memset(out->int_of_ifindex, 0xff, sizeof out->int_of_ifindex);
    memset(out->egr_of_ifid, 0xff, sizeof out->egr_of_ifid);
    for (uint32_t i = out->n_int; i-- > 0;)   // reverse: the first match wins
        if (out->int_ifaces[i].ifindex < 64) out->int_of_ifindex[out->int_ifaces[i].ifindex] = (int8_t)i;
    for (uint32_t i = out->n_egr; i-- > 0;)
        if (out->egress[i].ifid < 256) out->egr_of_ifid[out->egress[i].ifid] = (int8_t)i;
    memset(out->ing_of_ifindex, 0xff, sizeof out->ing_of_ifindex);
    for (uint32_t i = 0; i < out->n_ing; ++i) {
        const uint32_t x = out->ingress[i].ifindex16;
        if (x < 64) out->ing_of_ifindex[x] = out->ing_of_ifindex[x] == -1 ? (int8_t)i : (int8_t)-2;
    }
    // egress entries: the route to the link's remote (fib_lookup_as_egress / fib_lookup_egress_br
    // look up the entry's own remote address, fib_lookup.h:29-180) and the sibling's internal
    // interface, with the kernel's longest-prefix rule (ties keep the first route)
    for (uint32_t i = 0; i < out->n_egr; ++i) {
        DevBrEgress &e = out->egress[i];
        int best = -1;
        uint32_t best_len = 0;
        for (uint32_t r = 0; r < out->n_routes; ++r) {
            const DevBrRoute &rt = out->routes[r];
            if (rt.family != e.family) continue;
            uint32_t diff = 0;
            for (int w = 0; w < 4; ++w) diff |= (__builtin_bswap32(e.remote[w]) ^ rt.pfx[w]) & rt.mask[w];   // big-endian words
            if (diff == 0 && (best < 0 || rt.plen > best_len)) {
                best = (int)r;
                best_len = rt.plen;
            }
        }
        e.route = best;
        const uint32_t out_if = best >= 0 ? out->routes[best].ifindex : 0;
        e.sib_iface = -1;
        for (uint32_t k = 0; k < out->n_int; ++k)
            if (out->int_ifaces[k].ifindex == out_if) {
                e.sib_iface = (int)k;
                break;
            }
    }
}

}  // namespace hfv

using namespace hfv;

struct hfv_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    LaunchGeom geom{};
    int keysel = HFV_KEYSEL_ZERO;
    uint32_t inf_off = HFV_REC_INF_OFF, hf_off = HFV_REC_HF_OFF;
    // host shadow of mac_key_map
    hop_key shadow[HFV_MAX_KEYS];
    uint32_t valid[8] = {0};
    bool dirty = true;
    // publication
    DevState *host_img = nullptr;         // pinned staging image
    hipEvent_t img_free = nullptr;        // staging image may be rewritten once this fires
                                          // (= the last publish copy into dev_tab[active] is done)
    bool pub_pending = false;             // img_free not yet seen complete: other streams wait on it
    DevState *dev_tab[2] = {nullptr, nullptr};
    hipStream_t readers[2][8] = {};                // streams that launched with dev_tab[i]
    hipEvent_t reader_ev[2][8] = {};               // caller streams: recorded after each such launch
    int nreaders[2] = {0, 0};
    bool readers_overflow[2] = {false, false};
    int active = 0;
    // host-batch staging (hfv_verify_records_host)
    hipStream_t hstream[2] = {nullptr, nullptr};
    uint8_t *h_pin[2] = {nullptr, nullptr};
    uint8_t *d_rec[2] = {nullptr, nullptr};
    uint64_t *h_bits[2] = {nullptr, nullptr};
    uint64_t *d_bits[2] = {nullptr, nullptr};
    size_t host_chunk = 0;
    // attached pinned key map
    const void *keymap = nullptr;
    uint32_t keymap_seq = 0xffffffffu;
    char keymap_path[4096] = {0};
    // attached pinned router tables (hfv_ctx_attach_brconfig)
    const void *brmap = nullptr;
    uint32_t brmap_seq = 0xffffffffu;
    // dispatch timing (hfv_verify_records_timed)
    hipEvent_t tev[2] = {nullptr, nullptr};
    uint64_t *bat_clk = nullptr;   // device: hfv_verify_batches' block-0 clock stamps (hfv_debug_batches_clock)
    // router tables for hfv_br_process (published with the key table)
    DevBrConfig br{};
    hfv_br_config cfg_src{};   // the tables as installed (checked against the build options)
    // windowed host path (hfv_br_process_host): per-stream device/pinned chunk buffers
    size_t brh_win_cap = 0;               // bytes per frame the device windows hold
    uint8_t *brh_dwin[2] = {nullptr, nullptr};
    uint8_t *brh_dio[2] = {nullptr, nullptr};   // len u16 | ifindex u32 | action u8 | verdict u8 | egress i32
    uint8_t *brh_hio[2] = {nullptr, nullptr};   // pinned twin of brh_dio
    uint8_t *brh_hwin[2] = {nullptr, nullptr};  // pinned twin of brh_dwin (packed header windows)
    uint64_t *brh_dstats = nullptr;
    // host buffers registered with hfv_host_register (mapped: the kernels can address them)
    struct HostRange {
        uint8_t *host;
        size_t bytes;
        uint8_t *dev;
    };
    HostRange hreg[16] = {};
    int nhreg = 0;
    uint8_t *zc_meta = nullptr;   // zero-copy path: device len/ifindex/outputs for unregistered arrays
    size_t zc_cap = 0;
    // resident verify service (hfv_service_*)
    bool svc_running = false;
    int svc_keysel = HFV_KEYSEL_ZERO;
    uint32_t svc_inf_off = 0, svc_hf_off = 0, svc_idle_ms = 0;
    hipStream_t svc_stream = nullptr;
    SvcShared *svc_host = nullptr;   // descriptor ring + completions, coherent pinned memory
    SvcShared *svc_host_dev = nullptr;
    SvcDev *svc_dev = nullptr;       // device side: relayed descriptors, block completions, diagnostics
    uint32_t svc_launches = 0;       // grids launched (SvcArea parity)
    unsigned svc_grid = 0;           // blocks of the running grid (each reports its share)
    uint64_t svc_next = 1;           // next grid-local batch number (1, 2, ... per grid)
    uint64_t svc_base = 1;           // ticket of the running grid's batch 1 (tickets are monotonic per ctx)
    uint64_t svc_ticket = 1;         // next ticket
    std::vector<uint64_t> svc_lost;  // tickets of stopped grids that were never verified (bounded)
    uint64_t svc_tag = 0;            // generation of the running grid << 40 (see s_svc_tag)
    bool svc_stop_posted = false;    // the running grid's stop descriptor is already in the ring
    bool svc_timing = true;          // launch grids with dispatch start/stop events (hfv_service_set_timing)
    bool svc_timed = false;          // ... the running / last grid was
    hipEvent_t svc_ev[2] = {nullptr, nullptr};
    // work balance across the grid's blocks (SvcWeights, svc_balance)
    SvcWeights svc_w = {{kSvcWeightUnit, kSvcWeightUnit, kSvcWeightUnit, kSvcWeightUnit, kSvcWeightUnit,
                         kSvcWeightUnit, kSvcWeightUnit, kSvcWeightUnit},
                        kSvcWeightUnit, {0, 0, 0}};
    SvcWeights svc_w_used = svc_w;   // the running / last grid's
    bool svc_adapt = false;          // the running grid got all its batches up front (svc_run): measure it
    std::vector<uint64_t> svc_run_ns;   // ... their record counts
    uint64_t svc_call_ns[6] = {0, 0, 0, 0, 0, 0};   // hfv_debug_service_call_ns: the last svc_run's phases
};

static int device_numa(int device, cpu_set_t *cpus);
static void note_numa(int device);

// Any other data-path call on the ctx first stops a running service (after the batches
// already posted): its grid holds every CU's LDS, so other kernels could not start until
// it exits, and a call that waits for its own kernel would wait for the idle timeout.
static int svc_quiesce(hfv_ctx *ctx);
#define SVC_QUIESCE(ctx)                         \
    do {                                         \
        int q_ = svc_quiesce(ctx);               \
        if (q_) return q_;                       \
    } while (0)

// NULL is HIP's default stream, as for any HIP API taking a stream.
static hipStream_t pick_stream(hfv_ctx *, void *stream) { return (hipStream_t)stream; }

// Streams that launched with each device table since it was last published.  Before a
// table is rewritten, the publishing stream waits for an event recorded on each of them, so
// no per-launch event is needed on the hot path.
static void note_reader(hfv_ctx *ctx, hipStream_t st);
static bool own_stream(const hfv_ctx *ctx, hipStream_t st);

// HFV_PUB_FENCE=0 builds the round-2 behaviour (no cross-stream wait for a publish copy) for the
// A/B that names the loop failure's cause (`make nofence`); never a product build.
#ifndef HFV_PUB_FENCE
#define HFV_PUB_FENCE 1
#endif

// Test hooks.  They change what the library does (delays, launch shapes) and exist only in the
// test build, lib/libscionhfv_test.so (make: -DHFV_TEST_HOOKS); the product library has none of
// them (tests/test_abi.py checks the exports).  The GPU tests that need one run in a child process
// on the test build (tests/conftest.py: rerun_on_test_build).
#ifdef HFV_TEST_HOOKS
// hfv_debug_publish_delay: every publish copy waits behind a spin of this many microseconds on
// its stream, so a test can make the cross-stream race deterministic.
static uint32_t g_pub_delay_us = 0;
extern "C" int hfv_debug_publish_delay(uint32_t us)
{
    g_pub_delay_us = us;
    return 0;
}
// hfv_debug_br_grid: blocks per k_br_process launch (0 = one block per CU up to the tile count).
// With 1, a 1000-frame chunk runs as 16 active waves of one block -- the shape the round-2 loop
// failure ran in ("loop parity failure").
static unsigned g_br_grid = 0;
extern "C" int hfv_debug_br_grid(unsigned blocks)
{
    g_br_grid = blocks;
    return 0;
}
// hfv_debug_br_split: split launches that count verdicts into pieces of at most `frames` frames
// (0 = only where 32-bit block counters could overflow), so a test can check that split launches
// add up to the same counters and outputs.
static size_t g_br_split = 0;
extern "C" int hfv_debug_br_split(size_t frames)
{
    g_br_split = frames;
    return 0;
}
static LaunchGeom br_geom(const hfv_ctx *ctx)
{
    LaunchGeom g = ctx->geom;
    g.br_grid_cap = g_br_grid;
    g.br_split_cap = g_br_split;
    return g;
}
#else
static constexpr uint32_t g_pub_delay_us = 0;
#define br_geom(ctx) ((ctx)->geom)
#endif

// Make the shadow table visible to work enqueued next on `st` -- and, once the copy is queued,
// to work on any other stream (which waits for the copy until it has been seen complete);
// returns the table to use.
static int publish_keys(hfv_ctx *ctx, hipStream_t st, DevState **out)
{
    if (ctx->keymap) {   // pick up updates other processes made to the pinned map
        uint32_t seq = keymap_seq(ctx->keymap);
        if (seq != ctx->keymap_seq) {
            ctx->keymap_seq = keymap_snapshot(ctx->keymap, ctx->shadow, ctx->valid);
            ctx->dirty = true;
        }
    }
    if (ctx->brmap) {    // router tables republished by `hfv-loader attach`
        uint32_t seq = brcfg_seq(ctx->brmap);
        if (seq != ctx->brmap_seq) {
            hfv_br_config cfg;
            uint32_t detached = 0, feat_off = 0;
            ctx->brmap_seq = brcfg_snapshot(ctx->brmap, &cfg, &detached, &feat_off);
            if (br_config_check(&cfg) != 0)   // a corrupt or foreign file: keep the tables in use
                return fail(-EINVAL, "attached router config holds counts past the fixed capacity; "
                                     "previous tables kept");
            const uint32_t off = ctx->br.hf_check_off;
            ctx->cfg_src = cfg;   // what hfv_br_set_build_options checks against
            compile_br_config(&cfg, &ctx->br);
            ctx->br.hf_check_off = off;
            ctx->br.detached = detached;
            ctx->br.feat_off = feat_off & (HFV_BR_NO_IPV4 | HFV_BR_NO_IPV6 | HFV_BR_NO_SCION_PATH);
            ctx->dirty = true;
        }
    }
    if (ctx->dirty) {
        int next = ctx->active ^ 1;
        // wait (host) until the previous copy out of the staging image has been consumed
        HIP_TRY(hipEventSynchronize(ctx->img_free));
        for (uint32_t k = 0; k < HFV_MAX_KEYS; ++k) {
            uint32_t dk[4 * kDevKeyRows], t[8];
            if ((ctx->valid[k >> 5] >> (k & 31)) & 1u) {
                compile_dev_key(&ctx->shadow[k], dk);
                compile_dev_sched(&ctx->shadow[k], t);
            } else {
                memset(dk, 0, sizeof dk);
                memset(t, 0, sizeof t);
            }
            for (int r = 0; r < kDevKeyRows; ++r) memcpy(ctx->host_img->keys.rows[r][k], dk + 4 * r, 16);
            memcpy(ctx->host_img->keys.sched[0][k], t, 16);
            memcpy(ctx->host_img->keys.sched[1][k], t + 4, 16);
        }
        memcpy(ctx->host_img->keys.valid, ctx->valid, sizeof ctx->valid);
        ctx->host_img->br = ctx->br;
        // the device table may only be overwritten after every launch that read it completed
        if (ctx->readers_overflow[next]) {
            HIP_TRY(hipDeviceSynchronize());
        } else {
            // the events were recorded after each reader's last launch with the table, so the
            // fence holds even for a reader stream the caller has destroyed since
            for (int r = 0; r < ctx->nreaders[next]; ++r) {
                hipStream_t rs = ctx->readers[next][r];
                if (rs == st) continue;   // same stream: ordered already
                // the ctx's own streams live as long as the ctx: mark them now; a caller's
                // stream carries the event recorded after its last launch with the table
                if (own_stream(ctx, rs)) HIP_TRY(hipEventRecord(ctx->reader_ev[next][r], rs));
                HIP_TRY(hipStreamWaitEvent(st, ctx->reader_ev[next][r], 0));
            }
        }
        ctx->nreaders[next] = 0;
        ctx->readers_overflow[next] = false;
        if (g_pub_delay_us) HIP_TRY((hipError_t)launch_debug_spin(st, g_pub_delay_us));
        HIP_TRY(hipMemcpyAsync(ctx->dev_tab[next], ctx->host_img, sizeof(DevState), hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(ctx->img_free, st));
        ctx->active = next;
        ctx->dirty = false;
        ctx->pub_pending = true;
    } else if (HFV_PUB_FENCE && ctx->pub_pending) {
        // The copy into dev_tab[active] was enqueued on the stream that published it; work on any
        // other stream must not read the table before that copy lands.  (Round 2 skipped this: the
        // config-5 loop published on its chunk-0 stream and launched chunk 1 on a second stream,
        // whose kernel could read the half-written or previous table -- every MAC of that chunk
        // failed against a stale key, gpurun_out/r02c5: tx short by exactly one chunk.)
        if (hipEventQuery(ctx->img_free) == hipSuccess) ctx->pub_pending = false;
        else HIP_TRY(hipStreamWaitEvent(st, ctx->img_free, 0));
    }
    *out = ctx->dev_tab[ctx->active];
    return 0;
}

static bool own_stream(const hfv_ctx *ctx, hipStream_t st)
{
    return st && (st == ctx->stream || st == ctx->svc_stream || st == ctx->hstream[0] || st == ctx->hstream[1]);
}

static void note_reader(hfv_ctx *ctx, hipStream_t st)
{
    const int a = ctx->active;
    int r = 0;
    while (r < ctx->nreaders[a] && ctx->readers[a][r] != st) ++r;
    if (r == ctx->nreaders[a]) {
        if (r == 8) {
            ctx->readers_overflow[a] = true;
            return;
        }
        ctx->readers[a][ctx->nreaders[a]++] = st;
    }
    // a caller's stream may be destroyed before the next publish: remember where its launches
    // with this table end (one event record per launch; the ctx's own streams skip it)
    if (!own_stream(ctx, st) && hipEventRecord(ctx->reader_ev[a][r], st) != hipSuccess) ctx->readers_overflow[a] = true;
}

static int after_launch(hfv_ctx *ctx, hipStream_t st, int err, const char *what)
{
    if (err != hipSuccess) return hip_fail((hipError_t)err, what);
    note_reader(ctx, st);
    return 0;
}

extern "C" {

const char *hfv_last_error(void) { return g_err; }
int hfv_abi_version(void) { return HFV_ABI_VERSION; }

int hfv_ctx_create(int device, hfv_ctx **out)
{
    if (!out) return fail(-EINVAL, "out is NULL");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(-ENODEV, "no HIP device available");
    if (device < 0 || device >= count) return fail(-ENODEV, "device %d out of range (%d devices)", device, count);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(-ENODEV, "device %d is %s; libscionhfv is built for gfx950 only", device, prop.gcnArchName);
    DeviceGuard g(device);
    hfv_ctx *c = new (std::nothrow) hfv_ctx();
    if (!c) return fail(-ENOMEM, "ctx allocation");
    c->device = device;
    int rc = 0;
    do {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { rc = -EIO; break; }
        if (hipHostMalloc((void **)&c->host_img, sizeof(DevState), hipHostMallocDefault) != hipSuccess) { rc = -ENOMEM; break; }
        if (hipEventCreateWithFlags(&c->img_free, hipEventDisableTiming) != hipSuccess) { rc = -EIO; break; }
        for (int i = 0; i < 2; ++i) {
            if (hipMalloc((void **)&c->dev_tab[i], sizeof(DevState)) != hipSuccess) { rc = -ENOMEM; break; }
            if (hipMemset(c->dev_tab[i], 0, sizeof(DevState)) != hipSuccess) { rc = -EIO; break; }
            for (int r = 0; r < 8 && !rc; ++r)
                if (hipEventCreateWithFlags(&c->reader_ev[i][r], hipEventDisableTiming) != hipSuccess) rc = -EIO;
        }
        if (rc) break;
        if (hipMalloc((void **)&c->bat_clk, kBatchClkWords * sizeof(uint64_t)) != hipSuccess) { rc = -ENOMEM; break; }
        if (hipMemset(c->bat_clk, 0, kBatchClkWords * sizeof(uint64_t)) != hipSuccess) { rc = -EIO; break; }
        if (query_geometry(device, &c->geom) != 0) {
            hfv_ctx_destroy(c);
            return fail(-EINVAL, "device %d cannot hold a 1024-thread verify block with 156 KiB of LDS", device);
        }
    } while (0);
    if (rc) {
        hfv_ctx_destroy(c);
        return fail(rc, "hfv_ctx_create failed on device %d", device);
    }
    memset(c->shadow, 0, sizeof c->shadow);
    note_numa(device);
    *out = c;
    return 0;
}

int hfv_ctx_destroy(hfv_ctx *ctx)
{
    if (!ctx) return 0;
    DeviceGuard g(ctx->device);
    (void)svc_quiesce(ctx);
    if (ctx->svc_stream) {
        (void)hipStreamSynchronize(ctx->svc_stream);
        (void)hipStreamDestroy(ctx->svc_stream);
    }
    if (ctx->svc_host) (void)hipHostFree(ctx->svc_host);
    if (ctx->svc_dev) (void)hipFree(ctx->svc_dev);
    for (int i = 0; i < 2; ++i)
        if (ctx->svc_ev[i]) (void)hipEventDestroy(ctx->svc_ev[i]);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int i = 0; i < 2; ++i) {
        if (ctx->hstream[i]) { (void)hipStreamSynchronize(ctx->hstream[i]); (void)hipStreamDestroy(ctx->hstream[i]); }
        if (ctx->h_pin[i]) (void)hipHostFree(ctx->h_pin[i]);
        if (ctx->h_bits[i]) (void)hipHostFree(ctx->h_bits[i]);
        if (ctx->d_rec[i]) (void)hipFree(ctx->d_rec[i]);
        if (ctx->d_bits[i]) (void)hipFree(ctx->d_bits[i]);
        for (int r = 0; r < 8; ++r)
            if (ctx->reader_ev[i][r]) (void)hipEventDestroy(ctx->reader_ev[i][r]);
        if (ctx->dev_tab[i]) (void)hipFree(ctx->dev_tab[i]);
    }
    for (int i = 0; i < 2; ++i) {
        if (ctx->brh_dwin[i]) (void)hipFree(ctx->brh_dwin[i]);
        if (ctx->brh_hwin[i]) (void)hipHostFree(ctx->brh_hwin[i]);
        if (ctx->brh_dio[i]) (void)hipFree(ctx->brh_dio[i]);
        if (ctx->brh_hio[i]) (void)hipHostFree(ctx->brh_hio[i]);
    }
    if (ctx->brh_dstats) (void)hipFree(ctx->brh_dstats);
    if (ctx->zc_meta) (void)hipFree(ctx->zc_meta);
    if (ctx->bat_clk) (void)hipFree(ctx->bat_clk);
    keymap_close(ctx->keymap);
    brcfg_close(ctx->brmap);
    for (int i = 0; i < 2; ++i)
        if (ctx->tev[i]) (void)hipEventDestroy(ctx->tev[i]);
    if (ctx->img_free) { (void)hipEventSynchronize(ctx->img_free); (void)hipEventDestroy(ctx->img_free); }
    if (ctx->host_img) (void)hipHostFree(ctx->host_img);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return 0;
}

int hfv_ctx_device(const hfv_ctx *ctx) { return ctx ? ctx->device : -1; }
int hfv_ctx_numa_node(const hfv_ctx *ctx) { return ctx ? device_numa(ctx->device, nullptr) : -1; }
void *hfv_ctx_stream(hfv_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int hfv_ctx_set_keysel(hfv_ctx *ctx, int keysel)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (keysel != HFV_KEYSEL_ZERO && keysel != HFV_KEYSEL_IFID) return fail(-EINVAL, "unknown keysel %d", keysel);
    ctx->keysel = keysel;
    return 0;
}

int hfv_ctx_set_record_layout(hfv_ctx *ctx, uint32_t inf_off, uint32_t hf_off)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if ((inf_off & 7) || (hf_off & 7)) return fail(-EINVAL, "INF/HF offsets must be multiples of 8");
    ctx->inf_off = inf_off;
    ctx->hf_off = hf_off;
    return 0;
}

int hfv_ctx_synchronize(hfv_ctx *ctx)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

// ---- key table ------------------------------------------------------------------------

int hfv_key_set_hop_key(hfv_ctx *ctx, uint32_t index, const struct hop_key *hk)
{
    if (!ctx || !hk) return fail(-EINVAL, "null argument");
    if (index >= HFV_MAX_KEYS) return fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    if (ctx->keymap) {
        int rc = hfv_keymap_update(ctx->keymap_path, index, hk);
        if (rc) return rc;
    }
    ctx->shadow[index] = *hk;
    ctx->valid[index >> 5] |= 1u << (index & 31);
    ctx->dirty = true;
    return 0;
}

int hfv_key_add(hfv_ctx *ctx, uint32_t index, const struct aes_key *key)
{
    if (!ctx || !key) return fail(-EINVAL, "null argument");
    hop_key hk;
    hop_key_from_key(key->b, &hk);   // aes_key_expansion + aes_cmac_subkeys, K1 kept
    return hfv_key_set_hop_key(ctx, index, &hk);
}

int hfv_key_add_b64(hfv_ctx *ctx, uint32_t index, const char *base64)
{
    struct aes_key k;
    int rc = hfv_decode_key_b64(base64, &k);
    if (rc) return rc;
    return hfv_key_add(ctx, index, &k);
}

int hfv_key_remove(hfv_ctx *ctx, uint32_t index)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (index >= HFV_MAX_KEYS) return fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    if (!((ctx->valid[index >> 5] >> (index & 31)) & 1u)) return fail(-ENOENT, "key slot %u is empty", index);
    if (ctx->keymap) {
        int rc = hfv_keymap_erase(ctx->keymap_path, index);
        if (rc) return rc;
    }
    ctx->valid[index >> 5] &= ~(1u << (index & 31));
    memset(&ctx->shadow[index], 0, sizeof(hop_key));
    ctx->dirty = true;
    return 0;
}

int hfv_ctx_attach_keymap(hfv_ctx *ctx, const char *path)
{
    if (!ctx || !path) return fail(-EINVAL, "null argument");
    if (strlen(path) >= sizeof ctx->keymap_path) return fail(-ENAMETOOLONG, "path too long");
    const void *m = nullptr;
    int rc = keymap_open_ro(path, &m);
    if (rc == -ENOENT) {   // create an empty pinned map, as attachBr creates mac_key_map
        rc = keymap_create(path, HFV_KEYMAP_SLOTS);   // header only: never touches a slot another process may write
        if (!rc) rc = keymap_open_ro(path, &m);
    }
    if (rc) return fail(rc, "cannot attach key map %s", path);
    keymap_close(ctx->keymap);
    ctx->keymap = m;
    strcpy(ctx->keymap_path, path);
    ctx->keymap_seq = keymap_snapshot(m, ctx->shadow, ctx->valid);
    ctx->dirty = true;
    return 0;
}

int hfv_key_get(hfv_ctx *ctx, uint32_t index, struct hop_key *out)
{
    if (!ctx || !out) return fail(-EINVAL, "null argument");
    if (index >= HFV_MAX_KEYS) return fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    if (!((ctx->valid[index >> 5] >> (index & 31)) & 1u)) return fail(-ENOENT, "key slot %u is empty", index);
    *out = ctx->shadow[index];
    return 0;
}

int hfv_key_add_batch(hfv_ctx *ctx, uint32_t first, const struct aes_key *keys, size_t n)
{
    if (!ctx || (!keys && n)) return fail(-EINVAL, "null argument");
    if ((size_t)first + n > HFV_MAX_KEYS) return fail(-EINVAL, "slots %u..%zu exceed %d", first, first + n, HFV_MAX_KEYS);
    if (n == 0) return 0;
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    uint8_t *d_raw = nullptr;
    hop_key *d_hk = nullptr;
    HIP_TRY(hipMalloc((void **)&d_raw, 16 * n));
    if (hipMalloc((void **)&d_hk, sizeof(hop_key) * n) != hipSuccess) {
        (void)hipFree(d_raw);
        return fail(-ENOMEM, "hipMalloc");
    }
    int rc = 0;
    if (hipMemcpyAsync(d_raw, keys, 16 * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) rc = -EIO;
    if (!rc && launch_expand_keys(d_raw, n, d_hk, nullptr, 0, ctx->stream) != 0) rc = -EIO;
    hop_key *tmp = (hop_key *)malloc(sizeof(hop_key) * n);
    if (!tmp) rc = -ENOMEM;
    if (!rc && hipMemcpyAsync(tmp, d_hk, sizeof(hop_key) * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) rc = -EIO;
    if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = -EIO;
    if (rc) rc = fail(rc, "device key expansion failed");
    for (size_t i = 0; !rc && i < n; ++i) rc = hfv_key_set_hop_key(ctx, first + (uint32_t)i, &tmp[i]);   // first error wins
    free(tmp);
    (void)hipFree(d_raw);
    (void)hipFree(d_hk);
    return rc;
}

// ---- data path ------------------------------------------------------------------------

int hfv_verify_records(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits, void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!recs || !pass_bits) return fail(-EINVAL, "null buffer");
    if (((uintptr_t)recs & 7) || (stride & 7) || ((uintptr_t)pass_bits & 7))
        return fail(-EINVAL, "records, stride and bitmap must be 8-byte aligned");
    if (stride < (size_t)ctx->inf_off + 8 || stride < (size_t)ctx->hf_off + 12)
        return fail(-EINVAL, "stride %zu too small for INF@%u/HF@%u", stride, ctx->inf_off, ctx->hf_off);
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    const DevKeyTable *tab = &ds->keys;
    int e = launch_verify_records(ctx->geom, tab, &ctx->host_img->keys, ctx->keysel, (const uint8_t *)recs, stride, n, ctx->inf_off,
                                  ctx->hf_off, pass_bits, st);
    return after_launch(ctx, st, e, "verify_records launch");
}

int hfv_verify_records_timed(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits,
                             void *stream, float *kernel_ms)
{
    if (!ctx || !kernel_ms) return fail(-EINVAL, "null argument");
    *kernel_ms = 0.0f;
    if (n == 0) return 0;
    if (!recs || !pass_bits) return fail(-EINVAL, "null buffer");
    if (((uintptr_t)recs & 7) || (stride & 7) || ((uintptr_t)pass_bits & 7))
        return fail(-EINVAL, "records, stride and bitmap must be 8-byte aligned");
    if (stride < (size_t)ctx->inf_off + 8 || stride < (size_t)ctx->hf_off + 12)
        return fail(-EINVAL, "stride %zu too small for INF@%u/HF@%u", stride, ctx->inf_off, ctx->hf_off);
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    for (int i = 0; i < 2; ++i)
        if (!ctx->tev[i]) HIP_TRY(hipEventCreate(&ctx->tev[i]));
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    const DevKeyTable *tab = &ds->keys;
    int e = launch_verify_records(ctx->geom, tab, &ctx->host_img->keys, ctx->keysel, (const uint8_t *)recs, stride, n, ctx->inf_off,
                                  ctx->hf_off, pass_bits, st, ctx->tev[0], ctx->tev[1]);
    rc = after_launch(ctx, st, e, "verify_records launch");
    if (rc) return rc;
    HIP_TRY(hipEventSynchronize(ctx->tev[1]));
    HIP_TRY(hipEventElapsedTime(kernel_ms, ctx->tev[0], ctx->tev[1]));
    return 0;
}

// The batch list of hfv_verify_batches: checked as hfv_verify_records checks one batch; empty
// batches are dropped.
static int batches_check(const hfv_ctx *ctx, const struct hfv_batch *b, size_t count)
{
    if (!b && count) return fail(-EINVAL, "null batch list");
    for (size_t i = 0; i < count; ++i) {
        if (b[i].n == 0) continue;
        if (!b[i].recs || !b[i].pass_bits) return fail(-EINVAL, "batch %zu: null buffer", i);
        if (((uintptr_t)b[i].recs & 7) || (b[i].stride & 7) || ((uintptr_t)b[i].pass_bits & 7))
            return fail(-EINVAL, "batch %zu: records, stride and bitmap must be 8-byte aligned", i);
        if (b[i].stride < (size_t)ctx->inf_off + 8 || b[i].stride < (size_t)ctx->hf_off + 12)
            return fail(-EINVAL, "batch %zu: stride %zu too small for INF@%u/HF@%u", i, b[i].stride, ctx->inf_off,
                        ctx->hf_off);
        if (b[i].stride > (1u << 24)) return fail(-EINVAL, "batch %zu: stride %zu > 16 MiB", i, b[i].stride);
        if (b[i].n > ((size_t)1 << 36)) return fail(-EINVAL, "batch %zu: %zu records (at most 2^36)", i, b[i].n);
    }
    return 0;
}

// One launch per kBatchMax non-empty batches (and at most 2^31 tiles); ev0/ev1 (nullable) bracket
// the first and the last launch.
static int batches_launch(hfv_ctx *ctx, const struct hfv_batch *b, size_t count, hipStream_t st, hipEvent_t ev0,
                          hipEvent_t ev1)
{
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    BatchArgs a;
    memset(&a, 0, sizeof a);
    a.tab = &ds->keys;
    a.inf_off = ctx->inf_off;
    a.hf_off = ctx->hf_off;
    a.clk = ctx->bat_clk;
    for (int r = 0; r < kDevKeyRows; ++r) memcpy(&a.key0[4 * r], ctx->host_img->keys.rows[r][0], 16);
    a.key0_ok = ctx->host_img->keys.valid[0] & 1u;
    memcpy(a.t0, kTables.t0, sizeof a.t0);
    size_t last = count;   // the last non-empty batch: its launch records ev1
    while (last > 0 && b[last - 1].n == 0) --last;
    bool first = true;
    for (size_t i = 0; i < last;) {
        a.nb = 0;
        uint64_t tiles = 0;
        for (; i < last && a.nb < kBatchMax; ++i) {
            if (b[i].n == 0) continue;
            const uint64_t t = (b[i].n + 63) / 64;
            if (a.nb && tiles + t > (1ull << 31)) break;
            a.d[a.nb] = {(uint64_t)(uintptr_t)b[i].recs, (uint64_t)(uintptr_t)b[i].pass_bits, (uint64_t)b[i].n,
                         (uint64_t)b[i].stride};
            a.cum[a.nb] = (uint32_t)tiles;
            tiles += t;
            ++a.nb;
        }
        a.cum[a.nb] = (uint32_t)tiles;
        a.total = (uint32_t)tiles;
        const bool fin = i >= last;
        int e = launch_verify_batches(ctx->geom, ctx->keysel, a, st, first ? ev0 : nullptr, fin ? ev1 : nullptr);
        rc = after_launch(ctx, st, e, "verify_batches launch");
        if (rc) return rc;
        first = false;
    }
    return 0;
}

int hfv_verify_batches(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    int rc = batches_check(ctx, batches, count);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    return batches_launch(ctx, batches, count, pick_stream(ctx, stream), nullptr, nullptr);
}

int hfv_verify_batches_timed(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, void *stream,
                             float *kernel_ms)
{
    if (!ctx || !kernel_ms) return fail(-EINVAL, "null argument");
    *kernel_ms = 0.0f;
    int rc = batches_check(ctx, batches, count);
    if (rc) return rc;
    size_t nonempty = 0;
    for (size_t i = 0; i < count; ++i) nonempty += batches[i].n != 0;
    if (!nonempty) return 0;
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    for (int i = 0; i < 2; ++i)
        if (!ctx->tev[i]) HIP_TRY(hipEventCreate(&ctx->tev[i]));
    // the block finish stamps are atomic maxima: cleared before the timed launches (outside the events)
    HIP_TRY(hipMemsetAsync(ctx->bat_clk + 4 + kBatchStampBlocks, 0, kBatchStampBlocks * sizeof(uint64_t),
                           pick_stream(ctx, stream)));
    rc = batches_launch(ctx, batches, count, pick_stream(ctx, stream), ctx->tev[0], ctx->tev[1]);
    if (rc) return rc;
    HIP_TRY(hipEventSynchronize(ctx->tev[1]));
    HIP_TRY(hipEventElapsedTime(kernel_ms, ctx->tev[0], ctx->tev[1]));
    return 0;
}

// Diagnostic (not part of include/scion_hfv.h): block 0's shader clock (s_memtime) and 100 MHz
// s_memrealtime at the start and at the end of the last hfv_verify_batches launch (out[0..3]);
// with words >= 4 + 2 * 1024 also every block's s_memrealtime at its entry (out[4 + k]) and when it
// finished (out[4 + 1024 + k]).  The caller has synchronized that launch.
extern "C" int hfv_debug_batches_clock(hfv_ctx *ctx, uint64_t *out, size_t words)
{
    if (!ctx || !out || words < 4) return fail(-EINVAL, "bad argument");
    DeviceGuard g(ctx->device);
    if (words > kBatchClkWords) words = kBatchClkWords;
    HIP_TRY(hipMemcpy(out, ctx->bat_clk, words * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return 0;
}

// Diagnostic (not part of include/scion_hfv.h): one dense non-temporal streaming read of `count`
// (<= 64) device buffers on `stream`, waited for; *kernel_ms = its dispatch time.  bench.py prices
// the verify kernel against this rate over the same resident batches (roofline.achievable_peak).
extern "C" int hfv_debug_stream_read(hfv_ctx *ctx, const void *const *bufs, const size_t *bytes, size_t count,
                                     void *stream, float *kernel_ms)
{
    if (!ctx || !bufs || !bytes || !kernel_ms || count == 0 || count > kBatchMax) return fail(-EINVAL, "bad argument");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    for (int i = 0; i < 2; ++i)
        if (!ctx->tev[i]) HIP_TRY(hipEventCreate(&ctx->tev[i]));
    StreamArgs a;
    memset(&a, 0, sizeof a);
    a.nb = (uint32_t)count;
    a.sink = (uint32_t *)ctx->bat_clk;   // never written in practice (see k_stream_read)
    for (size_t i = 0; i < count; ++i) {
        if (((uintptr_t)bufs[i] & 15) || (bytes[i] & 15)) return fail(-EINVAL, "buffer %zu not 16-byte aligned", i);
        a.buf[i] = bufs[i];
        a.bytes[i] = bytes[i];
    }
    hipStream_t st = pick_stream(ctx, stream);
    int e = launch_stream_read(ctx->geom, a, st, ctx->tev[0], ctx->tev[1]);
    if (e != hipSuccess) return hip_fail((hipError_t)e, "stream read launch");
    HIP_TRY(hipEventSynchronize(ctx->tev[1]));
    HIP_TRY(hipEventElapsedTime(kernel_ms, ctx->tev[0], ctx->tev[1]));
    return 0;
}

// Diagnostic (not part of include/scion_hfv.h): the default KEYSEL_ZERO kernel with per-wave
// s_memrealtime stamps, for the timeline analysis in scripts/stamps.py.  stamps: device
// buffer of (grid * 16 waves) x 16 u64; returns the grid size in *grid.
extern "C" int hfv_debug_verify_stamped(hfv_ctx *ctx, const void *recs, size_t n, uint64_t *pass_bits,
                                        uint64_t *stamps, void *stream, int *grid)
{
    if (!ctx || !recs || !pass_bits || !stamps || !grid || n == 0) return fail(-EINVAL, "bad argument");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    const DevKeyTable *tab = &ds->keys;
    uint64_t tiles = (n + 63) / 64, blocks = (tiles + 15) / 16, cap = (uint64_t)ctx->geom.num_cus;
    *grid = (int)(blocks < cap ? blocks : cap);
    int e = launch_verify_stamped(ctx->geom, tab, &ctx->host_img->keys, (const uint8_t *)recs, n, pass_bits, stamps, st);
    return after_launch(ctx, st, e, "stamped launch");
}

int hfv_ctx_describe(const hfv_ctx *ctx, char *buf, size_t len)
{
    if (!ctx || !buf || !len) return fail(-EINVAL, "null argument");
    snprintf(buf, len,
             "verify: 1024-thread blocks, one per CU (%d CUs), four 32x-replicated round tables in LDS (128 KiB), "
             "T0 and slot-0 key rows in the kernel arguments; keysel ifid: five 16 B LDS rows per slot "
             "(round-1 folded key, rk2, schedule words of rounds 3..10); service grid %d blocks",
             ctx->geom.num_cus, ctx->geom.svc_blocks);
    return 0;
}

int hfv_verify_macinputs(hfv_ctx *ctx, const struct macinput *mi, const uint64_t *expected, const uint8_t *key_index,
                         size_t n, uint64_t *pass_bits, void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!mi || !expected || !pass_bits) return fail(-EINVAL, "null buffer");
    if (((uintptr_t)mi & 15) || ((uintptr_t)expected & 7) || ((uintptr_t)pass_bits & 7))
        return fail(-EINVAL, "macinputs must be 16-byte aligned, expected/bitmap 8-byte aligned");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    const DevKeyTable *tab = &ds->keys;
    int e = launch_verify_macinputs(ctx->geom, tab, mi, expected, key_index, n, pass_bits, st);
    return after_launch(ctx, st, e, "verify_macinputs launch");
}

int hfv_cmac_tags(hfv_ctx *ctx, const struct macinput *mi, const uint8_t *key_index, size_t n, struct aes_cmac *tags,
                  void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!mi || !tags) return fail(-EINVAL, "null buffer");
    if (((uintptr_t)mi & 15) || ((uintptr_t)tags & 15)) return fail(-EINVAL, "macinputs/tags must be 16-byte aligned");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    const DevKeyTable *tab = &ds->keys;
    int e = launch_cmac_tags(ctx->geom, tab, mi, key_index, n, tags, st);
    return after_launch(ctx, st, e, "cmac_tags launch");
}

int hfv_expand_keys(hfv_ctx *ctx, const struct aes_key *keys, size_t n, struct hop_key *out, void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!keys || !out) return fail(-EINVAL, "null buffer");
    if (((uintptr_t)keys & 15) || ((uintptr_t)out & 15)) return fail(-EINVAL, "buffers must be 16-byte aligned");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    int e = launch_expand_keys((const uint8_t *)keys, n, out, nullptr, 0, pick_stream(ctx, stream));
    if (e != hipSuccess) return hip_fail((hipError_t)e, "expand_keys launch");
    return 0;
}

int hfv_gen_records(hfv_ctx *ctx, void *recs, size_t stride, size_t n, uint64_t seed, uint64_t first_index,
                    void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!recs) return fail(-EINVAL, "null buffer");
    if (((uintptr_t)recs & 15) || (stride & 15) || stride < 64)
        return fail(-EINVAL, "records must be 16-byte aligned with stride >= 64, multiple of 16");
    if (ctx->inf_off != HFV_REC_INF_OFF || ctx->hf_off != HFV_REC_HF_OFF)
        return fail(-EINVAL, "the generator writes the default 64 B layout only");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    const DevKeyTable *tab = &ds->keys;
    int e = launch_gen_records(ctx->geom, tab, ctx->keysel, (uint8_t *)recs, stride, n, seed, first_index, st);
    return after_launch(ctx, st, e, "gen_records launch");
}

int hfv_verdict_counters(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, const uint64_t *pass_bits,
                         uint64_t *counters, void *stream)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!recs || !pass_bits || !counters) return fail(-EINVAL, "null buffer");
    if (stride < (size_t)ctx->inf_off + 8 || stride < (size_t)ctx->hf_off + 12)
        return fail(-EINVAL, "stride %zu too small for INF@%u/HF@%u", stride, ctx->inf_off, ctx->hf_off);
    if (((uintptr_t)pass_bits & 7) || ((uintptr_t)counters & 7)) return fail(-EINVAL, "bitmap and counters must be 8-byte aligned");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    int e = launch_count_verdicts(ctx->geom, (const uint8_t *)recs, stride, n, ctx->inf_off, ctx->hf_off, pass_bits,
                                  counters, st);
    if (e != hipSuccess) return hip_fail((hipError_t)e, "count_verdicts launch");
    return 0;
}

// ---- full border-router path (config 4) ---------------------------------------------------

int hfv_br_set_config(hfv_ctx *ctx, const struct hfv_br_config *cfg)
{
    if (!ctx || !cfg) return fail(-EINVAL, "null argument");
    if (br_config_check(cfg) == 0 && ctx->br.feat_off && hfv_br_config_check_options(cfg, ctx->br.feat_off))
        return -EINVAL;   // an address of a family the router is built without (br-loader's error)
    if (br_config_check(cfg))
        return fail(-EINVAL, "router table larger than the fixed capacity (%d interfaces, %d routes, %d tx ports)",
                    HFV_BR_MAX_IFACES, HFV_BR_MAX_ROUTES, HFV_BR_MAX_TXPORTS);
    const uint32_t off = ctx->br.hf_check_off, feat = ctx->br.feat_off;
    compile_br_config(cfg, &ctx->br);
    ctx->br.hf_check_off = off;
    ctx->br.feat_off = feat;
    ctx->cfg_src = *cfg;
    ctx->dirty = true;
    brcfg_close(ctx->brmap);   // explicit tables replace an attached pinned config
    ctx->brmap = nullptr;
    return 0;
}

int hfv_br_load_config(hfv_ctx *ctx, const char *toml_path, const struct hfv_br_next_hop *hops, size_t n_hops)
{
    if (!ctx || !toml_path) return fail(-EINVAL, "null argument");
    hfv_br_config cfg;
    int rc = hfv_br_config_load(toml_path, nullptr, 0, hops, n_hops, &cfg, nullptr, 0, nullptr, 0, nullptr, 0);
    if (rc) return rc;
    return hfv_br_set_config(ctx, &cfg);
}

int hfv_ctx_attach_brconfig(hfv_ctx *ctx, const char *path)
{
    if (!ctx || !path) return fail(-EINVAL, "null argument");
    const void *m = nullptr;
    int rc = brcfg_open_ro(path, &m);
    if (rc) return fail(rc, "cannot attach pinned router config %s", path);
    brcfg_close(ctx->brmap);
    ctx->brmap = m;
    ctx->brmap_seq = 0xffffffffu;   // loaded at the next batch boundary
    return 0;
}

int hfv_br_set_build_options(hfv_ctx *ctx, uint32_t disabled)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (hfv_br_config_check_options(&ctx->cfg_src, disabled)) return -EINVAL;
    ctx->br.feat_off = disabled;
    ctx->dirty = true;
    return 0;
}

int hfv_br_set_hf_check(hfv_ctx *ctx, int enable)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    ctx->br.hf_check_off = enable ? 0u : 1u;
    ctx->dirty = true;
    return 0;
}

static int br_args(hfv_ctx *ctx, uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex,
                   uint8_t *action, uint8_t *verdict, int32_t *egress_ifindex)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (!pkts || !len || !ingress_ifindex || !action || !verdict || !egress_ifindex) return fail(-EINVAL, "null buffer");
    if (slot < 64 || (slot & 7) || ((uintptr_t)pkts & 7)) return fail(-EINVAL, "slot must be >= 64 and a multiple of 8, frames 8-byte aligned");
    if (((uintptr_t)len & 1) || ((uintptr_t)ingress_ifindex & 3) || ((uintptr_t)egress_ifindex & 3))
        return fail(-EINVAL, "misaligned length/ifindex array");
    return 0;
}

int hfv_br_process(hfv_ctx *ctx, uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex,
                   size_t n, uint8_t *action, uint8_t *verdict, int32_t *egress_ifindex, uint64_t *stats,
                   void *stream)
{
    if (n == 0) return ctx ? 0 : fail(-EINVAL, "ctx is NULL");
    int rc = br_args(ctx, pkts, slot, len, ingress_ifindex, action, verdict, egress_ifindex);
    if (rc) return rc;
    if ((uintptr_t)stats & 7) return fail(-EINVAL, "misaligned stats");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    int e = launch_br_process(br_geom(ctx), ds, pkts, slot, (uint32_t)slot, (uint32_t)slot, len, ingress_ifindex, n,
                              action, verdict, egress_ifindex, stats, st);
    return after_launch(ctx, st, e, "br_process launch");
}

int hfv_br_process_timed(hfv_ctx *ctx, uint8_t *pkts, size_t slot, const uint16_t *len,
                         const uint32_t *ingress_ifindex, size_t n, uint8_t *action, uint8_t *verdict,
                         int32_t *egress_ifindex, uint64_t *stats, void *stream, float *kernel_ms)
{
    if (!kernel_ms) return fail(-EINVAL, "kernel_ms is NULL");
    *kernel_ms = 0.0f;
    if (n == 0) return ctx ? 0 : fail(-EINVAL, "ctx is NULL");
    int rc = br_args(ctx, pkts, slot, len, ingress_ifindex, action, verdict, egress_ifindex);
    if (rc) return rc;
    if ((uintptr_t)stats & 7) return fail(-EINVAL, "misaligned stats");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    for (int i = 0; i < 2; ++i)
        if (!ctx->tev[i]) HIP_TRY(hipEventCreate(&ctx->tev[i]));
    hipStream_t st = pick_stream(ctx, stream);
    DevState *ds;
    rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    int e = launch_br_process(br_geom(ctx), ds, pkts, slot, (uint32_t)slot, (uint32_t)slot, len, ingress_ifindex, n,
                              action, verdict, egress_ifindex, stats, st, ctx->tev[0], ctx->tev[1]);
    rc = after_launch(ctx, st, e, "br_process launch");
    if (rc) return rc;
    HIP_TRY(hipEventSynchronize(ctx->tev[1]));
    HIP_TRY(hipEventElapsedTime(kernel_ms, ctx->tev[0], ctx->tev[1]));
    return 0;
}

// Windowed host path.  Per chunk of kBrChunk frames, on alternating streams: strided H2D of
// the windows + metadata, the kernel (stride = window, lengths clamped to the caller's slot),
// strided D2H of the rewritten windows + results.  Then frames marked HFV_BR_ACTION_RETRY
// (headers beyond the window) go through again with whole slots.
}  // extern "C"

// Compact staging record of the host path: INF (8 B) at 0, HF (12 B) at 8, 4 B pad.
static constexpr size_t kHostRec = 24;

// Host threads for staging copies: HFV_HOST_THREADS, default min(8, cores).
static int host_threads()
{
    static const int t = [] {
        const char *e = getenv("HFV_HOST_THREADS");
        int v = e ? atoi(e) : 0;
        if (v <= 0) {
            unsigned hc = std::thread::hardware_concurrency();
            v = hc ? (int)(hc < 8 ? hc : 8) : 4;
        }
        return v;
    }();
    return t;
}

// NUMA placement of the host-side workers: the staging copies of a GPU's host path run on
// the CPUs of the NUMA node its PCIe root port hangs off (one process per GPU, so the
// first ctx of the process decides).  HFV_NUMA_PIN=0 leaves the threads unpinned.
static std::mutex g_numa_m;
static cpu_set_t g_numa_cpus;
static bool g_numa_set = false;

static void pin_to_numa()
{
    std::lock_guard<std::mutex> g(g_numa_m);
    if (g_numa_set) (void)pthread_setaffinity_np(pthread_self(), sizeof g_numa_cpus, &g_numa_cpus);
}

// NUMA node of `device` (from its PCI bus id in sysfs) and that node's CPUs that this
// process may run on; -1 if unknown.
static int device_numa(int device, cpu_set_t *cpus)
{
    char bus[64] = {0}, path[256];
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return -1;
    for (char *p = bus; *p; ++p)
        if (*p >= 'A' && *p <= 'F') *p = (char)(*p - 'A' + 'a');
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    if (node < 0 || !cpus) return node;
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    f = fopen(path, "r");
    if (!f) return node;
    cpu_set_t allowed;
    CPU_ZERO(cpus);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) CPU_ZERO(&allowed);
    int a, b;
    char sep;
    while (fscanf(f, "%d", &a) == 1) {
        b = a;
        if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
            if (fscanf(f, "%d", &b) != 1) break;
            if (fscanf(f, "%c", &sep) != 1) sep = 0;
        }
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &allowed)) CPU_SET(c, cpus);
        if (sep != ',') break;
    }
    fclose(f);
    return node;
}

static void note_numa(int device)
{
    const char *e = getenv("HFV_NUMA_PIN");
    if (e && atoi(e) == 0) return;
    cpu_set_t cpus;
    int node = device_numa(device, &cpus);
    std::lock_guard<std::mutex> g(g_numa_m);
    if (node >= 0 && !g_numa_set && CPU_COUNT(&cpus) > 0) {
        g_numa_cpus = cpus;
        g_numa_set = true;
    }
}

// Persistent host worker threads for the staging copies (spawning threads per copy cost more
// than the copies: 32 spawns per 2^20-frame router batch).  Part 0 of every job runs on the
// calling thread, parts 1..nt-1 on the workers.  Jobs come from one ctx thread at a time.
class HostPool {
  public:
    explicit HostPool(int nt) : nt_(nt)
    {
        for (int k = 1; k < nt_; ++k) th_.emplace_back([this, k] {
            pin_to_numa();
            work(k);
        });
    }
    ~HostPool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void run(size_t n, const std::function<void(size_t, size_t)> &fn)
    {
        std::unique_lock<std::mutex> lk(job_m_);   // one job at a time
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            n_ = n;
            left_ = nt_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0, n / nt_);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
        fn_ = nullptr;
    }
    int threads() const { return nt_; }

  private:
    void work(int k)
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(size_t, size_t)> *fn;
            size_t n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
                n = n_;
            }
            (*fn)(n * k / nt_, n * (k + 1) / nt_);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    int nt_;
    std::vector<std::thread> th_;
    std::mutex m_, job_m_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t, size_t)> *fn_ = nullptr;
    size_t n_ = 0;
    int left_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

static HostPool &host_pool()
{
    static HostPool pool(host_threads());
    return pool;
}

// fn(a, b) over [0, n) split into host_threads() contiguous parts (inline below 8192 items).
template <class F>
static void parallel_rows(size_t n, F fn)
{
    if (host_threads() <= 1 || n < 8192) {
        fn((size_t)0, n);
        return;
    }
    host_pool().run(n, std::function<void(size_t, size_t)>(fn));
}

// dst[i] = {INF, HF} of src record i (the verifier's 20 bytes).
static void gather_hf(uint8_t *dst, const uint8_t *src, size_t stride, uint32_t inf_off, uint32_t hf_off, size_t n)
{
    parallel_rows(n, [=](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            const uint8_t *r = src + i * stride;
            uint8_t *d = dst + i * kHostRec;
            memcpy(d, r + inf_off, 8);
            memcpy(d + 8, r + hf_off, 12);
        }
    });
}

// Row copies between frames in their slots and packed windows: dst row i <- src row i.
static void copy_rows(uint8_t *dst, size_t dpitch, const uint8_t *src, size_t spitch, size_t width, size_t n)
{
    parallel_rows(n, [=](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) memcpy(dst + i * dpitch, src + i * spitch, width);
    });
}

extern "C" {

static const size_t kBrChunk = (size_t)1 << 16;

static int brh_buffers(hfv_ctx *ctx, size_t window)
{
    for (int i = 0; i < 2; ++i) {
        if (!ctx->hstream[i]) HIP_TRY(hipStreamCreateWithFlags(&ctx->hstream[i], hipStreamNonBlocking));
        if (!ctx->brh_dio[i]) {
            HIP_TRY(hipMalloc((void **)&ctx->brh_dio[i], kBrChunk * 12));
            HIP_TRY(hipHostMalloc((void **)&ctx->brh_hio[i], kBrChunk * 12, hipHostMallocDefault));
        }
    }
    if (!ctx->brh_dstats) HIP_TRY(hipMalloc((void **)&ctx->brh_dstats, HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS * 8));
    if (ctx->brh_win_cap < window) {
        for (int i = 0; i < 2; ++i) {
            HIP_TRY(hipStreamSynchronize(ctx->hstream[i]));
            if (ctx->brh_dwin[i]) (void)hipFree(ctx->brh_dwin[i]);
            if (ctx->brh_hwin[i]) (void)hipHostFree(ctx->brh_hwin[i]);
            ctx->brh_dwin[i] = ctx->brh_hwin[i] = nullptr;
            HIP_TRY(hipMalloc((void **)&ctx->brh_dwin[i], kBrChunk * window));
            HIP_TRY(hipHostMalloc((void **)&ctx->brh_hwin[i], kBrChunk * window, hipHostMallocDefault));
        }
        ctx->brh_win_cap = window;
    }
    return 0;
}

// One chunk: frames[k * fstride] for k < cnt (window bytes each), metadata through pinned io.
static int brh_chunk(hfv_ctx *ctx, int sl, uint8_t *frames, size_t fstride, size_t maxlen, size_t window,
                     const uint16_t *len, const uint32_t *ifx, size_t cnt)
{
    hipStream_t st = ctx->hstream[sl];
    uint8_t *hio = ctx->brh_hio[sl], *dio = ctx->brh_dio[sl];
    memcpy(hio, len, cnt * 2);
    memcpy(hio + kBrChunk * 2, ifx, cnt * 4);
    HIP_TRY(hipMemcpyAsync(dio, hio, kBrChunk * 6, hipMemcpyHostToDevice, st));
    // the header windows, packed by host threads into pinned staging, then one linear DMA
    copy_rows(ctx->brh_hwin[sl], window, frames, fstride, window, cnt);
    HIP_TRY(hipMemcpyAsync(ctx->brh_dwin[sl], ctx->brh_hwin[sl], cnt * window, hipMemcpyHostToDevice, st));
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    int e = launch_br_process(br_geom(ctx), ds, ctx->brh_dwin[sl], window, (uint32_t)maxlen, (uint32_t)window,
                              (const uint16_t *)dio, (const uint32_t *)(dio + kBrChunk * 2), cnt,
                              dio + kBrChunk * 6, dio + kBrChunk * 7, (int32_t *)(dio + kBrChunk * 8),
                              ctx->brh_dstats, st);
    rc = after_launch(ctx, st, e, "br_process launch");
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->brh_hwin[sl], ctx->brh_dwin[sl], cnt * window, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(hio + kBrChunk * 6, dio + kBrChunk * 6, kBrChunk * 6, hipMemcpyDeviceToHost, st));
    return 0;
}

// A retired chunk (its stream synchronized): the rewritten windows back into the frames
// (host threads), and the per-frame results.
static void brh_results(hfv_ctx *ctx, int sl, uint8_t *frames, size_t fstride, size_t window, size_t cnt,
                        uint8_t *action, uint8_t *verdict, int32_t *egress)
{
    copy_rows(frames, fstride, ctx->brh_hwin[sl], window, window, cnt);
    const uint8_t *hio = ctx->brh_hio[sl];
    memcpy(action, hio + kBrChunk * 6, cnt);
    memcpy(verdict, hio + kBrChunk * 7, cnt);
    memcpy(egress, hio + kBrChunk * 8, cnt * 4);
}

// Device address of [p, p + bytes) if it lies in a mapped registered buffer, else NULL.
static uint8_t *host_dev_ptr(hfv_ctx *ctx, const void *p, size_t bytes)
{
    const uint8_t *q = (const uint8_t *)p;
    for (int i = 0; i < ctx->nhreg; ++i) {
        const hfv_ctx::HostRange &r = ctx->hreg[i];
        if (q >= r.host && q + bytes <= r.host + r.bytes) return r.dev + (q - r.host);
    }
    return nullptr;
}

// Zero-copy: the frames are in a registered (mapped) ring, so the kernel reads each header
// window across PCIe itself and writes back only the rewritten rows; no DMA of frame bytes and
// no retry pass (the whole frame stays addressable).  Per-frame metadata uses the caller's
// arrays in place when they are registered too, else one copy each way.
static int br_zero_copy(hfv_ctx *ctx, uint8_t *dframes, size_t slot, const uint16_t *len, const uint32_t *ifx,
                        size_t n, uint8_t *action, uint8_t *verdict, int32_t *egress, uint64_t *stats)
{
    hipStream_t st = ctx->stream;
    if (!ctx->brh_dstats) HIP_TRY(hipMalloc((void **)&ctx->brh_dstats, HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS * 8));
    HIP_TRY(hipMemsetAsync(ctx->brh_dstats, 0, HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS * 8, st));
    uint16_t *dlen = (uint16_t *)host_dev_ptr(ctx, len, n * 2);
    uint32_t *difx = (uint32_t *)host_dev_ptr(ctx, ifx, n * 4);
    uint8_t *dact = host_dev_ptr(ctx, action, n), *dver = host_dev_ptr(ctx, verdict, n);
    int32_t *degr = (int32_t *)host_dev_ptr(ctx, egress, n * 4);
    size_t need = n * 16;
    if ((!dlen || !difx || !dact || !dver || !degr) && ctx->zc_cap < need) {
        if (ctx->zc_meta) (void)hipFree(ctx->zc_meta);
        ctx->zc_meta = nullptr;
        HIP_TRY(hipMalloc((void **)&ctx->zc_meta, need));
        ctx->zc_cap = need;
    }
    uint8_t *m = ctx->zc_meta;
    if (!dlen) { dlen = (uint16_t *)m; HIP_TRY(hipMemcpyAsync(dlen, len, n * 2, hipMemcpyHostToDevice, st)); }
    if (!difx) { difx = (uint32_t *)(m + n * 4); HIP_TRY(hipMemcpyAsync(difx, ifx, n * 4, hipMemcpyHostToDevice, st)); }
    bool cp_act = !dact, cp_ver = !dver, cp_egr = !degr;
    if (cp_act) dact = m + n * 2;
    if (cp_ver) dver = m + n * 3;
    if (cp_egr) degr = (int32_t *)(m + n * 8);
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    int e = launch_br_process(br_geom(ctx), ds, dframes, slot, (uint32_t)slot, (uint32_t)slot, dlen, difx, n, dact, dver,
                              degr, ctx->brh_dstats, st);
    rc = after_launch(ctx, st, e, "br_process launch");
    if (rc) return rc;
    if (cp_act) HIP_TRY(hipMemcpyAsync(action, dact, n, hipMemcpyDeviceToHost, st));
    if (cp_ver) HIP_TRY(hipMemcpyAsync(verdict, dver, n, hipMemcpyDeviceToHost, st));
    if (cp_egr) HIP_TRY(hipMemcpyAsync(egress, degr, n * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (stats) {
        uint64_t tmp[HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS];
        HIP_TRY(hipMemcpy(tmp, ctx->brh_dstats, sizeof tmp, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < sizeof tmp / 8; ++k) stats[k] += tmp[k];
    }
    return 0;
}

}  // extern "C"

int hfv::br_zc_prepare(hfv_ctx *ctx)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    SVC_QUIESCE(ctx);
    HIP_TRY(hipSetDevice(ctx->device));
    return 0;
}

void hfv::forget_stream(hfv_ctx *ctx, void *stream)
{
    for (int a = 0; a < 2; ++a)
        for (int r = 0; r < ctx->nreaders[a];)
            if (ctx->readers[a][r] == (hipStream_t)stream) {
                // the last entry moves into slot r together with its fence event
                const int last = --ctx->nreaders[a];
                ctx->readers[a][r] = ctx->readers[a][last];
                std::swap(ctx->reader_ev[a][r], ctx->reader_ev[a][last]);
            } else {
                ++r;
            }
}

int hfv::br_dev_launch(hfv_ctx *ctx, void *stream, uint8_t *dframes, size_t slot, const uint16_t *dlen,
                       const uint32_t *difx, size_t n, uint8_t *dact, uint8_t *dver, int32_t *degr, uint64_t *dstats,
                       uint8_t *dout)
{
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    int e = launch_br_process(br_geom(ctx), ds, dframes, slot, (uint32_t)slot, (uint32_t)slot, dlen, difx, n, dact, dver,
                              degr, dstats, st, nullptr, nullptr, dout);
    return after_launch(ctx, st, e, "br_process launch");
}

extern "C" {

int hfv_br_process_host(hfv_ctx *ctx, uint8_t *frames, size_t slot, const uint16_t *len,
                        const uint32_t *ingress_ifindex, size_t n, size_t window, uint8_t *action,
                        uint8_t *verdict, int32_t *egress_ifindex, uint64_t *stats)
{
    if (n == 0) return ctx ? 0 : fail(-EINVAL, "ctx is NULL");
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (!frames || !len || !ingress_ifindex || !action || !verdict || !egress_ifindex) return fail(-EINVAL, "null buffer");
    if (slot < 64 || (slot & 7) || slot > 65535 * 8) return fail(-EINVAL, "slot must be >= 64 and a multiple of 8");
    if (window == 0) window = slot < 256 ? slot : 256;
    if (window < 64 || (window & 7) || window > slot) return fail(-EINVAL, "window must be a multiple of 8 in [64, slot]");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    uint8_t *dframes = host_dev_ptr(ctx, frames, n * slot);
    if (dframes) return br_zero_copy(ctx, dframes, slot, len, ingress_ifindex, n, action, verdict, egress_ifindex, stats);
    int rc = brh_buffers(ctx, window > slot ? slot : window);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(ctx->brh_dstats, 0, HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS * 8, ctx->hstream[0]));
    HIP_TRY(hipStreamSynchronize(ctx->hstream[0]));
    size_t nchunks = (n + kBrChunk - 1) / kBrChunk;
    size_t first_of[2] = {0, 0}, cnt_of[2] = {0, 0};
    for (size_t c = 0; c < nchunks + 2; ++c) {
        int sl = (int)(c & 1);
        if (c >= 2) {
            HIP_TRY(hipStreamSynchronize(ctx->hstream[sl]));
            size_t f = first_of[sl];
            brh_results(ctx, sl, frames + f * slot, slot, window, cnt_of[sl], action + f, verdict + f,
                        egress_ifindex + f);
        }
        if (c >= nchunks) continue;
        size_t first = c * kBrChunk, cnt = n - first < kBrChunk ? n - first : kBrChunk;
        rc = brh_chunk(ctx, sl, frames + first * slot, slot, slot, window, len + first, ingress_ifindex + first, cnt);
        if (rc) return rc;
        first_of[sl] = first;
        cnt_of[sl] = cnt;
    }
    // frames whose headers did not fit the window: whole slots, in chunks, through a bounce buffer
    size_t nretry = 0;
    for (size_t i = 0; i < n; ++i) nretry += action[i] == HFV_BR_ACTION_RETRY;
    if (nretry) {
        rc = brh_buffers(ctx, slot);
        if (rc) return rc;
        uint8_t *bounce = nullptr;
        size_t cap = nretry < kBrChunk ? nretry : kBrChunk;
        HIP_TRY(hipHostMalloc((void **)&bounce, cap * slot + cap * 8, hipHostMallocDefault));
        uint16_t *blen = (uint16_t *)(bounce + cap * slot);
        uint32_t *bif = (uint32_t *)(bounce + cap * slot + cap * 2);
        size_t *idx = (size_t *)malloc(cap * sizeof(size_t));
        size_t i = 0;
        while (rc == 0 && i < n) {
            size_t cnt = 0;
            for (; i < n && cnt < cap; ++i) {
                if (action[i] != HFV_BR_ACTION_RETRY) continue;
                memcpy(bounce + cnt * slot, frames + i * slot, slot);
                blen[cnt] = len[i];
                bif[cnt] = ingress_ifindex[i];
                idx[cnt++] = i;
            }
            if (!cnt) break;
            rc = brh_chunk(ctx, 0, bounce, slot, slot, slot, blen, bif, cnt);
            if (rc == 0 && hipStreamSynchronize(ctx->hstream[0]) != hipSuccess) rc = fail(-EIO, "retry chunk");
            for (size_t k = 0; rc == 0 && k < cnt; ++k) {
                size_t j = idx[k];
                memcpy(frames + j * slot, ctx->brh_hwin[0] + k * slot, slot);
                action[j] = ctx->brh_hio[0][kBrChunk * 6 + k];
                verdict[j] = ctx->brh_hio[0][kBrChunk * 7 + k];
                memcpy(&egress_ifindex[j], ctx->brh_hio[0] + kBrChunk * 8 + 4 * k, 4);
            }
        }
        free(idx);
        (void)hipHostFree(bounce);
        if (rc) return rc;
    }
    if (stats) {
        uint64_t tmp[HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS];
        HIP_TRY(hipMemcpy(tmp, ctx->brh_dstats, sizeof tmp, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < sizeof tmp / 8; ++k) stats[k] += tmp[k];
    }
    return 0;
}

int hfv_host_register(hfv_ctx *ctx, void *ptr, size_t bytes)
{
    if (!ctx || !ptr || !bytes) return fail(-EINVAL, "bad argument");
    if (ctx->nhreg == 16) return fail(-ENOMEM, "at most 16 registered host buffers per ctx");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
    void *dev = nullptr;
    hipError_t e = hipHostGetDevicePointer(&dev, ptr, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(ptr);
        return hip_fail(e, "hipHostGetDevicePointer");
    }
    ctx->hreg[ctx->nhreg++] = {(uint8_t *)ptr, bytes, (uint8_t *)dev};
    return 0;
}

int hfv_host_unregister(hfv_ctx *ctx, void *ptr)
{
    if (!ctx || !ptr) return fail(-EINVAL, "bad argument");
    DeviceGuard g(ctx->device);
    for (int i = 0; i < ctx->nhreg; ++i) {
        if (ctx->hreg[i].host != ptr) continue;
        HIP_TRY(hipDeviceSynchronize());   // no launch may still address it
        HIP_TRY(hipHostUnregister(ptr));
        ctx->hreg[i] = ctx->hreg[--ctx->nhreg];
        return 0;
    }
    return fail(-EINVAL, "buffer was not registered with this ctx");
}

// Zero-copy host batch: the records lie in a registered (mapped) host buffer, so one verify
// launch reads each record's INF/HF words across PCIe itself (20 of the 64 bytes; no bulk
// H2D copy).  The bitmap is written in place when it is registered too, else to a device
// buffer and copied back.
static int verify_records_zero_copy(hfv_ctx *ctx, const uint8_t *drecs, size_t stride, size_t n, uint64_t *pass_bits)
{
    hipStream_t st = ctx->stream;
    const size_t words = (n + 63) / 64;
    uint64_t *dbits = (uint64_t *)host_dev_ptr(ctx, pass_bits, words * 8);
    if (!dbits) {
        if (ctx->zc_cap < words * 8) {
            if (ctx->zc_meta) (void)hipFree(ctx->zc_meta);
            ctx->zc_meta = nullptr;
            ctx->zc_cap = 0;
            HIP_TRY(hipMalloc((void **)&ctx->zc_meta, words * 8));
            ctx->zc_cap = words * 8;
        }
        dbits = (uint64_t *)ctx->zc_meta;
    }
    DevState *ds;
    int rc = publish_keys(ctx, st, &ds);
    if (rc) return rc;
    int e = launch_verify_records(ctx->geom, &ds->keys, &ctx->host_img->keys, ctx->keysel, drecs, stride, n, ctx->inf_off, ctx->hf_off,
                                  dbits, st, nullptr, nullptr, /*interleaved=*/true);
    rc = after_launch(ctx, st, e, "verify_records launch (zero-copy)");
    if (rc) return rc;
    if (dbits == (uint64_t *)ctx->zc_meta) HIP_TRY(hipMemcpyAsync(pass_bits, dbits, words * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

// Host batch: chunks of records go host -> pinned -> device, verified, bitmap back; two
// streams alternate so chunk k's copy-in overlaps chunk k-1's kernel and copy-out.  Records
// in a registered buffer (hfv_host_register) take the zero-copy path instead.
int hfv_verify_records_host(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!recs || !pass_bits) return fail(-EINVAL, "null buffer");
    if ((stride & 7) || stride < (size_t)ctx->hf_off + 12 || stride < (size_t)ctx->inf_off + 8)
        return fail(-EINVAL, "bad stride %zu", stride);
    if (((uintptr_t)recs & 7) || ((uintptr_t)pass_bits & 7)) return fail(-EINVAL, "records and bitmap must be 8-byte aligned");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    if (const uint8_t *drecs = host_dev_ptr(ctx, recs, (n - 1) * stride + ctx->hf_off + 12))
        return verify_records_zero_copy(ctx, drecs, stride, n, pass_bits);
    // Staging: each chunk's records are gathered on the host into a compact pinned layout of
    // kHostRec bytes per record (INF at 0, HF at 8: the 20 bytes the verifier reads), so
    // PCIe moves 24 B instead of the record stride; the gather is split over host threads
    // and chunk c's gather overlaps chunk c-1's copy, kernel and copy-back on the other stream.
    const size_t chunk = (size_t)1 << 18;   // records per chunk
    if (ctx->host_chunk < chunk * kHostRec) {
        for (int i = 0; i < 2; ++i) {
            if (ctx->h_pin[i]) (void)hipHostFree(ctx->h_pin[i]);
            if (ctx->d_rec[i]) (void)hipFree(ctx->d_rec[i]);
            if (ctx->h_bits[i]) (void)hipHostFree(ctx->h_bits[i]);
            if (ctx->d_bits[i]) (void)hipFree(ctx->d_bits[i]);
            ctx->h_pin[i] = ctx->d_rec[i] = nullptr;
            ctx->h_bits[i] = ctx->d_bits[i] = nullptr;
            if (!ctx->hstream[i]) HIP_TRY(hipStreamCreateWithFlags(&ctx->hstream[i], hipStreamNonBlocking));
            HIP_TRY(hipHostMalloc((void **)&ctx->h_pin[i], chunk * kHostRec, hipHostMallocDefault));
            HIP_TRY(hipMalloc((void **)&ctx->d_rec[i], chunk * kHostRec));
            HIP_TRY(hipHostMalloc((void **)&ctx->h_bits[i], chunk / 8, hipHostMallocDefault));
            HIP_TRY(hipMalloc((void **)&ctx->d_bits[i], chunk / 8));
        }
        ctx->host_chunk = chunk * kHostRec;
    }
    size_t nchunks = (n + chunk - 1) / chunk;
    size_t pending_words[2] = {0, 0};
    size_t pending_first[2] = {0, 0};
    for (size_t c = 0; c < nchunks + 2; ++c) {
        int slot = (int)(c & 1);
        hipStream_t st = ctx->hstream[slot];
        if (c >= 2) {   // retire chunk c-2 (same slot)
            HIP_TRY(hipStreamSynchronize(st));
            memcpy(pass_bits + pending_first[slot], ctx->h_bits[slot], pending_words[slot] * 8);
        }
        if (c >= nchunks) continue;
        size_t first = c * chunk, cnt = n - first < chunk ? n - first : chunk;
        gather_hf(ctx->h_pin[slot], (const uint8_t *)recs + first * stride, stride, ctx->inf_off, ctx->hf_off, cnt);
        HIP_TRY(hipMemcpyAsync(ctx->d_rec[slot], ctx->h_pin[slot], cnt * kHostRec, hipMemcpyHostToDevice, st));
        DevState *ds;
        int rc = publish_keys(ctx, st, &ds);
        if (rc) return rc;
        const DevKeyTable *tab = &ds->keys;
        int e = launch_verify_records(ctx->geom, tab, &ctx->host_img->keys, ctx->keysel, ctx->d_rec[slot], kHostRec, cnt, 0, 8,
                                      ctx->d_bits[slot], st);
        rc = after_launch(ctx, st, e, "verify_records launch");
        if (rc) return rc;
        size_t words = (cnt + 63) / 64;
        HIP_TRY(hipMemcpyAsync(ctx->h_bits[slot], ctx->d_bits[slot], words * 8, hipMemcpyDeviceToHost, st));
        pending_words[slot] = words;
        pending_first[slot] = first / 64;
    }
    return 0;
}

// ---- resident verify service ----------------------------------------------------------
// The host side of k_verify_service (hfv_kernels.hip): tickets 1, 2, ... go to ring slot
// (t - 1) % kSvcRing; ticket t is posted only once ticket t - kSvcRing is done.  Ring and
// completion words hold svc_tag | t, the tag changing with every grid, so nothing is cleared
// between grids.

}  // extern "C"

// Grid-local batch t is complete once the relay has forwarded its completion (every block of
// the grid reported its share of it).
static bool svc_is_done(const hfv_ctx *ctx, uint64_t t)
{
    return __atomic_load_n(&ctx->svc_host->done[(t - 1) % kSvcRing], __ATOMIC_ACQUIRE) >= (ctx->svc_tag | t);
}

// The running grid has exited on the stop the host posted: it verified every batch before it
// (each block reaches the stop only after its share of all earlier batches), including those
// whose completion the relay did not forward (it leaves at the stop).
static bool svc_exited_clean(const hfv_ctx *ctx)
{
    return ctx->svc_running && ctx->svc_stop_posted && __atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE) == 0 &&
           hipStreamQuery(ctx->svc_stream) == hipSuccess;
}

// Device-side completion of grid-local batch t from a copy of SvcDev::done (after an idle or
// watchdog exit, when the relay may not have forwarded everything).
static bool svc_dev_done(const hfv_ctx *ctx, const std::vector<uint64_t> &done, uint64_t t)
{
    const uint64_t *d = &done[((t - 1) % kSvcRing) * kSvcMaxBlocks];
    for (unsigned k = 0; k < ctx->svc_grid; ++k)
        if (d[k] < (ctx->svc_tag | t)) return false;
    return true;
}


// Copy `bytes` at byte offset `off` of the ctx's SvcDev to host memory (diagnostics and the
// balance, after a grid; on the ctx's own stream, which a running grid does not occupy).
static int svc_dev_read(hfv_ctx *ctx, void *dst, size_t off, size_t bytes)
{
    if (!ctx->svc_dev) return fail(-EINVAL, "the verify service has not run");
    HIP_TRY(hipMemcpyAsync(dst, reinterpret_cast<const char *>(ctx->svc_dev) + off, bytes, hipMemcpyDeviceToHost,
                           ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

// SvcDev::done into a host vector for svc_dev_done.
static int svc_read_done(hfv_ctx *ctx, std::vector<uint64_t> &done)
{
    done.assign((size_t)kSvcRing * kSvcMaxBlocks, 0);
    return svc_dev_read(ctx, done.data(), offsetof(SvcDev, done), done.size() * 8);
}

static int svc_wait_done(hfv_ctx *ctx, uint64_t t, int timeout_ms)
{
    struct timespec t0, now;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t spin = 0;; ++spin) {
        if (svc_is_done(ctx, t)) return 0;
        if ((spin & 255) != 255) {
            __builtin_ia32_pause();
            continue;
        }
        if (hipStreamQuery(ctx->svc_stream) == hipSuccess) {   // the grid is gone
            if (svc_exited_clean(ctx)) return 0;
            std::vector<uint64_t> done;
            int rc = svc_read_done(ctx, done);
            if (rc) return rc;
            if (svc_dev_done(ctx, done, t)) return 0;
            const uint64_t st = __atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE);
            return fail(-EIO, "verify service exited (%s); ticket %llu will not complete",
                        st == kSvcIdleTimeout ? "idle timeout" : st == kSvcWatchdog ? "watchdog" : "grid ended",
                        (unsigned long long)(ctx->svc_base + t - 1));
        }
        clock_gettime(CLOCK_MONOTONIC, &now);
        double ms = (now.tv_sec - t0.tv_sec) * 1e3 + (now.tv_nsec - t0.tv_nsec) * 1e-6;
        if (timeout_ms >= 0 && ms > timeout_ms)
            return fail(-ETIMEDOUT, "ticket %llu not done after %d ms", (unsigned long long)(ctx->svc_base + t - 1),
                        timeout_ms);
    }
}

static int svc_post(hfv_ctx *ctx, uint64_t recs, uint64_t bits, uint64_t n, uint64_t stride, uint64_t *ticket)
{
    const uint64_t t = ctx->svc_next;   // grid-local batch number
    if (t > kSvcRing) {   // the slot's previous batch must be done (and its descriptor read)
        int rc = svc_wait_done(ctx, t - kSvcRing, 60000);
        if (rc) return rc;
    }
    SvcDesc *d = &ctx->svc_host->desc[(t - 1) % kSvcRing];
    d->recs = recs;
    d->bits = bits;
    d->n = n;
    d->stride = stride;
    __atomic_store_n(&d->seq, ctx->svc_tag | t, __ATOMIC_RELEASE);
    ctx->svc_next = t + 1;
    if (ticket) {   // a stop descriptor takes a grid slot but no ticket
        *ticket = ctx->svc_base + t - 1;
        ctx->svc_ticket = *ticket + 1;
    }
    return 0;
}

// Re-derive the block weights from the grid that just stopped (svc_run grids only: every batch
// was posted before the launch, so no block waited for the host and a block's tiles over its
// time from table fill to its last completed share is its verify rate).  Weights follow the
// XCDs' mean rates (block j on XCD j % 8) and block 0's own, averaged with the previous weights
// (halves run-to-run noise), clamped to [1/2, 2] of nominal.  Grids shorter than 50 us carry
// too little signal and leave them alone: with the grid's duration (grid_ns: its dispatch events;
// < 0 when it was not timed, then block 0's own stamps) below that, the G stamps are not even
// copied (a synchronous 16 KiB copy after every short grid).
static void svc_balance(hfv_ctx *ctx, double grid_ns)
{
    const uint64_t G = ctx->svc_grid;
    if (G < 16 || ctx->svc_run_ns.empty()) return;
    if (grid_ns >= 0.0 && grid_ns < 50000.0) return;
    if (grid_ns < 0.0) {   // untimed grid: block 0's span first (s_memrealtime, 100 MHz)
        uint64_t b0[2] = {0, 0};
        if (svc_dev_read(ctx, &b0[0], offsetof(SvcDev, blk_start), 8) ||
            svc_dev_read(ctx, &b0[1], offsetof(SvcDev, blk_fin), 8) || b0[1] < b0[0] + 5000)
            return;
    }
    std::vector<uint64_t> bt(2 * kSvcMaxBlocks);   // blk_start[0..G), blk_fin[0..G) (adjacent in SvcDev)
    static_assert(offsetof(SvcDev, blk_fin) == offsetof(SvcDev, blk_start) + kSvcMaxBlocks * 8, "layout");
    if (svc_dev_read(ctx, bt.data(), offsetof(SvcDev, blk_start), G * 8) ||
        svc_dev_read(ctx, bt.data() + kSvcMaxBlocks, offsetof(SvcDev, blk_fin), G * 8))
        return;
    const uint64_t *blk_start = bt.data(), *blk_fin = bt.data() + kSvcMaxBlocks;
    const SvcWeights &wu = ctx->svc_w_used;
    std::vector<uint64_t> cum(G + 1, 0);
    for (uint64_t k = 0; k < G; ++k) cum[k + 1] = cum[k] + (k ? wu.w[k % 8] : wu.w0);
    const uint64_t W = cum[G];
    std::vector<double> tiles(G, 0.0);
    for (size_t i = 0; i < ctx->svc_run_ns.size();) {   // runs of equal batch sizes at once
        size_t j = i;
        while (j < ctx->svc_run_ns.size() && ctx->svc_run_ns[j] == ctx->svc_run_ns[i]) ++j;
        const uint64_t T = (ctx->svc_run_ns[i] + 63) / 64;
        for (uint64_t k = 0; k < G; ++k)
            tiles[k] += (double)(j - i) * (double)(T * cum[k + 1] / W - T * cum[k] / W);
        i = j;
    }
    double rx[8] = {0}, r0 = 0, rsum = 0;
    int cx[8] = {0};
    uint64_t span = 0;
    for (uint64_t k = 0; k < G; ++k) {
        const uint64_t a = blk_start[k], b = blk_fin[k];
        if (b <= a || tiles[k] <= 0) return;   // a block without a measurement: keep the weights
        if (b - a > span) span = b - a;
        const double r = tiles[k] / (double)(b - a);
        rsum += r;
        if (k == 0) r0 = r;
        else {
            rx[k % 8] += r;
            cx[k % 8] += 1;
        }
    }
    if (span < 5000) return;   // 100 MHz ticks: 50 us
    const double mean = rsum / (double)G;
    // A grid some of whose blocks ran far below the others was disturbed from outside (a
    // transient on the box: blocks' rates normally stay within a few % of each other); learning
    // from it would carry the disturbance into the next grids' shares.
    double rmin = 1e300, rmax = 0;
    for (uint64_t k = 0; k < G; ++k) {
        const uint64_t a = blk_start[k], b = blk_fin[k];
        const double r = tiles[k] / (double)(b - a);
        rmin = r < rmin ? r : rmin;
        rmax = r > rmax ? r : rmax;
    }
    if (rmax > 1.6 * rmin) return;
    auto blend = [&](uint32_t old, double rate) {
        double w = 0.5 * old + 0.5 * kSvcWeightUnit * rate / mean;
        if (w < kSvcWeightUnit / 2) w = kSvcWeightUnit / 2;
        if (w > kSvcWeightUnit * 2) w = kSvcWeightUnit * 2;
        return (uint32_t)(w + 0.5);
    };
    for (int x = 0; x < 8; ++x)
        if (cx[x]) ctx->svc_w.w[x] = blend(ctx->svc_w.w[x], rx[x] / cx[x]);
    ctx->svc_w.w0 = blend(ctx->svc_w.w0, r0);
}

static int svc_stop(hfv_ctx *ctx, float *kernel_ms)
{
    if (kernel_ms) *kernel_ms = 0.0f;
    if (!ctx->svc_running) return 0;
    const uint64_t last = ctx->svc_next - 1 - (ctx->svc_stop_posted ? 1 : 0);   // last batch posted
    int rc = 0;
    if (!ctx->svc_stop_posted && __atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE) == 0)
        rc = svc_post(ctx, 0, 0, kSvcStopN, 0, nullptr);
    // the grid exits on the stop descriptor, or on its idle timeout if the post failed.  Spin
    // on the stream for a while first: the blocking wait sleeps on an interrupt, whose wake-up
    // costs more than the last batches of a short run.
    hipError_t e = hipErrorNotReady;
    struct timespec t0, now;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t spin = 0;; ++spin) {
        e = hipStreamQuery(ctx->svc_stream);
        if (e != hipErrorNotReady) break;
        __builtin_ia32_pause();
        if ((spin & 1023) == 1023) {
            clock_gettime(CLOCK_MONOTONIC, &now);
            if ((now.tv_sec - t0.tv_sec) * 1000000000ll + (now.tv_nsec - t0.tv_nsec) > 20000000ll) {   // 20 ms
                e = hipStreamSynchronize(ctx->svc_stream);
                break;
            }
        }
    }
    ctx->svc_running = false;
    if (e != hipSuccess) return hip_fail(e, "verify service");
    if (rc) return rc;
    if (kernel_ms && ctx->svc_timed) HIP_TRY(hipEventElapsedTime(kernel_ms, ctx->svc_ev[0], ctx->svc_ev[1]));
    if (ctx->svc_adapt && __atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE) == 0) {
        // the grid's own duration decides whether its stamps carry signal (the host
        // time since the launch call can be far longer than the grid ran): its dispatch events when
        // it was timed, else block 0's stamps (two words) before all G stamps are fetched
        double grid_ns = -1.0;
        float ms = 0.0f;
        if (ctx->svc_timed && hipEventElapsedTime(&ms, ctx->svc_ev[0], ctx->svc_ev[1]) == hipSuccess) grid_ns = ms * 1e6;
        svc_balance(ctx, grid_ns);
    }
    ctx->svc_adapt = false;
    // A grid that left on the stop descriptor verified every batch before it (each block
    // reaches the stop only after its share of all earlier batches).  An idle or watchdog
    // exit is clean unless it left a posted batch unverified (batches may complete out of
    // order; only the newest kSvcRing can still be open): scan those in a copy of the device
    // completion words (the relay may have left before forwarding them; not paid on a normal stop).
    if (__atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE) == 0) return 0;
    std::vector<uint64_t> done;
    rc = svc_read_done(ctx, done);
    if (rc) {
        // the completion words cannot be read: every ticket that may still have been open is
        // recorded as lost, so no poll or wait reports it done (fail closed)
        for (uint64_t t = last; t > 0 && t + kSvcRing > last; --t) {
            if (ctx->svc_lost.size() >= 4096) ctx->svc_lost.erase(ctx->svc_lost.begin(), ctx->svc_lost.begin() + 1024);
            ctx->svc_lost.push_back(ctx->svc_base + t - 1);
        }
        return rc;
    }
    uint64_t first_lost = 0;
    for (uint64_t t = last; t > 0 && t + kSvcRing > last; --t)
        if (!svc_dev_done(ctx, done, t)) {
            first_lost = ctx->svc_base + t - 1;
            if (ctx->svc_lost.size() >= 4096) ctx->svc_lost.erase(ctx->svc_lost.begin(), ctx->svc_lost.begin() + 1024);
            ctx->svc_lost.push_back(first_lost);
        }
    if (first_lost)
        return fail(-ETIMEDOUT, "verify service exited on its idle timeout before ticket %llu",
                    (unsigned long long)first_lost);
    return 0;
}

// Ticket state: 1 done, 0 pending, -EIO lost (its grid stopped without verifying it),
// -EINVAL never issued.  Tickets of stopped grids were verified unless they exited on a
// timeout (svc_lost); tickets of the running grid are done once their completion was
// forwarded, or once the grid has left on its stop.
static int svc_ticket_state(const hfv_ctx *ctx, uint64_t ticket)
{
    if (!ctx->svc_host || ticket == 0 || ticket >= ctx->svc_ticket) return -EINVAL;
    for (uint64_t l : ctx->svc_lost)
        if (l == ticket) return -EIO;
    if (ticket < ctx->svc_base || !ctx->svc_running) return 1;
    return svc_is_done(ctx, ticket - ctx->svc_base + 1) || svc_exited_clean(ctx) ? 1 : 0;
}

static int svc_quiesce(hfv_ctx *ctx) { return ctx->svc_running ? svc_stop(ctx, nullptr) : 0; }

static bool svc_keys_changed(hfv_ctx *ctx)
{
    return ctx->dirty || (ctx->keymap && keymap_seq(ctx->keymap) != ctx->keymap_seq);
}

extern "C" {

// A new service grid in two halves, so that a submit can post its batches into the ring
// between them and the grid finds them there when it starts: svc_begin (generation tag, key
// table, bookkeeping) and svc_launch.
static int svc_begin(hfv_ctx *ctx, uint32_t idle_ms, DevState **ds)
{
    if (!ctx->svc_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&ctx->svc_stream, hipStreamNonBlocking));
        HIP_TRY(hipHostMalloc((void **)&ctx->svc_host, sizeof(SvcShared),
                              hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer((void **)&ctx->svc_host_dev, ctx->svc_host, 0));
        HIP_TRY(hipMalloc((void **)&ctx->svc_dev, sizeof(SvcDev)));
        for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreate(&ctx->svc_ev[i]));
        memset(ctx->svc_host, 0, sizeof(SvcShared));
        HIP_TRY(hipMemsetAsync(ctx->svc_dev, 0, sizeof(SvcDev), ctx->svc_stream));
    }
    // a new generation: words an earlier grid left in the ring, the mirror and the completion
    // tables carry a smaller tag and never match
    ctx->svc_tag += 1ull << 40;
    __atomic_store_n(&ctx->svc_host->status, 0, __ATOMIC_RELEASE);
    int rc = publish_keys(ctx, ctx->svc_stream, ds);
    if (rc) return rc;
    ctx->svc_keysel = ctx->keysel;
    ctx->svc_inf_off = ctx->inf_off;
    ctx->svc_hf_off = ctx->hf_off;
    ctx->svc_idle_ms = idle_ms ? idle_ms : 1000;
    ctx->svc_next = 1;
    ctx->svc_base = ctx->svc_ticket;
    ctx->svc_stop_posted = false;
    ctx->svc_adapt = false;
    return 0;
}

#ifdef HFV_TEST_HOOKS
static uint32_t g_svc_relay_delay_us = 0;   // hfv_debug_relay_delay
#else
static constexpr uint32_t g_svc_relay_delay_us = 0;
#endif

static inline uint64_t mono_ns()
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// call_ns (nullable): svc_run's phase stamps (hfv_debug_service_call_ns), [3] before and [4] after
// the launch call; other callers (submitv, start) leave them alone
static int svc_launch(hfv_ctx *ctx, DevState *ds, uint64_t *call_ns = nullptr)
{
    const bool noev = !ctx->svc_timing;
    ctx->svc_timed = !noev;
    // the batches (and the stop) the caller posted before the launch (svc_run, submitv): the
    // first kSvcInline travel in the kernel arguments, so the blocks start on them without any
    // host round trip; the relay fetches the rest
    SvcArgs a;
    memset(&a, 0, sizeof a);
    a.tab = &ds->keys;
    a.host = ctx->svc_host_dev;
    a.dev = ctx->svc_dev;
    a.inf_off = ctx->inf_off;
    a.hf_off = ctx->hf_off;
    a.idle_ticks = (uint64_t)ctx->svc_idle_ms * 100000ull;
    a.tag = ctx->svc_tag;
    ctx->svc_w_used = ctx->svc_w;
    a.weights = ctx->svc_w_used;
    const uint64_t posted = ctx->svc_next - 1;
    a.n_inline = (uint32_t)(posted < kSvcInline ? posted : kSvcInline);
    for (uint32_t i = 0; i < a.n_inline; ++i) {
        const SvcDesc &d = ctx->svc_host->desc[i];
        a.inl[i] = {d.recs, d.bits, d.n, d.stride};
    }
    a.relay_delay_us = g_svc_relay_delay_us;
    a.launch = ctx->svc_launches;
    // slot 0's device key rows as published for this grid (the host image is what the last
    // publish copied into the device table), and T0
    for (int r = 0; r < kDevKeyRows; ++r) memcpy(&a.key0[4 * r], ctx->host_img->keys.rows[r][0], 16);
    a.key0_ok = ctx->host_img->keys.valid[0] & 1u;
    memcpy(a.t0, kTables.t0, sizeof a.t0);
    if (call_ns) call_ns[3] = mono_ns();
    int e = launch_verify_service(ctx->geom, ctx->keysel, a, ctx->svc_stream, noev ? nullptr : ctx->svc_ev[0],
                                  noev ? nullptr : ctx->svc_ev[1], &ctx->svc_grid);
    if (call_ns) call_ns[4] = mono_ns();
    int rc = after_launch(ctx, ctx->svc_stream, e, "verify service launch");
    if (rc) return rc;
    ++ctx->svc_launches;
    ctx->svc_running = true;
    return 0;
}

int hfv_service_start(hfv_ctx *ctx, uint32_t idle_ms)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    DeviceGuard g(ctx->device);
    if (ctx->svc_running && ctx->svc_stop_posted) {   // a run_async grid leaving on its own stop
        int rc = svc_stop(ctx, nullptr);
        if (rc) return rc;
    }
    if (ctx->svc_running) return 0;
    DevState *ds;
    int rc = svc_begin(ctx, idle_ms, &ds);
    if (rc) return rc;
    return svc_launch(ctx, ds);
}

static int svc_check_batch(const hfv_ctx *ctx, const void *recs, size_t stride, size_t n, const uint64_t *pass_bits)
{
    if (n && (!recs || !pass_bits)) return fail(-EINVAL, "null buffer");
    if (n >= kSvcStopN / 2) return fail(-EINVAL, "batch too large");
    if (((uintptr_t)recs & 7) || (stride & 7) || ((uintptr_t)pass_bits & 7))
        return fail(-EINVAL, "records, stride and bitmap must be 8-byte aligned");
    if (stride < (size_t)ctx->inf_off + 8 || stride < (size_t)ctx->hf_off + 12)
        return fail(-EINVAL, "stride %zu too small for INF@%u/HF@%u", stride, ctx->inf_off, ctx->hf_off);
    return 0;
}

// Restart the grid if it left on its idle timeout or if keys/keysel/layout changed (a batch
// boundary); if no grid runs, begin one and return its table in *launch (the caller posts its
// batches, then launches it with svc_launch), else *launch = nullptr.
static int svc_ready(hfv_ctx *ctx, DevState **launch)
{
    *launch = nullptr;
    if (ctx->svc_running && ctx->svc_stop_posted) {
        // a grid started by hfv_service_run_async has its stop behind its batches and exits by
        // itself: nothing posted now would be read, so reap it and begin a fresh grid
        int rc = svc_stop(ctx, nullptr);
        if (rc) return rc;
    }
    if (ctx->svc_running && __atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE) != 0) {
        // the grid left on its idle timeout: reap it (batches it left unverified are recorded
        // as lost for hfv_service_wait/poll) and start a fresh one
        (void)svc_stop(ctx, nullptr);
    }
    // key, key-selection or layout changes take effect at this batch boundary; the grid's
    // batch counter is 32-bit, so the service also restarts every 2^31 batches
    if (ctx->svc_running && (svc_keys_changed(ctx) || ctx->svc_keysel != ctx->keysel ||
                             ctx->svc_inf_off != ctx->inf_off || ctx->svc_hf_off != ctx->hf_off ||
                             ctx->svc_next >= (1ull << 31))) {
        int rc = svc_stop(ctx, nullptr);
        if (rc) return rc;
    }
    if (!ctx->svc_running) return svc_begin(ctx, ctx->svc_idle_ms, launch);
    return 0;
}

int hfv_service_submit(hfv_ctx *ctx, const void *recs, size_t stride, size_t n, uint64_t *pass_bits,
                       uint64_t *ticket)
{
    if (!ctx || !ticket) return fail(-EINVAL, "null argument");
    *ticket = 0;
    struct hfv_batch b = {recs, stride, n, pass_bits};
    return hfv_service_submitv(ctx, &b, 1, ticket);
}

int hfv_service_submitv(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket)
{
    if (!ctx || !first_ticket || (!batches && count)) return fail(-EINVAL, "null argument");
    *first_ticket = 0;
    for (size_t i = 0; i < count; ++i) {
        int rc = svc_check_batch(ctx, batches[i].recs, batches[i].stride, batches[i].n, batches[i].pass_bits);
        if (rc) {
            if (count == 1) return rc;
            char why[256];
            snprintf(why, sizeof why, "%s", hfv_last_error());
            return fail(rc, "batch %zu: %s", i, why);
        }
    }
    if (count == 0) return 0;
    DeviceGuard g(ctx->device);
    DevState *launch = nullptr;
    int rc = svc_ready(ctx, &launch);
    if (rc) return rc;
    for (size_t i = 0; i < count; ++i) {
        // a new grid is launched once the ring holds the first batches (at most a ring's
        // worth: posting more waits for completions), so it finds them when it starts
        if (launch && i == (size_t)kSvcRing) {
            rc = svc_launch(ctx, launch);
            launch = nullptr;
            if (rc) return rc;
        }
        uint64_t t = 0;
        rc = svc_post(ctx, (uint64_t)(uintptr_t)batches[i].recs, (uint64_t)(uintptr_t)batches[i].pass_bits,
                      batches[i].n, batches[i].stride, &t);
        if (rc) return rc;   // batches 0..i-1 are posted (tickets *first_ticket ..)
        if (i == 0) *first_ticket = t;
    }
    return launch ? svc_launch(ctx, launch) : 0;
}

static int svc_run(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket,
                   float *kernel_ms, bool wait);

int hfv_service_run(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket,
                    float *kernel_ms)
{
    return svc_run(ctx, batches, count, first_ticket, kernel_ms, true);
}

int hfv_service_run_async(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket)
{
    return svc_run(ctx, batches, count, first_ticket, nullptr, false);
}

static int svc_run(hfv_ctx *ctx, const struct hfv_batch *batches, size_t count, uint64_t *first_ticket,
                   float *kernel_ms, bool wait)
{
    if (!ctx || !first_ticket || (!batches && count)) return fail(-EINVAL, "null argument");
    ctx->svc_call_ns[0] = mono_ns();
    *first_ticket = 0;
    if (kernel_ms) *kernel_ms = 0.0f;
    for (size_t i = 0; i < count; ++i) {
        int rc = svc_check_batch(ctx, batches[i].recs, batches[i].stride, batches[i].n, batches[i].pass_bits);
        if (rc) {
            char why[256];
            snprintf(why, sizeof why, "%s", hfv_last_error());
            return fail(rc, "batch %zu: %s", i, why);
        }
    }
    DeviceGuard g(ctx->device);
    int rc = svc_quiesce(ctx);
    if (rc) return rc;
    DevState *ds;
    ctx->svc_call_ns[1] = mono_ns();
    rc = svc_begin(ctx, ctx->svc_idle_ms, &ds);
    if (rc) return rc;
    ctx->svc_call_ns[2] = mono_ns();
    ctx->svc_adapt = true;   // every batch is in the ring before the grid starts: measure its balance
    ctx->svc_run_ns.resize(count);
    for (size_t i = 0; i < count; ++i) ctx->svc_run_ns[i] = batches[i].n;
    // the batches, then the stop right behind them, are in the ring before the grid starts (a
    // longer run launches once the ring is full): the grid exits as soon as its blocks finish
    // their share of the last batch, with no stop to post and relay afterwards
    bool launched = false;
    for (size_t i = 0; i <= count && !rc; ++i) {
        if (!launched && ctx->svc_next > (uint64_t)kSvcRing) {
            // a run longer than the ring: the grid is launched mid-post, so the phase stamps of
            // this call would mix posting and launching -- they are left at 0 for it
            memset(ctx->svc_call_ns, 0, sizeof ctx->svc_call_ns);
            rc = svc_launch(ctx, ds);
            launched = true;
            if (rc) break;
        }
        if (i == count) {
            rc = svc_post(ctx, 0, 0, kSvcStopN, 0, nullptr);
            ctx->svc_stop_posted = rc == 0;
            break;
        }
        uint64_t t = 0;
        rc = svc_post(ctx, (uint64_t)(uintptr_t)batches[i].recs, (uint64_t)(uintptr_t)batches[i].pass_bits,
                      batches[i].n, batches[i].stride, &t);
        if (i == 0) *first_ticket = t;
    }
    if (!launched) {
        int lr = svc_launch(ctx, ds, ctx->svc_call_ns);
        if (lr) return lr;
        ctx->svc_call_ns[5] = mono_ns();
    }
    if (!wait) return rc;   // the grid exits after the stop posted behind the batches
    int sr = svc_stop(ctx, kernel_ms);
    return rc ? rc : sr;
}

int hfv_service_poll(hfv_ctx *ctx, uint64_t ticket)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    int st = svc_ticket_state(ctx, ticket);
    // A pending ticket of a grid that left without its stop (idle timeout or watchdog: the grid
    // sets the status word in pinned memory first) would never complete: its relay wave stopped
    // forwarding completions when it published the stop.  Only then (a read of pinned memory
    // decides it, no HIP call on the poll path) reap the grid: svc_stop reads the
    // device completion words and records the tickets it left unverified.
    if (st == 0 && ctx->svc_running && __atomic_load_n(&ctx->svc_host->status, __ATOMIC_ACQUIRE) != 0 &&
        hipStreamQuery(ctx->svc_stream) == hipSuccess) {
        DeviceGuard g(ctx->device);
        const int rc = svc_stop(ctx, nullptr);
        // -ETIMEDOUT: the grid left tickets unverified, now recorded as lost (poll reports -EIO for
        // those below).  Any other failure means the lost tickets could not be read: report it rather
        // than fall through to a state that would call them done (fail closed).
        if (rc && rc != -ETIMEDOUT) return rc;
        st = svc_ticket_state(ctx, ticket);
    }
    if (st == -EINVAL) return fail(-EINVAL, "unknown ticket %llu", (unsigned long long)ticket);
    if (st == -EIO) return fail(-EIO, "verify service stopped before ticket %llu", (unsigned long long)ticket);
    return st;
}

int hfv_service_wait(hfv_ctx *ctx, uint64_t ticket, int timeout_ms)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    int st = svc_ticket_state(ctx, ticket);
    if (st == -EINVAL) return fail(-EINVAL, "unknown ticket %llu", (unsigned long long)ticket);
    if (st == -EIO) return fail(-EIO, "verify service stopped before ticket %llu", (unsigned long long)ticket);
    if (st == 1) return 0;
    if (!ctx->svc_running) return fail(-EIO, "verify service stopped before ticket %llu", (unsigned long long)ticket);
    return svc_wait_done(ctx, ticket - ctx->svc_base + 1, timeout_ms);
}

int hfv_service_stop(hfv_ctx *ctx, float *kernel_ms)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    DeviceGuard g(ctx->device);
    return svc_stop(ctx, kernel_ms);
}

int hfv_service_running(const hfv_ctx *ctx) { return ctx && ctx->svc_running ? 1 : 0; }

int hfv_service_set_timing(hfv_ctx *ctx, int enable)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    ctx->svc_timing = enable != 0;
    return 0;
}

int hfv_service_set_grid(hfv_ctx *ctx, int blocks)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    if (blocks < 0) return fail(-EINVAL, "blocks %d < 0", blocks);
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);   // the next grid takes the new shape
    ctx->geom.svc_blocks = blocks == 0 || blocks > ctx->geom.num_cus ? ctx->geom.num_cus : blocks;
    return 0;
}

// Diagnostic (not part of include/scion_hfv.h): the block weights the next service grid will
// use (w[0..7] per XCD, then block 0's), in units of 1/1024 of an equal share.
int hfv_debug_service_weights(hfv_ctx *ctx, uint32_t out[9])
{
    if (!ctx || !out) return fail(-EINVAL, "bad argument");
    for (int x = 0; x < 8; ++x) out[x] = ctx->svc_w.w[x];
    out[8] = ctx->svc_w.w0;
    return 0;
}

// Diagnostic (not part of include/scion_hfv.h): out[i] = s_memrealtime (100 MHz) when block
// 0 loaded ring slot i's descriptor from the mirror (i < kSvcRing; inline batches are not
// loaded); out[kSvcRing .. kSvcRing + 3] = block 0 wave 0's s_memtime and s_memrealtime at its
// start and at its exit (the shader clock over the grid's life); out[kSvcRing + 4 + i] =
// s_memrealtime when the relay published slot i (2 * kSvcRing + 4 words).
int hfv_debug_service_clocks(hfv_ctx *ctx, uint64_t *out)
{
    if (!ctx || !out || !ctx->svc_dev) return fail(-EINVAL, "bad argument");
    static_assert(offsetof(SvcDev, relay) == offsetof(SvcDev, run_clock) + 32, "layout");
    int rc = svc_dev_read(ctx, out, offsetof(SvcDev, load_clock), kSvcRing * 8);
    if (!rc) rc = svc_dev_read(ctx, out + kSvcRing, offsetof(SvcDev, run_clock), 4 * 8);
    if (!rc) rc = svc_dev_read(ctx, out + kSvcRing + 4, offsetof(SvcDev, relay_clock), kSvcRing * 8);
    return rc;
}

// Diagnostic (not part of include/scion_hfv.h): the last grid's per-block stamps: out[0 .. G)
// = s_memrealtime (100 MHz) after the table fill, out[G .. 2G) = at the block's last completed
// share (what svc_balance reads); with words >= 4G also s_memtime (the shader clock) at those two
// points in out[2G .. 3G) and out[3G .. 4G).  Returns G in *grid.
int hfv_debug_service_blocks(hfv_ctx *ctx, uint64_t *out, size_t words, int *grid)
{
    if (!ctx || !out || !grid || !ctx->svc_dev) return fail(-EINVAL, "bad argument");
    const size_t g = ctx->svc_grid;
    if (words < 2 * g) return fail(-EINVAL, "need %zu words", 2 * g);
    *grid = (int)g;
    int rc = svc_dev_read(ctx, out, offsetof(SvcDev, blk_start), g * 8);
    if (!rc) rc = svc_dev_read(ctx, out + g, offsetof(SvcDev, blk_fin), g * 8);
    if (!rc && words >= 4 * g) rc = svc_dev_read(ctx, out + 2 * g, offsetof(SvcDev, blk_clk0), g * 8);
    if (!rc && words >= 4 * g) rc = svc_dev_read(ctx, out + 3 * g, offsetof(SvcDev, blk_clk1), g * 8);
    return rc;
}

// Diagnostic (not part of include/scion_hfv.h): the last grid's relay counters (SvcRelayStat,
// 8 words): the host round trip probed at grid start, host reads and their summed / longest
// round trips (100 MHz ticks), descriptors relayed, completions forwarded, waits of a block for
// a descriptor, descriptors in the kernel arguments.
int hfv_debug_service_relay(hfv_ctx *ctx, uint64_t out[8])
{
    if (!ctx || !out || !ctx->svc_dev) return fail(-EINVAL, "bad argument");
    int rc = svc_dev_read(ctx, out, offsetof(SvcDev, relay), 8 * 8);
    const uint32_t last = ctx->svc_launches ? ctx->svc_launches - 1 : 0;   // the last grid's area
    if (!rc)
        rc = svc_dev_read(ctx, &out[kRelayBlockWaits], offsetof(SvcDev, area) + (last & 1) * sizeof(SvcArea) +
                                                            offsetof(SvcArea, block_waits), 8);
    return rc;
}

// Diagnostic (not part of include/scion_hfv.h): INTEGRATION.md section 2's data-plane loop,
// timed -- per RX batch one hfv_service_submit, then hfv_service_wait on the ticket `depth`
// batches back (a feeder keeping `depth` batches in flight), the last tickets at the end; *ns =
// host nanoseconds from the first submit to the last wait's return.  The same public calls a C
// maintainer writes, without a foreign-function layer in between (bench.py's `per_call` leg).
int hfv_debug_feed_loop(hfv_ctx *ctx, const struct hfv_batch *b, size_t count, uint32_t depth, uint64_t *ns)
{
    if (!ctx || !ns || (!b && count) || depth == 0) return fail(-EINVAL, "bad argument");
    std::vector<uint64_t> t(count);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (size_t i = 0; i < count; ++i) {
        int rc = hfv_service_submit(ctx, b[i].recs, b[i].stride, b[i].n, b[i].pass_bits, &t[i]);
        if (!rc && i >= depth) rc = hfv_service_wait(ctx, t[i - depth], 10000);
        if (rc) return rc;
    }
    for (size_t i = count > depth ? count - depth : 0; i < count; ++i) {
        int rc = hfv_service_wait(ctx, t[i], 10000);
        if (rc) return rc;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *ns = (uint64_t)((t1.tv_sec - t0.tv_sec) * 1000000000ll + (t1.tv_nsec - t0.tv_nsec));
    return 0;
}

// Diagnostic (not part of include/scion_hfv.h): the host-side phases of the last
// hfv_service_run / run_async call in nanoseconds: [0] argument checks and stopping a previous
// grid, [1] the new grid's bookkeeping (svc_begin), [2] posting the batches and building the
// kernel arguments, [3] the launch call itself, [4] the rest (ticket state) to the return.  All 0
// for a call with more batches than the ring holds (its grid is launched mid-post).
int hfv_debug_service_call_ns(hfv_ctx *ctx, uint64_t out[5])
{
    if (!ctx || !out) return fail(-EINVAL, "bad argument");
    const uint64_t *c = ctx->svc_call_ns;
    for (int i = 0; i < 5; ++i) out[i] = c[i + 1] >= c[i] ? c[i + 1] - c[i] : 0;
    return 0;
}

#ifdef HFV_TEST_HOOKS
// Test hook (test build only): every host read of later service grids' relay wave takes `us`
// microseconds longer (a slow PCIe link), 0 = off.
int hfv_debug_relay_delay(uint32_t us)
{
    g_svc_relay_delay_us = us > 100000u ? 100000u : us;
    return 0;
}
#endif

// ---- memory helpers -------------------------------------------------------------------

int hfv_dev_alloc(hfv_ctx *ctx, size_t bytes, void **ptr)
{
    if (!ctx || !ptr) return fail(-EINVAL, "null argument");
    DeviceGuard g(ctx->device);
    if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess) return fail(-ENOMEM, "hipMalloc(%zu)", bytes);
    return 0;
}

int hfv_dev_free(hfv_ctx *ctx, void *ptr)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    HIP_TRY(hipFree(ptr));
    return 0;
}

int hfv_memcpy_h2d(hfv_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

int hfv_memcpy_d2h(hfv_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!ctx) return fail(-EINVAL, "ctx is NULL");
    DeviceGuard g(ctx->device);
    SVC_QUIESCE(ctx);
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // extern "C"
