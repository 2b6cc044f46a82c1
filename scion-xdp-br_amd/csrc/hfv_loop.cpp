// hfv_loop.cpp -- config 5's end-to-end loop in one process: an RX ring in host memory fed by
// producer threads (the NIC / veth side: tcpreplay of gen_packets.py's frames,
// br/evaluation/gen_packets.py:41-71, README.md:131-139), the border router on the GPU
// (the router kernel zero-copy: it reads the header windows of the pinned, mapped ring
// over PCIe and writes the rewritten rows back), and consumer threads on the TX side that
// transmit redirected frames and drop the rest while counting them (count_and_drop.py).
//
// The ring is `chunks` chunks of `chunk` frame slots.  A chunk moves free -> filled (a
// producer copied frames into it) -> processed (the GPU stage ran the router over it) ->
// free (a consumer read the verdicts and the transmitted frames), each stage on its own
// threads, so producer, GPU and consumer work on different chunks at once.  Producer and
// consumer threads run on the CPUs of the GPU's NUMA node.
#include <arpa/inet.h>
#include <errno.h>
#include <linux/if_packet.h>
#include <net/ethernet.h>
#include <net/if.h>
#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "hfv_internal.h"

namespace {

// Order-independent digest of a transmitted frame (with its egress port): the test compares
// the sum over all transmitted frames with the oracle's.
static uint64_t frame_hash(const uint8_t *p, size_t n, int32_t egress)
{
    uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)(uint32_t)egress << 32) ^ n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
        h ^= h >> 29;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = (h ^ w) * 0x94D049BB133111EBull;
    return h ^ (h >> 31);
}

// Wait politely: spin briefly, then sleep in short steps (the box's CPU share is a quota; a
// dozen threads spinning flat out get the whole process throttled).
static void relax(unsigned &spins)
{
    if (++spins < 256) {
        __builtin_ia32_pause();
        return;
    }
    struct timespec ts = {0, 20000};
    nanosleep(&ts, nullptr);
}

static double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// Pin the calling thread to the CPUs of `numa_node` it may use; returns that set (empty when the
// node is unknown or none of its CPUs is allowed: the thread then stays where it was).
static cpu_set_t pin(int numa_node)
{
    cpu_set_t allowed, cpus;
    CPU_ZERO(&cpus);
    if (numa_node < 0) return cpus;
    char path[128];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", numa_node);
    FILE *f = fopen(path, "r");
    if (!f) return cpus;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) { fclose(f); return cpus; }
    int a, b;
    char sep = 0;
    while (fscanf(f, "%d", &a) == 1) {
        b = a;
        if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
            if (fscanf(f, "%d", &b) != 1) break;
            if (fscanf(f, "%c", &sep) != 1) sep = 0;
        }
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &allowed)) CPU_SET(c, &cpus);
        if (sep != ',') break;
    }
    fclose(f);
    if (CPU_COUNT(&cpus) > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof cpus, &cpus);
    return cpus;
}

// The thread runs on a CPU of `cpus` now (checked where a thread ends its work).
static bool on_node(const cpu_set_t &cpus)
{
    const int cpu = sched_getcpu();
    return CPU_COUNT(&cpus) > 0 && cpu >= 0 && CPU_ISSET(cpu, &cpus);
}

// ---- packet sockets (the evaluation's veth ends) ---------------------------------------------
// One AF_PACKET socket per side, bound to its interface: RX shared by the producer threads
// (recvmmsg straight into ring slots), TX shared by the consumers (sendmmsg from ring slots).
static int packet_socket(const char *ifname, bool rx, int *out)
{
    const unsigned idx = if_nametoindex(ifname);
    if (!idx) return -ENODEV;
    const int fd = socket(AF_PACKET, SOCK_RAW, rx ? htons(ETH_P_ALL) : 0);
    if (fd < 0) return -errno;
    struct sockaddr_ll a;
    memset(&a, 0, sizeof a);
    a.sll_family = AF_PACKET;
    a.sll_protocol = rx ? htons(ETH_P_ALL) : 0;
    a.sll_ifindex = (int)idx;
    if (bind(fd, (struct sockaddr *)&a, sizeof a) != 0) {
        const int e = -errno;
        close(fd);
        return e;
    }
    if (rx) {
#ifdef PACKET_IGNORE_OUTGOING
        int one = 1;   // only frames arriving on the interface, not ones sent from it
        (void)setsockopt(fd, SOL_PACKET, PACKET_IGNORE_OUTGOING, &one, sizeof one);
#endif
        int buf = 64 << 20;   // a burst of a few hundred thousand frames
        if (setsockopt(fd, SOL_SOCKET, SO_RCVBUFFORCE, &buf, sizeof buf) != 0)
            (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
    }
    *out = fd;
    return 0;
}

static double mono_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// Ring slot of chunk k: state = 3k (free for chunk k), 3k + 1 (filled), 3k + 2 (processed); the
// consumer of chunk k hands the slot to chunk k + chunks.  Tagging the state with the chunk
// number keeps two producers (or consumers) whose chunks share a slot from both taking it.
struct Chunk {
    std::atomic<uint64_t> state{0};
    size_t n = 0;                     // frames in it
};

// Test-only router stage on the host (hfv_debug_loop_host_stage, in the test build
// lib/libscionhfv_test.so only): with it set, hfv_loop_run takes no ctx, keeps the ring in
// ordinary memory and calls the function on each filled chunk in place of the kernel, so the
// ring, the threads and the packet-socket I/O run on a machine without a GPU
// (tests/test_loop_pktio.py drives them over veth pairs with the oracle router).  The product
// library has no such seam: its router stage is always the kernel.
#ifdef HFV_TEST_HOOKS
static hfv::hfv_loop_host_stage_fn g_host_stage = nullptr;
static void *g_host_stage_user = nullptr;
#else
static constexpr hfv::hfv_loop_host_stage_fn g_host_stage = nullptr;
static constexpr void *g_host_stage_user = nullptr;
#endif

}  // namespace

using namespace hfv;

#ifdef HFV_TEST_HOOKS
extern "C" int hfv_debug_loop_host_stage(hfv::hfv_loop_host_stage_fn fn, void *user)
{
    g_host_stage = fn;
    g_host_stage_user = user;
    return 0;
}
#endif

extern "C" int hfv_loop_run(hfv_ctx *ctx, const struct hfv_loop_config *c, struct hfv_loop_stats *out)
{
    const hfv::hfv_loop_host_stage_fn host_stage = g_host_stage;
    void *const host_user = g_host_stage_user;
    const bool pkt_rx = c && c->rx_ifname, pkt_tx = c && c->tx_ifname;
    if ((!ctx && !host_stage) || !c || !out || (!pkt_rx && (!c->frames || !c->lens || c->n_frames == 0)))
        return fail(-EINVAL, "null argument");
    if (c->slot < 128 || (c->slot & 15) || c->chunk == 0 || c->chunks < 2 || c->total == 0 || c->dma < 0 || c->dma > 2)
        return fail(-EINVAL, "slot must be a multiple of 16 and >= 128, chunk > 0, chunks >= 2, total > 0, dma 0..2");
    for (size_t i = 0; !pkt_rx && i < c->n_frames; ++i)
        if (c->lens[i] > c->slot || c->lens[i] > c->frame_stride) return fail(-EINVAL, "frame %zu longer than its slot", i);
    memset(out, 0, sizeof *out);
    const size_t nslots = c->chunk * c->chunks;
    const int producers = c->producers > 0 ? c->producers : 1, consumers = c->consumers > 0 ? c->consumers : 1;
    int rx_fd = -1, tx_fd = -1, rc = 0;
    if (pkt_rx && (rc = packet_socket(c->rx_ifname, true, &rx_fd)) != 0)
        return fail(rc, "loop: AF_PACKET socket on %s: %s", c->rx_ifname, strerror(-rc));
    if (pkt_tx && (rc = packet_socket(c->tx_ifname, false, &tx_fd)) != 0) {
        if (rx_fd >= 0) close(rx_fd);
        return fail(rc, "loop: AF_PACKET socket on %s: %s", c->tx_ifname, strerror(-rc));
    }
    auto close_sockets = [&]() {
        if (rx_fd >= 0) close(rx_fd);
        if (tx_fd >= 0) close(tx_fd);
    };
    // the RX ring and the per-frame metadata in pinned, mapped host memory: the kernel reads
    // and writes them in place (zero-copy), or the DMA engines copy them (dma = 1: both ways;
    // dma = 2: in only, the kernel writing its changes back into the ring)
    const size_t ring_bytes = (nslots * c->slot + 4095) & ~(size_t)4095;
    const size_t meta_bytes = (nslots * 16 + 4095) & ~(size_t)4095;
    uint8_t *ring = nullptr, *meta = nullptr, *dring = nullptr, *dmeta = nullptr;
    if (host_stage) {
        ring = (uint8_t *)aligned_alloc(4096, ring_bytes);
        meta = (uint8_t *)aligned_alloc(4096, meta_bytes);
        if (!ring || !meta) {
            free(ring);
            free(meta);
            close_sockets();
            return fail(-ENOMEM, "loop: ring allocation");
        }
    } else {
        rc = br_zc_prepare(ctx);   // stops a running service; the ctx's device is current
        if (rc) {
            close_sockets();
            return rc;
        }
        if (hipHostMalloc((void **)&ring, ring_bytes, hipHostMallocMapped) != hipSuccess ||
            hipHostMalloc((void **)&meta, meta_bytes, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void **)&dring, ring, 0) != hipSuccess ||
            hipHostGetDevicePointer((void **)&dmeta, meta, 0) != hipSuccess) {
            if (ring) (void)hipHostFree(ring);
            if (meta) (void)hipHostFree(meta);
            close_sockets();
            return fail(-ENOMEM, "loop: pinned ring allocation");
        }
    }
    memset(meta, 0, meta_bytes);
    // per-frame metadata, chunk by chunk: len u16 (in a 4 B/frame field) | ingress ifindex u32 |
    // egress i32 | action u8 | verdict u8, so each chunk's inputs and outputs are one contiguous range each
    const size_t C = c->chunk;
    auto len_of = [&](size_t s) { return (uint16_t *)(meta + s * C * 16); };
    auto ifx_of = [&](size_t s) { return (uint32_t *)(meta + s * C * 16 + C * 4); };
    auto egr_of = [&](size_t s) { return (int32_t *)(meta + s * C * 16 + C * 8); };
    auto act_of = [&](size_t s) { return meta + s * C * 16 + C * 12; };
    auto ver_of = [&](size_t s) { return meta + s * C * 16 + C * 13; };
    const int node = ctx ? hfv_ctx_numa_node(ctx) : -1;
    std::vector<Chunk> ch(c->chunks);
    for (size_t i = 0; i < c->chunks; ++i) ch[i].state.store(3 * i);
    const uint64_t nchunks_total = (c->total + c->chunk - 1) / c->chunk;
    std::atomic<bool> abort{false};
    // packet RX: the time of the last frame received (or of the start) and the end of input
    const double idle_s = (c->idle_ms > 0 ? c->idle_ms : 1000) * 1e-3;
    std::atomic<double> last_rx{mono_s()};
    std::atomic<bool> rx_done{false};
    std::atomic<uint64_t> rx_trunc{0}, tx_err{0};
    // Fill up to n slots from the RX socket; returns the frames received (fewer once the input
    // has been idle for idle_s, which ends the input for every producer).
    auto receive = [&](size_t base, size_t n, uint16_t *len, uint32_t *ifx) -> size_t {
        constexpr size_t kBatch = 64;
        struct mmsghdr mm[kBatch];
        struct iovec iov[kBatch];
        size_t got = 0;
        while (got < n && !rx_done.load(std::memory_order_relaxed) && !abort.load(std::memory_order_relaxed)) {
            struct pollfd pf = {rx_fd, POLLIN, 0};
            if (poll(&pf, 1, 5) <= 0) {
                if (mono_s() - last_rx.load(std::memory_order_relaxed) > idle_s) rx_done.store(true);
                continue;
            }
            const size_t want = n - got < kBatch ? n - got : kBatch;
            for (size_t j = 0; j < want; ++j) {
                iov[j].iov_base = ring + (base + got + j) * c->slot;
                iov[j].iov_len = c->slot;
                memset(&mm[j], 0, sizeof mm[j]);
                mm[j].msg_hdr.msg_iov = &iov[j];
                mm[j].msg_hdr.msg_iovlen = 1;
            }
            const int r = recvmmsg(rx_fd, mm, (unsigned)want, MSG_DONTWAIT | MSG_TRUNC, nullptr);
            if (r <= 0) continue;
            last_rx.store(mono_s(), std::memory_order_relaxed);
            // keep the frames that fit a slot, packed in arrival order
            size_t kept = 0;
            for (int j = 0; j < r; ++j) {
                const size_t l = mm[j].msg_len;
                if (l > c->slot || (mm[j].msg_hdr.msg_flags & MSG_TRUNC)) {
                    rx_trunc.fetch_add(1);
                    continue;
                }
                if (kept != (size_t)j) memmove(ring + (base + got + kept) * c->slot, ring + (base + got + j) * c->slot, l);
                len[got + kept] = (uint16_t)l;
                ifx[got + kept] = c->rx_ifindex;
                ++kept;
            }
            got += kept;
        }
        return got;
    };
    // Send the redirected frames of a chunk out of the TX socket, in batches.
    auto transmit = [&](size_t base, size_t n, const uint16_t *len, const uint8_t *act) {
        constexpr size_t kBatch = 64;
        struct mmsghdr mm[kBatch];
        struct iovec iov[kBatch];
        size_t m = 0;
        auto flush = [&]() {
            size_t sent = 0;
            for (int tries = 0; sent < m && tries < 64; ++tries) {
                const int r = sendmmsg(tx_fd, mm + sent, (unsigned)(m - sent), 0);
                if (r > 0) {
                    sent += (size_t)r;
                } else {
                    struct timespec ts = {0, 20000};   // ENOBUFS: the device queue is full
                    nanosleep(&ts, nullptr);
                }
            }
            if (sent < m) tx_err.fetch_add(m - sent);
            m = 0;
        };
        for (size_t i = 0; i < n; ++i) {
            if (act[i] != 4) continue;
            iov[m].iov_base = ring + (base + i) * c->slot;
            iov[m].iov_len = len[i];
            memset(&mm[m], 0, sizeof mm[m]);
            mm[m].msg_hdr.msg_iov = &iov[m];
            mm[m].msg_hdr.msg_iovlen = 1;
            if (++m == kBatch) flush();
        }
        if (m) flush();
    };

    // producers: chunk k by producer k % P (tcpreplay --loop of the frame list)
    std::vector<double> busy(producers, 0.0);
    std::atomic<uint32_t> threads_on_node{0};
    auto produce = [&](int p) {
        const cpu_set_t mine = pin(node);
        struct Check {   // counts the thread as on its GPU's node if it ends its work there
            const cpu_set_t &m;
            std::atomic<uint32_t> &n;
            ~Check() { if (on_node(m)) n.fetch_add(1); }
        } check{mine, threads_on_node};
        for (uint64_t k = (uint64_t)p; k < nchunks_total && !abort.load(std::memory_order_relaxed); k += producers) {
            Chunk &cc = ch[k % c->chunks];
            for (unsigned spins = 0; cc.state.load(std::memory_order_acquire) != 3 * k; relax(spins))
                if (abort.load(std::memory_order_relaxed)) return;
            const double tb = now_s();
            const size_t sl = k % c->chunks, base = sl * C;
            uint16_t *len = len_of(sl);
            uint32_t *ifx = ifx_of(sl);
            const uint64_t first = k * C;
            size_t n = (size_t)(c->total - first < C ? c->total - first : C);
            if (pkt_rx) {
                n = receive(base, n, len, ifx);   // fewer (or none) once the input went idle
            } else {
                for (size_t i = 0; i < n; ++i) {
                    const size_t f = (size_t)((first + i) % c->n_frames);
                    memcpy(ring + (base + i) * c->slot, c->frames + f * c->frame_stride, c->lens[f]);
                    len[i] = c->lens[f];
                    ifx[i] = c->rx_ifindex;
                }
            }
            cc.n = n;
            busy[p] += now_s() - tb;
            cc.state.store(3 * k + 1, std::memory_order_release);
        }
    };
    // consumers: transmit redirected frames (digest + byte count per egress), drop the rest
    std::vector<hfv_loop_stats> part(consumers);
    auto consume = [&](int q) {
        const cpu_set_t mine = pin(node);
        struct Check {
            const cpu_set_t &m;
            std::atomic<uint32_t> &n;
            ~Check() { if (on_node(m)) n.fetch_add(1); }
        } check{mine, threads_on_node};
        hfv_loop_stats &s = part[q];
        memset(&s, 0, sizeof s);
        for (uint64_t k = (uint64_t)q; k < nchunks_total && !abort.load(std::memory_order_relaxed); k += consumers) {
            Chunk &cc = ch[k % c->chunks];
            for (unsigned spins = 0; cc.state.load(std::memory_order_acquire) != 3 * k + 2; relax(spins))
                if (abort.load(std::memory_order_relaxed)) return;
            const double tb = now_s();
            const size_t sl = k % c->chunks, base = sl * C;
            const uint16_t *len = len_of(sl);
            const int32_t *egr = egr_of(sl);
            const uint8_t *act = act_of(sl), *ver = ver_of(sl);
            for (size_t i = 0; i < cc.n; ++i) {
                s.rx_pkts++;
                if ((ver[i] >> 3) < HFV_BR_COUNTERS) s.verdict_pkts[ver[i] >> 3]++;   // enum verdict: counter << 3 | code
                if (act[i] == 4) {   // XDP_REDIRECT to egr[i]
                    s.tx_pkts++;
                    s.tx_bytes += len[i];
                    if (c->digest) s.tx_digest += frame_hash(ring + (base + i) * c->slot, len[i], egr[i]);
                } else {
                    s.drop_pkts++;
                }
            }
            if (pkt_tx) transmit(base, cc.n, len, act);
            s.consumer_busy_s += now_s() - tb;
            cc.state.store(3 * (k + c->chunks), std::memory_order_release);
        }
    };
    // the GPU stage: the router over each filled chunk, in ring order, `inflight` chunks at once
    // on their own streams (a chunk is a few hundred microseconds of PCIe-bound kernel; the
    // launch and completion wait of one overlap the others)
    const int D = c->inflight > 0 ? (c->inflight < (int)c->chunks ? c->inflight : (int)c->chunks) : 2;
    std::vector<hipStream_t> ss(D, nullptr), ss2(D, nullptr);
    std::vector<hipEvent_t> ev(D, nullptr), ev2(D, nullptr);
    // DMA in: each chunk's frame copy goes out in two halves on two streams (HIP gives each stream
    // its own copy-engine queue, and one engine does not fill the link: with a chunk on one
    // stream, runs landed at 166-172 or 213-265 Mpkt/s depending on the engines the streams got)
    const bool split = c->dma == 2;
    uint64_t *dstats = nullptr;
    const size_t stats_bytes = HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS * 8;
    for (int i = 0; i < D && !rc && !host_stage; ++i) {
        if (hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
            rc = fail(-EIO, "loop: stream/event creation failed");
        if (!rc && split &&
            (hipStreamCreateWithFlags(&ss2[i], hipStreamNonBlocking) != hipSuccess ||
             hipEventCreateWithFlags(&ev2[i], hipEventDisableTiming) != hipSuccess))
            rc = fail(-EIO, "loop: stream/event creation failed");
    }
    std::vector<uint8_t *> dfr(D, nullptr), dmt(D, nullptr);   // DMA variant: device twin per stream
    for (int i = 0; i < D && !rc && c->dma && !host_stage; ++i)
        if (hipMalloc((void **)&dfr[i], C * c->slot) != hipSuccess || hipMalloc((void **)&dmt[i], C * 16) != hipSuccess)
            rc = fail(-ENOMEM, "loop: device chunk buffers");
    if (!rc && c->stats && !host_stage && (hipMalloc((void **)&dstats, stats_bytes) != hipSuccess ||
                            hipMemset(dstats, 0, stats_bytes) != hipSuccess))
        rc = fail(-ENOMEM, "loop: device counters");
    // streams, events and device buffers before the clock starts; the threads only when they are there
    std::vector<std::thread> th;
    const double t0 = now_s();
    for (int p = 0; p < producers && !rc; ++p) th.emplace_back(produce, p);
    for (int q = 0; q < consumers && !rc; ++q) th.emplace_back(consume, q);
    double gpu_busy = 0, gpu_wait = 0;
    uint64_t launched = 0, retired = 0;
    // hand finished chunks to the consumers, in order: one (waiting for it) or all that are done
    auto retire = [&](bool block) {
        while (retired < launched) {
            hipEvent_t e = ev[retired % D];
            if (block) {
                if (hipEventSynchronize(e) != hipSuccess) rc = fail(-EIO, "loop: router kernel failed");
            } else if (hipEventQuery(e) != hipSuccess) {
                return;
            }
            if (rc) return;
            ch[retired % c->chunks].state.store(3 * retired + 2, std::memory_order_release);
            ++retired;
            if (block) return;
        }
    };
    for (uint64_t k = 0; k < nchunks_total && !rc; ++k) {
        Chunk &cc = ch[k % c->chunks];
        const double tw = now_s();
        for (unsigned spins = 0; cc.state.load(std::memory_order_acquire) != 3 * k + 1; relax(spins)) retire(false);
        const double tb = now_s();
        while (!rc && launched - retired >= (uint64_t)D) retire(true);   // its stream's previous chunk
        if (rc) break;
        const size_t sl = k % c->chunks;
        uint8_t *fr = ring + sl * C * c->slot, *cm = meta + sl * C * 16;
        const int q = (int)(k % D);
        if (host_stage) {   // test-only host router stage: synchronous, in ring order
            if (cc.n && host_stage(host_user, fr, c->slot, (const uint16_t *)cm, (const uint32_t *)(cm + C * 4), cc.n,
                                   cm + C * 12, cm + C * 13, (int32_t *)(cm + C * 8)) != 0)
                rc = fail(-EIO, "loop: host stage failed");
            if (!rc) ch[sl].state.store(3 * k + 2, std::memory_order_release);
            ++launched;
            ++retired;
            gpu_wait += tb - tw;
            gpu_busy += now_s() - tb;
            continue;
        }
        if (cc.n == 0) {   // packet input ended before this chunk: nothing to route
            while (!rc && retired < launched) retire(true);
            if (!rc) ch[sl].state.store(3 * k + 2, std::memory_order_release);
            ++launched;
            ++retired;
            continue;
        }
        if (!c->dma) {   // the kernel on the mapped ring (device addresses of the same pages)
            uint8_t *dfr_zc = dring + sl * C * c->slot, *dm = dmeta + sl * C * 16;
            rc = br_dev_launch(ctx, ss[q], dfr_zc, c->slot, (uint16_t *)dm, (uint32_t *)(dm + C * 4), cc.n, dm + C * 12,
                               dm + C * 13, (int32_t *)(dm + C * 8), dstats);
        } else if (c->dma == 1) {   // frames and inputs in by DMA, the router in HBM, frames and outputs back by DMA
            uint8_t *m = dmt[q];
            if (hipMemcpyAsync(dfr[q], fr, cc.n * c->slot, hipMemcpyHostToDevice, ss[q]) != hipSuccess ||
                hipMemcpyAsync(m, cm, C * 8, hipMemcpyHostToDevice, ss[q]) != hipSuccess)
                rc = fail(-EIO, "loop: H2D copy");
            if (!rc)
                rc = br_dev_launch(ctx, ss[q], dfr[q], c->slot, (uint16_t *)m, (uint32_t *)(m + C * 4), cc.n, m + C * 12,
                                   m + C * 13, (int32_t *)(m + C * 8), dstats);
            if (!rc && (hipMemcpyAsync(fr, dfr[q], cc.n * c->slot, hipMemcpyDeviceToHost, ss[q]) != hipSuccess ||
                        hipMemcpyAsync(cm + C * 8, m + C * 8, C * 6, hipMemcpyDeviceToHost, ss[q]) != hipSuccess))
                rc = fail(-EIO, "loop: D2H copy");
        } else {   // frames and inputs in by DMA; the router reads HBM and writes only the bytes it
                   // changes, and its outputs, straight into the mapped ring (no copy back)
            uint8_t *m = dmt[q], *dfr_zc = dring + sl * C * c->slot, *dm = dmeta + sl * C * 16;
            const size_t half = split ? cc.n / 2 * c->slot : 0, all = cc.n * c->slot;
            if (split && (hipStreamWaitEvent(ss2[q], ev[q], 0) != hipSuccess ||   // its previous kernel is done with dfr[q]
                          hipMemcpyAsync(dfr[q] + half, fr + half, all - half, hipMemcpyHostToDevice, ss2[q]) != hipSuccess ||
                          hipEventRecord(ev2[q], ss2[q]) != hipSuccess))
                rc = fail(-EIO, "loop: H2D copy");
            if (!rc && (hipMemcpyAsync(dfr[q], fr, split ? half : all, hipMemcpyHostToDevice, ss[q]) != hipSuccess ||
                        hipMemcpyAsync(m, cm, C * 8, hipMemcpyHostToDevice, ss[q]) != hipSuccess ||
                        (split && hipStreamWaitEvent(ss[q], ev2[q], 0) != hipSuccess)))
                rc = fail(-EIO, "loop: H2D copy");
            if (!rc)
                rc = br_dev_launch(ctx, ss[q], dfr[q], c->slot, (uint16_t *)m, (uint32_t *)(m + C * 4), cc.n, dm + C * 12,
                                   dm + C * 13, (int32_t *)(dm + C * 8), dstats, dfr_zc);
        }
        if (!rc && hipEventRecord(ev[q], ss[q]) != hipSuccess) rc = fail(-EIO, "loop: event record failed");
        if (!rc) ++launched;
        retire(false);
        gpu_wait += tb - tw;
        gpu_busy += now_s() - tb;
    }
    while (!rc && retired < launched) retire(true);
    if (!rc && dstats) {
        std::vector<uint64_t> tmp(stats_bytes / 8);
        if (hipMemcpy(tmp.data(), dstats, stats_bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = fail(-EIO, "loop: counters");
        else
            for (size_t i = 0; i < tmp.size(); ++i) c->stats[i] += tmp[i];
    }
    if (rc) abort.store(true);
    for (auto &t : th) t.join();
    out->rx_truncated = rx_trunc.load();
    out->numa_node = node;
    out->threads = (uint32_t)(producers + consumers);
    out->threads_on_node = threads_on_node.load();
    out->tx_errors = tx_err.load();
    close_sockets();
    const double t1 = now_s();
    out->seconds = t1 - t0;
    out->gpu_busy_s = gpu_busy;
    out->gpu_wait_s = gpu_wait;
    for (int p = 0; p < producers; ++p) out->producer_busy_s += busy[p];
    for (int q = 0; q < consumers; ++q) {
        out->rx_pkts += part[q].rx_pkts;
        out->tx_pkts += part[q].tx_pkts;
        out->tx_bytes += part[q].tx_bytes;
        out->drop_pkts += part[q].drop_pkts;
        out->tx_digest += part[q].tx_digest;
        for (int v = 0; v < HFV_BR_COUNTERS; ++v) out->verdict_pkts[v] += part[q].verdict_pkts[v];
        out->consumer_busy_s += part[q].consumer_busy_s;
    }
    for (int i = 0; i < D; ++i) {
        if (ss[i]) {
            (void)hipStreamSynchronize(ss[i]);
            forget_stream(ctx, ss[i]);
            (void)hipStreamDestroy(ss[i]);
        }
        if (ev[i]) (void)hipEventDestroy(ev[i]);
        if (ss2[i]) {
            (void)hipStreamSynchronize(ss2[i]);
            (void)hipStreamDestroy(ss2[i]);
        }
        if (ev2[i]) (void)hipEventDestroy(ev2[i]);
    }
    if (dstats) (void)hipFree(dstats);
    for (int i = 0; i < D; ++i) {
        if (dfr[i]) (void)hipFree(dfr[i]);
        if (dmt[i]) (void)hipFree(dmt[i]);
    }
    if (host_stage) {
        free(ring);
        free(meta);
    } else {
        (void)hipHostFree(ring);
        (void)hipHostFree(meta);
    }
    return rc;
}
