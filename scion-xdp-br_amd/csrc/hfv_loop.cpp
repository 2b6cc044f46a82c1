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
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

static void pin(int numa_node)
{
    if (numa_node < 0) return;
    char path[128];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", numa_node);
    FILE *f = fopen(path, "r");
    if (!f) return;
    cpu_set_t allowed, cpus;
    CPU_ZERO(&cpus);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) { fclose(f); return; }
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
}

// Ring slot of chunk k: state = 3k (free for chunk k), 3k + 1 (filled), 3k + 2 (processed); the
// consumer of chunk k hands the slot to chunk k + chunks.  Tagging the state with the chunk
// number keeps two producers (or consumers) whose chunks share a slot from both taking it.
struct Chunk {
    std::atomic<uint64_t> state{0};
    size_t n = 0;                     // frames in it
};

}  // namespace

using namespace hfv;

extern "C" int hfv_loop_run(hfv_ctx *ctx, const struct hfv_loop_config *c, struct hfv_loop_stats *out)
{
    if (!ctx || !c || !out || !c->frames || !c->lens || c->n_frames == 0) return fail(-EINVAL, "null argument");
    if (c->slot < 128 || (c->slot & 15) || c->chunk == 0 || c->chunks < 2 || c->total == 0 || c->dma < 0 || c->dma > 2)
        return fail(-EINVAL, "slot must be a multiple of 16 and >= 128, chunk > 0, chunks >= 2, total > 0, dma 0..2");
    for (size_t i = 0; i < c->n_frames; ++i)
        if (c->lens[i] > c->slot || c->lens[i] > c->frame_stride) return fail(-EINVAL, "frame %zu longer than its slot", i);
    memset(out, 0, sizeof *out);
    const size_t nslots = c->chunk * c->chunks;
    const int producers = c->producers > 0 ? c->producers : 1, consumers = c->consumers > 0 ? c->consumers : 1;
    // the RX ring and the per-frame metadata in pinned, mapped host memory: the kernel reads
    // and writes them in place (zero-copy), or the DMA engines copy them (dma = 1: both ways;
    // dma = 2: in only, the kernel writing its changes back into the ring)
    int rc = br_zc_prepare(ctx);   // stops a running service; the ctx's device is current
    if (rc) return rc;
    const size_t ring_bytes = (nslots * c->slot + 4095) & ~(size_t)4095;
    const size_t meta_bytes = (nslots * 16 + 4095) & ~(size_t)4095;
    uint8_t *ring = nullptr, *meta = nullptr, *dring = nullptr, *dmeta = nullptr;
    if (hipHostMalloc((void **)&ring, ring_bytes, hipHostMallocMapped) != hipSuccess ||
        hipHostMalloc((void **)&meta, meta_bytes, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&dring, ring, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&dmeta, meta, 0) != hipSuccess) {
        if (ring) (void)hipHostFree(ring);
        if (meta) (void)hipHostFree(meta);
        return fail(-ENOMEM, "loop: pinned ring allocation");
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
    const int node = hfv_ctx_numa_node(ctx);
    std::vector<Chunk> ch(c->chunks);
    for (size_t i = 0; i < c->chunks; ++i) ch[i].state.store(3 * i);
    const uint64_t nchunks_total = (c->total + c->chunk - 1) / c->chunk;
    std::atomic<bool> abort{false};

    // producers: chunk k by producer k % P (tcpreplay --loop of the frame list)
    std::vector<double> busy(producers, 0.0);
    auto produce = [&](int p) {
        pin(node);
        for (uint64_t k = (uint64_t)p; k < nchunks_total && !abort.load(std::memory_order_relaxed); k += producers) {
            Chunk &cc = ch[k % c->chunks];
            for (unsigned spins = 0; cc.state.load(std::memory_order_acquire) != 3 * k; relax(spins))
                if (abort.load(std::memory_order_relaxed)) return;
            const double tb = now_s();
            const size_t sl = k % c->chunks, base = sl * C;
            uint16_t *len = len_of(sl);
            uint32_t *ifx = ifx_of(sl);
            const uint64_t first = k * C;
            const size_t n = (size_t)(c->total - first < C ? c->total - first : C);
            for (size_t i = 0; i < n; ++i) {
                const size_t f = (size_t)((first + i) % c->n_frames);
                memcpy(ring + (base + i) * c->slot, c->frames + f * c->frame_stride, c->lens[f]);
                len[i] = c->lens[f];
                ifx[i] = c->rx_ifindex;
            }
            cc.n = n;
            busy[p] += now_s() - tb;
            cc.state.store(3 * k + 1, std::memory_order_release);
        }
    };
    // consumers: transmit redirected frames (digest + byte count per egress), drop the rest
    std::vector<hfv_loop_stats> part(consumers);
    auto consume = [&](int q) {
        pin(node);
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
    static const int split_env = getenv("HFV_LOOP_SPLIT") ? atoi(getenv("HFV_LOOP_SPLIT")) : 1;
    const bool split = c->dma == 2 && split_env;
    uint64_t *dstats = nullptr;
    const size_t stats_bytes = HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS * 8;
    for (int i = 0; i < D && !rc; ++i) {
        if (hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
            rc = fail(-EIO, "loop: stream/event creation failed");
        if (!rc && split &&
            (hipStreamCreateWithFlags(&ss2[i], hipStreamNonBlocking) != hipSuccess ||
             hipEventCreateWithFlags(&ev2[i], hipEventDisableTiming) != hipSuccess))
            rc = fail(-EIO, "loop: stream/event creation failed");
    }
    std::vector<uint8_t *> dfr(D, nullptr), dmt(D, nullptr);   // DMA variant: device twin per stream
    for (int i = 0; i < D && !rc && c->dma; ++i)
        if (hipMalloc((void **)&dfr[i], C * c->slot) != hipSuccess || hipMalloc((void **)&dmt[i], C * 16) != hipSuccess)
            rc = fail(-ENOMEM, "loop: device chunk buffers");
    if (!rc && c->stats && (hipMalloc((void **)&dstats, stats_bytes) != hipSuccess ||
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
    (void)hipHostFree(ring);
    (void)hipHostFree(meta);
    return rc;
}
