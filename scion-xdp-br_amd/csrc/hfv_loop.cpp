// hfv_loop.cpp -- config 5's end-to-end loop in one process: an RX ring in host memory fed by
// producer threads (the NIC / veth side: tcpreplay of gen_packets.py's frames,
// br/evaluation/gen_packets.py:41-71, README.md:131-139), the border router on the GPU
// (hfv_br_process_host, zero-copy: the kernel reads the header windows of the registered ring
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

struct Chunk {
    std::atomic<uint32_t> state{0};   // 0 free, 1 filled, 2 processed
    uint64_t seq = 0;                 // first frame number in it
    size_t n = 0;                     // frames in it
};

}  // namespace

using namespace hfv;

extern "C" int hfv_loop_run(hfv_ctx *ctx, const struct hfv_loop_config *c, struct hfv_loop_stats *out)
{
    if (!ctx || !c || !out || !c->frames || !c->lens || c->n_frames == 0) return fail(-EINVAL, "null argument");
    if (c->slot < 64 || (c->slot & 63) || c->chunk == 0 || c->chunks < 2 || c->total == 0)
        return fail(-EINVAL, "slot must be a multiple of 64, chunk > 0, chunks >= 2, total > 0");
    for (size_t i = 0; i < c->n_frames; ++i)
        if (c->lens[i] > c->slot || c->lens[i] > c->frame_stride) return fail(-EINVAL, "frame %zu longer than its slot", i);
    memset(out, 0, sizeof *out);
    const size_t nslots = c->chunk * c->chunks;
    const int producers = c->producers > 0 ? c->producers : 1, consumers = c->consumers > 0 ? c->consumers : 1;
    // the RX ring and the per-frame metadata, registered so the kernel reads and writes them in place
    uint8_t *ring = (uint8_t *)aligned_alloc(4096, (nslots * c->slot + 4095) & ~(size_t)4095);
    const size_t meta_bytes = (nslots * 16 + 4095) & ~(size_t)4095;
    uint8_t *meta = (uint8_t *)aligned_alloc(4096, meta_bytes);
    if (!ring || !meta) {
        free(ring);
        free(meta);
        return fail(-ENOMEM, "ring allocation");
    }
    memset(meta, 0, meta_bytes);
    uint16_t *len = (uint16_t *)meta;
    uint32_t *ifx = (uint32_t *)(meta + nslots * 4);
    int32_t *egr = (int32_t *)(meta + nslots * 8);
    uint8_t *act = meta + nslots * 12, *ver = meta + nslots * 13;
    int rc = hfv_host_register(ctx, ring, (nslots * c->slot + 4095) & ~(size_t)4095);
    if (!rc) {
        rc = hfv_host_register(ctx, meta, meta_bytes);
        if (rc) hfv_host_unregister(ctx, ring);
    }
    if (rc) {
        free(ring);
        free(meta);
        return rc;
    }
    const int node = hfv_ctx_numa_node(ctx);
    std::vector<Chunk> ch(c->chunks);
    const uint64_t nchunks_total = (c->total + c->chunk - 1) / c->chunk;
    std::atomic<bool> abort{false};

    // producers: chunk k by producer k % P (tcpreplay --loop of the frame list)
    auto produce = [&](int p) {
        pin(node);
        for (uint64_t k = (uint64_t)p; k < nchunks_total && !abort.load(std::memory_order_relaxed); k += producers) {
            Chunk &cc = ch[k % c->chunks];
            while (cc.state.load(std::memory_order_acquire) != 0)
                if (abort.load(std::memory_order_relaxed)) return;
            const size_t base = (k % c->chunks) * c->chunk;
            const uint64_t first = k * c->chunk;
            const size_t n = (size_t)(c->total - first < c->chunk ? c->total - first : c->chunk);
            for (size_t i = 0; i < n; ++i) {
                const size_t f = (size_t)((first + i) % c->n_frames);
                memcpy(ring + (base + i) * c->slot, c->frames + f * c->frame_stride, c->lens[f]);
                len[base + i] = c->lens[f];
                ifx[base + i] = c->rx_ifindex;
            }
            cc.seq = first;
            cc.n = n;
            cc.state.store(1, std::memory_order_release);
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
            while (cc.state.load(std::memory_order_acquire) != 2)
                if (abort.load(std::memory_order_relaxed)) return;
            const size_t base = (k % c->chunks) * c->chunk;
            for (size_t i = 0; i < cc.n; ++i) {
                const size_t j = base + i;
                s.rx_pkts++;
                if ((ver[j] >> 3) < HFV_BR_COUNTERS) s.verdict_pkts[ver[j] >> 3]++;   // enum verdict: counter << 3 | code
                if (act[j] == 4) {   // XDP_REDIRECT to egr[j]
                    s.tx_pkts++;
                    s.tx_bytes += len[j];
                    if (c->digest) s.tx_digest += frame_hash(ring + j * c->slot, len[j], egr[j]);
                } else {
                    s.drop_pkts++;
                }
            }
            cc.state.store(0, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    const double t0 = now_s();
    for (int p = 0; p < producers; ++p) th.emplace_back(produce, p);
    for (int q = 0; q < consumers; ++q) th.emplace_back(consume, q);
    // the GPU stage: the router over each filled chunk, in ring order
    for (uint64_t k = 0; k < nchunks_total && !rc; ++k) {
        Chunk &cc = ch[k % c->chunks];
        while (cc.state.load(std::memory_order_acquire) != 1) {
        }
        const size_t base = (k % c->chunks) * c->chunk;
        rc = hfv_br_process_host(ctx, ring + base * c->slot, c->slot, len + base, ifx + base, cc.n, 0, act + base,
                                 ver + base, egr + base, c->stats);
        cc.state.store(2, std::memory_order_release);
    }
    if (rc) abort.store(true);
    for (auto &t : th) t.join();
    const double t1 = now_s();
    out->seconds = t1 - t0;
    for (int q = 0; q < consumers; ++q) {
        out->rx_pkts += part[q].rx_pkts;
        out->tx_pkts += part[q].tx_pkts;
        out->tx_bytes += part[q].tx_bytes;
        out->drop_pkts += part[q].drop_pkts;
        out->tx_digest += part[q].tx_digest;
        for (int v = 0; v < HFV_BR_COUNTERS; ++v) out->verdict_pkts[v] += part[q].verdict_pkts[v];
    }
    hfv_host_unregister(ctx, meta);
    hfv_host_unregister(ctx, ring);
    free(ring);
    free(meta);
    return rc;
}
