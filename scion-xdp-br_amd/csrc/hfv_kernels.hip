// hfv_kernels.hip -- gfx950 (MI355X) kernels for SCION hop-field AES-CMAC verification.
//
// Replaces the per-packet BPF call chain verify_hop_field -> aes_cmac_16bytes ->
// aes_cypher (br/src/bpf/xdp.c:77-91, aes/include/aes/aes.h:129-141, aes/src/aes.c:249-293)
// with one lane per packet:
//
//   * The four AES round tables T0..T3 live in LDS (128 KiB), replicated 32x so that lane L
//     always reads copy L%32: byte address (x << 8) | (t&1) << 7 | (L&31) << 2 | (t>>1) << 16
//     holds table t at index x.  ds_read_b32 banks are (addr/4) % 32 over each 32-lane half,
//     so every lookup is bank-conflict free whatever the data (hfv_aes_dev.h).
//   * The LDS byte address of a lookup is built with ONE v_perm_b32: byte 1 <- the state
//     byte, byte 0 <- the lane's copy/table bits, byte 2 <- the T2/T3 bit.
//   * Round keys: a single key (KEYSEL_ZERO, the reference rule xdp.c:82) is wave-uniform
//     and stays in SGPRs; per-interface keys (KEYSEL_IFID, config 3) come from five 16-byte
//     LDS rows per slot, the schedule words of rounds 3..10 precomputed (hfv_aes_dev.h).
//   * Verdicts: one __ballot per wave = 64 pass bits per 64 records.
//   * Persistent grid of one 1024-thread block per CU, so the table fill is paid once per
//     block; the next tile's record bytes are loaded while the current tile computes.
//
// Rejected variants measured in rounds 1-4 (bitsliced and hybrid AES, LDS-DMA and VGPR table
// fills, per-lane key rows gathered from L2, the 48 KiB key image beside two tables, two
// packets per lane, 2 blocks per CU) are documented in DESIGN.md and profiles/ab_index.md;
// their code is in the history (commit c3ddbb7).  Nothing read from the environment selects a
// kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_ext.h>

#include "hfv_aes_dev.h"
#include "hfv_internal.h"

namespace hfv {

// ---------------------------------------------------------------------------------------
// record verify: macinput from INF/HF (path_processing.h:39-81), CMAC, 48-bit compare
// ---------------------------------------------------------------------------------------
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(1))) uint8_t GlobalU8;
typedef __attribute__((address_space(1))) uint64_t GlobalU64;

struct RecWords {
    uint2 inf;    // INF bytes 0-7: flags rsv segid[2] | ts[4]
    uint2 hfa;    // HF bytes 0-7: flags exp ing[2] | eg[2] mac0 mac1
    uint32_t hfb; // HF bytes 8-11: mac2..mac5
};

// Unconditional loads (no branch around them, so the compiler can keep a counted vmcnt for
// the prefetch): lanes past the end re-read the last record and are masked off later.
// Non-temporal: the records are read once per launch.
__device__ __forceinline__ RecWords load_rec(const uint8_t *recs, uint64_t stride, uint64_t i, uint64_t last,
                                             uint32_t inf_off, uint32_t hf_off)
{
    RecWords r;
    // global address space, so these are global_load (vmcnt only), not flat loads that also
    // count in lgkmcnt
    const GlobalU8 *p = (const GlobalU8 *)(recs) + (i < last ? i : last) * stride;
    typedef const __attribute__((address_space(1))) u32x2 *P2;
    typedef const __attribute__((address_space(1))) uint32_t *P1;
    const u32x2 a = __builtin_nontemporal_load(reinterpret_cast<P2>(p + inf_off));
    const u32x2 b = __builtin_nontemporal_load(reinterpret_cast<P2>(p + hf_off));
    r.hfb = __builtin_nontemporal_load(reinterpret_cast<P1>(p + hf_off + 8));
    r.inf = make_uint2(a.x, a.y);
    r.hfa = make_uint2(b.x, b.y);
    return r;
}

// macinput words (scion.h:122-132) with the AS-ingress beta rule (path_processing.h:73-77):
// beta = SegID, xor'ed with MAC[0:2] when the Cons flag is clear.
__device__ __forceinline__ void rec_macinput(const RecWords &r, uint32_t w[4])
{
    uint32_t noncons_mask = (r.inf.x & 1u) ? 0u : 0xffff0000u;
    w[0] = (r.inf.x & 0xffff0000u) ^ (r.hfa.y & noncons_mask);
    w[1] = r.inf.y;
    w[2] = r.hfa.x & 0xffffff00u;
    w[3] = r.hfa.y & 0xffffu;
}

// AS-ingress IFID & 0xff (xdp.c:151-157): low byte of the big-endian Cons ? ingress : egress
__device__ __forceinline__ uint32_t rec_key_slot(const RecWords &r)
{
    return (r.inf.x & 1u) ? (r.hfa.x >> 24) : ((r.hfa.y >> 8) & 0xffu);
}

__device__ __forceinline__ bool rec_tag_matches(const RecWords &r, uint32_t t0, uint32_t t1)
{
    uint32_t e0 = __builtin_amdgcn_alignbit(r.hfb, r.hfa.y, 16);   // mac0..mac3
    uint32_t e1 = r.hfb >> 16;                                      // mac4, mac5
    return t0 == e0 && ((t1 ^ e1) & 0xffffu) == 0;
}

// One tile = 64 records = one wave: the verdict ballot (bit L = record L of the tile passed).
// `in`: this lane's record exists.  KEYSEL_ZERO: the wave-uniform slot-0 key (the caller
// handles an empty slot 0); KEYSEL_IFID: the slot's LDS rows, an empty slot fails closed
// (xdp.c:83-84).
// PIN: the round issue order of round_full (the launch kernel's choice, see there).
template <int KEYSEL, bool PIN = false>
__device__ __forceinline__ uint64_t verify_tile(const RecWords &r, bool in, const Lane &l, const UniformKey *ukey)
{
    uint32_t w[4], t0, t1;
    rec_macinput(r, w);
    bool ok = in;
    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
        cmac48_macinput<4, UniformKey, PIN>(w, *ukey, l, t0, t1);
    } else {
        const uint32_t slot = rec_key_slot(r);
        cmac48_sched(w, slot, l, t0, t1);
        ok = ok && slot_valid(slot);
    }
    return __ballot(ok && rec_tag_matches(r, t0, t1));
}

// The block's prologue: the round tables from T0 in the kernel arguments (one memory hop, the
// kernarg segment; round 4: 3.0 us from block entry to the fill barrier, against 4.1-4.5 us
// with a second hop to a table image), and config 3's key rows.  nthr: the threads taking part.
template <int KEYSEL, class P>
__device__ __forceinline__ void fill_block(P t0, const DevKeyTable *tab, uint32_t nthr)
{
    if (threadIdx.x < nthr) fill_ttab_karg<4>(t0, threadIdx.x >> 6, nthr >> 6);
    if constexpr (KEYSEL == HFV_KEYSEL_IFID) {
        if (threadIdx.x < nthr) fill_keys5(tab, nthr);
    }
}

// STAMP = 1 is a diagnostic build (hfv_debug_verify_stamped, scripts/stamps.py): lane 0 of
// every wave records s_memrealtime (100 MHz, chip-wide) at entry, after the table fill, after
// each of its first 10 tiles and at exit into stamps[wave * 16 + k], and s_memtime after the
// fill and at exit (slots 12, 13) for the in-kernel clock.  Nothing else reads the stamps.
//
// DYN = 1 (the default): block b owns the contiguous tile range [b*T/G, (b+1)*T/G) and its
// waves pull tiles from an LDS counter, so waves that the LDS arbiter serves less often take
// fewer tiles instead of finishing last (a static deal left the last ~20 % of the kernel with
// few waves active: scripts/stamps.py).  A wave claims its next tile before computing the
// current one, so the next tile's record loads overlap the rounds.
// DYN = 0: grid-stride tiles (wave w takes w, w + W, ...), for records in registered host
// memory, where 256 ranges far apart thrash the GPU's translation of 4 KiB host pages
// (zero-copy 2^20: 1.60 -> 1.27 ms).
constexpr int kBlock = 1024;
constexpr uint32_t kWaves = kBlock / 64;

template <int KEYSEL, int DYN, int STAMP = 0>
__global__ __launch_bounds__(kBlock) void k_verify_records(const DevKeyTable *__restrict__ tab,
                                                           const uint8_t *__restrict__ recs, uint64_t stride,
                                                           uint64_t n, uint32_t inf_off, uint32_t hf_off,
                                                           uint64_t *__restrict__ bits,
                                                           uint64_t *__restrict__ stamps, const RecArgs ka)
{
    const uint64_t ntiles = (n + 63) / 64;
    const uint64_t last = n - 1;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = wave_uniform(threadIdx.x / 64);
    uint64_t *st = STAMP ? stamps + ((uint64_t)blockIdx.x * kWaves + wv) * 16 : nullptr;
    if constexpr (STAMP) {
        if (lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
    }
    // DYN: this block's tile range; static: the grid-stride walk
    const uint64_t b0 = DYN ? ntiles * blockIdx.x / gridDim.x : 0;
    const uint64_t count = DYN ? ntiles * (blockIdx.x + 1) / gridDim.x - b0 : ntiles;
    const uint64_t stride_t = DYN ? kWaves : (uint64_t)gridDim.x * kWaves;
    uint64_t t = DYN ? wv : (uint64_t)blockIdx.x * kWaves + wv;   // the wave's first tile (static)
    UniformKey ukey(ka.key0, ka.key0_ok);   // from the kernel arguments: no second memory hop
    if (DYN && threadIdx.x == 0) s_next_tile = kWaves;
    // the wave's first records are in flight while its share of the tables is written
    RecWords cur = load_rec(recs, stride, (b0 + t) * 64 + lane, last, inf_off, hf_off);
    fill_block<KEYSEL>(ka.t0, tab, kBlock);
    __syncthreads();
    const Lane l = lane_bases();
    if constexpr (STAMP) {
        if (lane == 0) {
            st[1] = __builtin_amdgcn_s_memrealtime();
            st[12] = __builtin_amdgcn_s_memtime();   // shader clock, for the in-kernel frequency
        }
    }
    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
        if (!ukey.ok) {   // no key in slot 0: every packet fails closed (xdp.c:83-84)
            for (uint64_t tt = t; tt < count; tt += stride_t)
                if (lane == 0) bits[b0 + tt] = 0;
            return;
        }
    }
    // Verdict words wait in a per-wave stash (lane j: the wave's j-th tile) and go out as one
    // store per 64 tiles: a store per tile sits in the in-order vmcnt queue, and the loop latch
    // (which waits for the prefetched record words) would wait for its write acknowledgement
    // every tile.
    uint64_t st_word = 0, st_tile = 0;
    uint32_t stashed = 0;
    int nst = 0;
    while (t < count) {
        uint64_t nt;
        if constexpr (DYN) {
            uint32_t c = 0;
            if (lane == 0) c = atomicAdd(&s_next_tile, 1u);
            nt = wave_uniform(c);
        } else {
            nt = t + stride_t;
        }
        RecWords nxt = load_rec(recs, stride, (b0 + nt) * 64 + lane, last, inf_off, hf_off);
        const uint64_t ballot = verify_tile<KEYSEL, true>(cur, (b0 + t) * 64 + lane < n, l, &ukey);
        if (lane == stashed) {
            st_word = ballot;
            st_tile = b0 + t;
        }
        if (++stashed == 64) {
            ((GlobalU64 *)bits)[st_tile] = st_word;
            stashed = 0;
        }
        if constexpr (STAMP) {
            if (lane == 0 && nst < 10) st[2 + nst] = __builtin_amdgcn_s_memrealtime();
            ++nst;
        }
        cur = nxt;
        t = nt;
    }
    if (lane < stashed) ((GlobalU64 *)bits)[st_tile] = st_word;
    if constexpr (STAMP) {
        if (lane == 0) {
            st[13] = __builtin_amdgcn_s_memtime();
            st[15] = __builtin_amdgcn_s_memrealtime();
            // placement: HW_REG_HW_ID (hwreg 4, all 32 bits) and HW_REG_XCC_ID (hwreg 20)
            st[14] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                     ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
        }
    }
}

// ---------------------------------------------------------------------------------------
// stream-ordered batch list (hfv_verify_batches): up to kBatchMax batches in ONE launch
// ---------------------------------------------------------------------------------------
// The batches' tiles are numbered one after the other (batch j holds global tiles
// [cum[j], cum[j+1])) and block k verifies the contiguous range [T*k/G, T*(k+1)/G) of that
// space, its waves claiming tiles from an LDS counter as k_verify_records does.  A block's
// range spans one or two batches, so a wave changes batch about once per block range: the
// batch's descriptor sits in SGPRs, read from the kernel arguments (scalar loads) only when a
// claim leaves it.  Against the resident service (k_verify_service) this launch has no relay
// wave, no completion protocol and no system-scope verdict stores (the launch is stream
// ordered: the kernel's end publishes the bitmaps), and it pays the table fill once for all
// of its batches instead of once per batch as a launch per batch does.
typedef const __attribute__((address_space(4))) BatchArgs *BArgs;

struct BatchTile {   // the wave's current batch (wave-uniform)
    uint64_t recs, bits, n, stride;
    uint32_t lo, hi;   // its global tiles [lo, hi)
    uint32_t j;
};

__device__ __forceinline__ void batch_enter(BArgs a, uint32_t j, BatchTile &b)
{
    b.j = j;
    b.recs = a->d[j].recs;
    b.bits = a->d[j].bits;
    b.n = a->d[j].n;
    b.stride = a->d[j].stride;
    b.lo = a->cum[j];
    b.hi = a->cum[j + 1];
}

// global tile g -> its batch (g only grows along a wave's claims; g < a->total)
__device__ __forceinline__ void batch_map(BArgs a, uint32_t g, BatchTile &b)
{
    if (g < b.hi) return;
    uint32_t j = b.j + 1;
    while (g >= a->cum[j + 1]) ++j;
    batch_enter(a, j, b);
}

__device__ __forceinline__ RecWords batch_load(const BatchTile &b, uint32_t g, uint32_t lane, uint32_t inf_off,
                                               uint32_t hf_off)
{
    const uint64_t first = (uint64_t)(g - b.lo) * 64;
    const uint64_t left = b.n - 1 - first;                      // uniform: last valid lane
    const uint32_t lim = left < 63 ? (uint32_t)left : 63u;
    const uint32_t off = (lane < lim ? lane : lim) * (uint32_t)b.stride;
    const GlobalU8 *p = (const GlobalU8 *)(b.recs + first * b.stride) + off;
    typedef const __attribute__((address_space(1))) u32x2 *P2;
    typedef const __attribute__((address_space(1))) uint32_t *P1;
    RecWords r;
    const u32x2 x = __builtin_nontemporal_load(reinterpret_cast<P2>(p + inf_off));
    const u32x2 y = __builtin_nontemporal_load(reinterpret_cast<P2>(p + hf_off));
    r.hfb = __builtin_nontemporal_load(reinterpret_cast<P1>(p + hf_off + 8));
    r.inf = make_uint2(x.x, x.y);
    r.hfa = make_uint2(y.x, y.y);
    return r;
}

// DEPTH: tiles whose record loads are in flight ahead of the one being verified (1: the next
// tile's, as k_verify_records; 2: the next two -- HFV_BATCH_DEPTH, an A/B build switch).  Every
// load is issued unconditionally (a claim past the block's range re-reads its last tile), so the
// waitcnt pass keeps a counted vmcnt for the tiles still ahead instead of a vmcnt(0).
#ifndef HFV_BATCH_DEPTH
#define HFV_BATCH_DEPTH 1
#endif
// HFV_BATCH_PIN: each AES round's issue order pinned (16 addresses, 16 reads, 8 xor3; round_full)
#ifndef HFV_BATCH_PIN
#define HFV_BATCH_PIN 1
#endif
template <int KEYSEL, int DEPTH>
__global__ __launch_bounds__(kBlock) void k_verify_batches(const BatchArgs args)
{
    static_assert(DEPTH == 1 || DEPTH == 2, "prefetch depth");
    const BArgs a = (BArgs)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = wave_uniform(threadIdx.x / 64);
    const uint32_t total = a->total;
    const uint32_t b0 = (uint32_t)((uint64_t)total * blockIdx.x / gridDim.x);
    const uint32_t b1 = (uint32_t)((uint64_t)total * (blockIdx.x + 1) / gridDim.x);
    if (b1 == b0) return;   // (the launcher gives every block at least one tile)
    const uint32_t last = b1 - 1;
    const uint32_t inf_off = a->inf_off, hf_off = a->hf_off;
    UniformKey ukey(a->key0, a->key0_ok);
    // diagnostics, stored before the first record loads are issued (a store issued after them would
    // make the loop's first reuse of its data registers wait for every load ahead of it: vmcnt(0))
    if (threadIdx.x == 0 && a->clk) {
        a->clk[4 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();   // the block's entry
        if (blockIdx.x == 0) {                                         // the shader clock over the grid
            a->clk[0] = __builtin_amdgcn_s_memtime();
            a->clk[1] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (threadIdx.x == 0) s_next_tile = kWaves;
    auto at = [&](uint32_t x) { return x < b1 ? x : last; };   // the tile a load reads for claim x
    auto claim = [&]() -> uint32_t {
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(&s_next_tile, 1u);
        return b0 + wave_uniform(c);
    };
    // Record buffers: the loop is unrolled DEPTH + 1 times over DEPTH + 1 fixed register slots, slot
    // u verified in step u while the loads of the tile DEPTH claims ahead land in the slot step u - 1
    // just verified -- so no loop-carried register copy (which would wait for the loads it copies,
    // a vmcnt(0) at the latch) stands between a tile's loads and its use.
    constexpr int S = DEPTH + 1;
    RecWords buf[S];
    BatchTile bt[S];
    uint32_t gg[S];
    gg[0] = b0 + wv;        // the wave's first tile (static), its loads in flight while the tables are written
    bt[0].hi = 0;
    bt[0].j = ~0u;          // batch_map starts its search at batch 0
    batch_map(a, at(gg[0]), bt[0]);
    buf[0] = batch_load(bt[0], at(gg[0]), lane, inf_off, hf_off);
#pragma unroll
    for (int d = 1; d < DEPTH; ++d) {
        gg[d] = claim();
        bt[d] = bt[d - 1];
        batch_map(a, at(gg[d]), bt[d]);
        buf[d] = batch_load(bt[d], at(gg[d]), lane, inf_off, hf_off);
    }
    fill_block<KEYSEL>(a->t0, a->tab, kBlock);
    __syncthreads();
    const Lane l = lane_bases();
    // verdict words wait in a per-wave stash (lane k: the wave's k-th tile, with its own bitmap
    // address, since a wave's tiles may belong to two batches) and go out as one scattered store
    uint64_t st_word = 0, st_addr = 0;
    uint32_t stashed = 0;
    // KEYSEL_ZERO with slot 0 empty fails every packet closed (xdp.c:83-84): a loop of its own after
    // the tile loop (a verify skipped inside the tile loop would leave the prefetched loads unconsumed
    // on that path, and a store on a path into the loop's header would make its first register reuse
    // wait for it: either way the waitcnt pass drains every load at the loop top)
    const bool fail_closed = KEYSEL == HFV_KEYSEL_ZERO && !ukey.ok;
    // the exits leave the unrolled body straight to `done` (a flag checked at the loop top would
    // route them through the loop's header, whose waitcnt state would then hold the loads they left
    // in flight: a vmcnt(0) there on every iteration)
    if (gg[0] >= b1 || fail_closed) goto done;
    for (;;) {
#pragma unroll
        for (int u = 0; u < S; ++u) {
            const int in_slot = (u + DEPTH) % S, prev = (u + DEPTH - 1) % S;   // the free slot, the newest mapped
            gg[in_slot] = claim();
            bt[in_slot] = bt[prev];
            batch_map(a, at(gg[in_slot]), bt[in_slot]);
            buf[in_slot] = batch_load(bt[in_slot], at(gg[in_slot]), lane, inf_off, hf_off);
            const uint64_t rec = (uint64_t)(gg[u] - bt[u].lo) * 64 + lane;
            const uint64_t ballot = verify_tile<KEYSEL, HFV_BATCH_PIN != 0>(buf[u], rec < bt[u].n, l, &ukey);
            if (lane == stashed) {
                st_word = ballot;
                st_addr = bt[u].bits + (uint64_t)(gg[u] - bt[u].lo) * 8;
            }
            if (++stashed == 64) {
                *(GlobalU64 *)st_addr = st_word;
                stashed = 0;
            }
            if (gg[(u + 1) % S] >= b1) goto done;   // claims only grow: every later slot is past the range too
        }
    }
done:
    if (lane < stashed) *(GlobalU64 *)st_addr = st_word;
    if (fail_closed) {   // the block's verdict words are 0
        for (uint32_t g = b0 + wv; g < b1; g += kWaves) {
            batch_map(a, g, bt[0]);
            if (lane == 0) *(GlobalU64 *)(bt[0].bits + (uint64_t)(g - bt[0].lo) * 8) = 0;
        }
    }
    if (lane == 0 && a->clk)   // the block's last wave to leave sets its finish stamp
        __hip_atomic_fetch_max(&a->clk[4 + kBatchStampBlocks + blockIdx.x], __builtin_amdgcn_s_memrealtime(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x == 0 && a->clk) {
        a->clk[2] = __builtin_amdgcn_s_memtime();
        a->clk[3] = __builtin_amdgcn_s_memrealtime();
    }
}

int launch_verify_batches(const LaunchGeom &g, int keysel, const BatchArgs &args, void *stream, void *ev_start,
                          void *ev_stop)
{
    auto k = keysel == HFV_KEYSEL_IFID ? k_verify_batches<HFV_KEYSEL_IFID, HFV_BATCH_DEPTH>
                                       : k_verify_batches<HFV_KEYSEL_ZERO, HFV_BATCH_DEPTH>;
    // one block per CU, but no more blocks than tiles: every block owns at least one tile
    uint64_t blocks = args.total;
    if (blocks > (uint64_t)g.num_cus) blocks = (uint64_t)g.num_cus;
    hipExtLaunchKernelGGL(k, dim3((unsigned)(blocks ? blocks : 1)), dim3(kBlock), 0, (hipStream_t)stream,
                          (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0u, args);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// diagnostic: the HBM streaming-read rate of a list of device buffers (hfv_debug_stream_read),
// the achievable peak a bench run prices its verify kernel against -- the same resident batches,
// read densely (16 B per lane per load, non-temporal), 4 blocks of 1024 threads per CU
// (scripts/ubench/stream_read.hip: 7.05 TB/s on a 1 GiB buffer, round 1)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_stream_read(const StreamArgs args)
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint32_t acc = 0;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nthr = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t j = 0; j < args.nb; ++j) {
        const u32x4 *p = (const u32x4 *)args.buf[j];
        const uint64_t n = args.bytes[j] / 16;
        for (uint64_t i = tid; i < n; i += nthr) {
            const u32x4 v = __builtin_nontemporal_load(p + i);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9e3779b9u) args.sink[0] = acc;   // keeps the loads; never true for the bench's records in practice
}

int launch_stream_read(const LaunchGeom &g, const StreamArgs &args, void *stream, void *ev_start, void *ev_stop)
{
    hipExtLaunchKernelGGL(k_stream_read, dim3(4 * g.num_cus), dim3(1024), 0, (hipStream_t)stream,
                          (hipEvent_t)ev_start, (hipEvent_t)ev_stop, 0u, args);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// resident verify service (hfv_service_*): one persistent 1024-thread block per CU verifies
// batch after batch while the round tables (and the key image) stay in LDS
// ---------------------------------------------------------------------------------------
// The host posts batch descriptors into a ring in coherent host memory (SvcShared,
// hfv_internal.h); one wave of block 0 relays them into a device-memory mirror that all
// blocks read (svc_relay).  In every batch, block k owns the contiguous tile range
// [T*k/G, T*(k+1)/G) (T = tiles of the batch, G = grid).  Its waves claim tiles from ONE
// block-local counter that runs on across batches: block tile number g belongs to the batch
// b with base_b <= g < base_b + count_b, base_{b+1} = base_b + count_b (modulo 2^32).  Waves
// roll from one batch into the next without a block barrier, so the tail of batch b
// overlaps the start of batch b + 1, and the table fill is paid once per service instead of
// once per batch.
//
// Descriptor cache: batch b sits in s_svc[b % kSvcRing].  The host posts ticket t = b + 1
// only after ticket t - kSvcRing completed, so when a block loads batch L every batch up to
// L - kSvcRing is verified; an unverified claim g therefore lies in one of the newest
// kSvcRing batches and never in the slot being overwritten.  (Round 4 measured a dynamic tail:
// the last 1-2 batches of a run claimed in chunks from device-scope counters instead of fixed
// shares.  Chunks of 32 tiles: -0.5 % grid time, within noise; chunks of 8 from per-XCD
// counters: +11 %, a claim's round trip is as long as the chunk.  Removed;
// profiles/ab_index.md.)
//
// Completion: verdict words are written through (system-scope stores); a wave counts its
// verified tiles in the slot's LDS counter once those stores are acknowledged (vmcnt(0)),
// and the wave that completes the block's share stores the ticket into dev->done[slot][k]
// (svc_complete, device memory); the relay wave forwards a batch's completion to the host
// once every block has reported it.
// The service kernel's argument struct, read in place in the kernarg segment.
typedef const __attribute__((address_space(4))) SvcArgs *KArgs;

__device__ __forceinline__ SvcDescLite karg_desc(KArgs a, uint32_t i)
{
    SvcDescLite d;
    d.recs = a->inl[i].recs;
    d.bits = a->inl[i].bits;
    d.n = a->inl[i].n;
    d.stride = a->inl[i].stride;
    return d;
}
// svc_cum over the kernel argument's weights
__device__ __forceinline__ uint64_t karg_cum(KArgs a, uint64_t k)
{
    SvcWeights w;
    for (int x = 0; x < 8; ++x) w.w[x] = a->weights.w[x];
    w.w0 = a->weights.w0;
    return svc_cum(w, k);
}

struct alignas(16) SvcSlot {
    uint32_t base, count;   // block tile numbers [base, base + count)
    uint32_t done, stop;    // tiles of the batch this block has verified; 1: exit descriptor
    uint64_t recs, bits, n, stride, tile0;   // the batch, and the first tile of the block's range
    uint64_t pad;
};
static __shared__ SvcSlot s_svc[kSvcRing];
static __shared__ uint32_t s_svc_next, s_svc_loaded, s_svc_lock;
// Generation tag of this service grid (kernel argument, gen << 40): the host ring, the device
// mirror and the completion words carry tag | ticket, so words a previous grid left behind
// never match and nothing has to be cleared between grids.
static __shared__ uint64_t s_svc_tag;
// This block's share bounds (SvcWeights): tiles [T * s_svc_c0 / s_svc_w, T * s_svc_c1 / s_svc_w).
static __shared__ uint64_t s_svc_c0, s_svc_c1, s_svc_w;
__device__ __forceinline__ void svc_share(uint64_t ntiles, uint64_t &t0, uint32_t &count)
{
    t0 = ntiles * s_svc_c0 / s_svc_w;
    count = (uint32_t)(ntiles * s_svc_c1 / s_svc_w - t0);
}

struct SvcTile {   // one claimed tile, wave-uniform
    uint64_t recs, bits, n, stride, tile0, tile;   // tile = tile0 + (g - base)
    uint32_t b, base, count;
};
enum SvcClaim { kSvcFound = 0, kSvcStop = 1, kSvcPending = 2 };

// One tile's words for the resident service: the tile's base address is wave-uniform (one
// SGPR pair) and each lane adds a 32-bit offset (global_load ... saddr form); lanes past the
// batch's last record re-read it.
__device__ __forceinline__ RecWords load_tile(const SvcTile &t, uint32_t lane, uint32_t inf_off, uint32_t hf_off)
{
    const uint64_t first = t.tile * 64;
    const uint64_t left = t.n - 1 - first;                       // uniform: last valid lane
    const uint32_t lim = left < 63 ? (uint32_t)left : 63u;
    const uint32_t off = (lane < lim ? lane : lim) * (uint32_t)t.stride;
    const GlobalU8 *p = (const GlobalU8 *)(t.recs + first * t.stride) + off;
    typedef const __attribute__((address_space(1))) u32x2 *P2;
    typedef const __attribute__((address_space(1))) uint32_t *P1;
    RecWords r;
    const u32x2 a = *reinterpret_cast<P2>(p + inf_off);
    const u32x2 b = *reinterpret_cast<P2>(p + hf_off);
    r.hfb = *reinterpret_cast<P1>(p + hf_off + 8);
    r.inf = make_uint2(a.x, a.y);
    r.hfa = make_uint2(b.x, b.y);
    return r;
}

__device__ __forceinline__ uint64_t wave_uniform64(uint64_t x)
{
    return (uint64_t)wave_uniform((uint32_t)x) | ((uint64_t)wave_uniform((uint32_t)(x >> 32)) << 32);
}

// This block's share of batch b is verified (one lane).  The verdict words were written
// through to memory (system-scope stores) and every wave waited for their acknowledgement
// before counting its tiles, so nothing of the batch is left in L2.  The completion word goes
// to device memory (agent scope: written through to the memory side, where the relay wave of
// block 0 reads it); no grid-wide atomic (256 blocks on one counter serialise at the
// memory-side atomic unit: ~40 us per batch at 256 blocks, profiles/r01/service/) and no
// host-memory store whose acknowledgement a compute wave would wait for.
__device__ __attribute__((noinline)) void svc_complete(SvcDev *dev, uint64_t tag, uint32_t b)
{
    dev->blk_fin[blockIdx.x] = __builtin_amdgcn_s_memrealtime();   // read by the host after the grid
    dev->blk_clk1[blockIdx.x] = __builtin_amdgcn_s_memtime();
    __hip_atomic_store(&dev->done[b % kSvcRing][blockIdx.x], tag | ((uint64_t)b + 1), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t memrealtime() { return __builtin_amdgcn_s_memrealtime(); }

// Test hook (hfv_debug_relay_delay): a host round trip `us` microseconds longer.
__device__ __forceinline__ void relay_spin(uint32_t us)
{
    if (!us) return;
    const uint64_t t0 = memrealtime();
    while (memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(4);
}

// Descriptor relay and completion forwarder: block 0's last wave, all 64 lanes, for the grid's
// life.  It fetches the descriptors the host posts after the inline ones (batches n_inline,
// n_inline + 1, ...) into the device mirror `dev->mir`, in ticket order, up to 64 per host read:
// lane 0 looks at the next slot's seq; once it is posted, every lane reads the seq of one of
// the next 64 slots, the posted prefix's fields are read, copied (write-through agent-scope
// stores) and their seqs published after the fields are acknowledged.  It also forwards batch
// completions to the host ring (dev->done[slot][0..G) -> host->done[slot]), which the host
// needs only while the grid runs (to reuse ring slots, and for hfv_service_poll/wait).  The
// blocks never wait for this wave unless a batch's descriptor was posted after the grid
// started and has not been fetched yet (kRelayBlockWaits).  It owns the idle timeout: after
// idle_ticks without a new post it publishes a stop descriptor.  It leaves as soon as it has
// published a stop: a grid that exits on its stop has verified everything before it, and the
// host infers those completions from the grid's exit, so the relay never holds the grid open.
__device__ __attribute__((noinline)) void svc_relay(KArgs a, uint32_t lane, uint32_t G)
{
    SvcShared *host = a->host;
    SvcDev *dev = a->dev;
    const uint64_t tag = a->tag;
    const uint32_t n_in = a->n_inline;
    bool stop = n_in && a->inl[n_in - 1].n == kSvcStopN;
    uint32_t b = n_in;                       // next batch to relay
    uint32_t stop_b = stop ? n_in - 1 : ~0u;
    uint32_t f = 0;                          // next batch whose completion is forwarded
    uint64_t reads = 0, rticks = 0, rmax = 0, descs = 0, fwd = 0;
    auto timed_wait = [&]() {                // wait for this wave's host reads; account the trip
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    // one host-memory read at grid start: the PCIe round trip this grid saw (diagnostic)
    uint64_t t0 = memrealtime();
    uint64_t probe_v = __hip_atomic_load(&host->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    timed_wait();
    relay_spin(a->relay_delay_us);   // (the test hook's delay counts as part of the round trip)
    const uint64_t probe = memrealtime() - t0 + (probe_v == 0x5eedull ? 1 : 0);
    uint64_t t_idle = memrealtime();
    while (!stop) {
        bool prog = false;
        // is the next slot posted?
        uint64_t s0 = 0;
        t0 = memrealtime();
        if (lane == 0) s0 = __hip_atomic_load(&host->desc[b % kSvcRing].seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_wait();
        relay_spin(a->relay_delay_us);
        uint64_t rt = memrealtime() - t0;
        ++reads;
        rticks += rt;
        rmax = rt > rmax ? rt : rmax;
        if (wave_uniform64(s0) == (tag | ((uint64_t)b + 1))) {
            // read ahead: the seqs of the next 64 slots, then the fields of the posted prefix
            const uint32_t bi = b + lane;
            const uint64_t want = tag | ((uint64_t)bi + 1);
            SvcDesc *h = &host->desc[bi % kSvcRing];
            t0 = memrealtime();
            const uint64_t seq = __hip_atomic_load(&h->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            timed_wait();
            const uint64_t ready = __ballot(seq == want);
            const uint32_t k = ~ready ? (uint32_t)__builtin_ctzll(~ready) : 64u;   // >= 1: lane 0 saw it
            uint64_t recs = 0, bits = 0, n = 0, stride = 0;
            if (lane < k) {   // fields only after their seq was seen (the wait above)
                typedef uint64_t u64x4 __attribute__((ext_vector_type(4)));
                const u64x4 v = __builtin_nontemporal_load(reinterpret_cast<const u64x4 *>(&h->recs));
                recs = v.x;
                bits = v.y;
                n = v.z;
                stride = v.w;
            }
            timed_wait();
            relay_spin(a->relay_delay_us);
            rt = memrealtime() - t0;
            reads += 2;
            rticks += rt;
            rmax = rt > rmax ? rt : rmax;
            const uint64_t stops = __ballot(lane < k && n == kSvcStopN);
            const uint32_t kk = stops ? (uint32_t)__builtin_ctzll(stops) + 1u : k;
            SvcDesc *m = &dev->mir[bi % kSvcRing];
            if (lane < kk) {   // write-through field stores, acknowledged before the seqs
                __hip_atomic_store(&m->recs, recs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&m->bits, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&m->n, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&m->stride, stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane < kk) {
                __hip_atomic_store(&m->seq, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dev->relay_clock[bi % kSvcRing] = memrealtime();
            }
            if (stops) {
                stop = true;
                stop_b = b + kk - 1;
            }
            b += kk;
            descs += kk;
            prog = true;
            t_idle = memrealtime();
        } else if (memrealtime() - t_idle > a->idle_ticks) {
            if (lane == 0) {
                SvcDesc *m = &dev->mir[b % kSvcRing];
                __hip_atomic_store(&m->n, kSvcStopN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&m->seq, tag | ((uint64_t)b + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&host->status, kSvcIdleTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            stop = true;
            stop_b = b++;
            prog = true;
        }
        // forward the completions of batches every block has reported (none after the stop:
        // the grid's exit tells the host)
        while (!stop && f < b && f < stop_b) {
            const uint64_t want = tag | ((uint64_t)f + 1);
            bool ok = true;
            for (uint32_t k = lane; k < G; k += 64)
                ok = ok && __hip_atomic_load(&dev->done[f % kSvcRing][k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
            if (__ballot(!ok)) break;
            if (lane == 0) __hip_atomic_store(&host->done[f % kSvcRing], want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ++f;
            ++fwd;
            prog = true;
        }
        if (!prog) __builtin_amdgcn_s_sleep(8);
    }
    if (lane == 0) {   // read by the host after the grid
        dev->relay[kRelayProbeTicks] = probe;
        dev->relay[kRelayReads] = reads;
        dev->relay[kRelayReadTicks] = rticks;
        dev->relay[kRelayReadMax] = rmax;
        dev->relay[kRelayDescs] = descs;
        dev->relay[kRelayForwarded] = fwd;
        dev->relay[kRelayInline] = n_in;
    }
}

// Load batch b into its slot (one lane, holding s_svc_lock, s_svc_loaded == b) from the
// device mirror.  blocking: poll until the relay publishes it (bounded by a watchdog: the
// relay itself publishes a stop descriptor after idle_ticks); otherwise one look.  Returns
// false if the descriptor is not there yet.
__device__ __attribute__((noinline)) bool svc_load(KArgs a, uint32_t b, bool blocking)
{
    const uint32_t slot = b % kSvcRing;
    SvcDev *dev = a->dev;
    SvcDesc *d = &dev->mir[slot];
    bool stop = false;
    const uint64_t want = s_svc_tag | ((uint64_t)b + 1);
    if (__hip_atomic_load(&d->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
        if (!blocking) return false;
        __hip_atomic_fetch_add(&dev->area[a->launch & 1].block_waits, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = memrealtime();
        while (__hip_atomic_load(&d->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
            if (memrealtime() - t0 > 2 * a->idle_ticks + 100000000ull) {
                __hip_atomic_store(&a->host->status, kSvcWatchdog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                stop = true;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // fields only after seq was seen
    // the batch's records were written (by a kernel or a copy into device memory) before the
    // host posted it: drop this CU's stale L1 lines (agent scope, buffer_inv sc1)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (blockIdx.x == 0) dev->load_clock[slot] = memrealtime();
    SvcSlot &s = s_svc[slot];
    const SvcSlot &p = s_svc[(b + kSvcRing - 1) % kSvcRing];
    s.base = b ? p.base + p.count : 0u;
    s.done = 0;
    uint64_t n = 0;
    if (!stop) {
        s.recs = __hip_atomic_load(&d->recs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s.bits = __hip_atomic_load(&d->bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        n = __hip_atomic_load(&d->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s.stride = __hip_atomic_load(&d->stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        stop = n == kSvcStopN;
    }
    s.stop = stop;
    if (stop) {
        s.count = 0;
    } else {
        uint64_t t0;
        uint32_t cnt;
        svc_share((n + 63) / 64, t0, cnt);
        s.n = n;
        s.tile0 = t0;
        s.count = cnt;
        if (s.count == 0) svc_complete(dev, a->tag, b);
    }
    __hip_atomic_store(&s_svc_loaded, b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return true;
}

// The batches in the kernel arguments (batches 0 .. n_inline - 1, posted before the launch):
// wave 0 of every block fills their LDS slots before the prologue barrier, lane i batch i,
// the slots' base tile numbers by a prefix sum over the lanes.  Their records were written
// before the grid was launched, so no acquire fence is needed for them.
__device__ __attribute__((noinline)) void svc_load_inline(KArgs a, uint32_t lane)
{
    const uint32_t n_in = a->n_inline;
    const uint64_t c0 = karg_cum(a, blockIdx.x), c1 = karg_cum(a, blockIdx.x + 1);
    const uint64_t w = karg_cum(a, gridDim.x);
    uint32_t cnt = 0;
    uint64_t t0 = 0;
    SvcDescLite d = {0, 0, 0, 0};
    bool stop = false;
    if (lane < n_in) {
        d = karg_desc(a, lane);
        stop = d.n == kSvcStopN;
        if (!stop) {
            const uint64_t nt = (d.n + 63) / 64;
            t0 = nt * c0 / w;
            cnt = (uint32_t)(nt * c1 / w - t0);
        }
    }
    uint32_t incl = cnt;   // inclusive prefix sum of the counts over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
        if ((int)lane >= o) incl += y;
    }
    if (lane < n_in) {
        SvcSlot &s = s_svc[lane];
        s.base = incl - cnt;
        s.count = cnt;
        s.done = 0;
        s.stop = stop;
        s.recs = d.recs;
        s.bits = d.bits;
        s.n = d.n;
        s.stride = d.stride;
        s.tile0 = t0;
        if (!stop && cnt == 0) svc_complete(a->dev, a->tag, lane);
    }
    if (lane == 0) s_svc_loaded = n_in;
}

// The wave has just entered batch b: if batch b + 1 is not loaded yet and nobody is loading,
// take one look for its descriptor now, so the block's waves find it loaded when they reach
// the end of batch b instead of waiting there.
__device__ __forceinline__ void svc_prefetch(KArgs a, uint32_t lane, uint32_t b)
{
    if (lane == 0 && __hip_atomic_load(&s_svc_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == b + 1) {
        uint32_t expect = 0;
        if (__hip_atomic_compare_exchange_strong(&s_svc_lock, &expect, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
            if (__hip_atomic_load(&s_svc_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == b + 1)
                (void)svc_load(a, b + 1, false);
            __hip_atomic_store(&s_svc_lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// Map block tile number g to its batch (mb: batch of the wave's previous claim, g only
// grows).  Not blocking: kSvcPending if g lies in a batch the host has not posted yet.
__device__ __forceinline__ SvcClaim svc_map(KArgs a, uint32_t lane, uint32_t g, bool blocking, uint32_t &mb,
                                            const SvcTile &hint, SvcTile &t)
{
    if (g - hint.base < hint.count) {   // same batch as the wave's current tile: no LDS reads
        t = hint;
        t.tile = hint.tile0 + (g - hint.base);
        return kSvcFound;
    }
    uint64_t t_wait = 0;
    for (;;) {
        const uint32_t L =
            wave_uniform(__hip_atomic_load(&s_svc_loaded, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        // The slots hold batches [L - kSvcRing, L); the oldest one's slot is the one a loader
        // of batch L overwrites, possibly right now, and that batch is verified (the host posts
        // ticket t only after ticket t - kSvcRing completed), so g never lies in it: skip it.
        uint32_t lo = L >= kSvcRing ? L - kSvcRing + 1 : 0u;
        if (mb > lo) lo = mb;
        // the loaded batch holding g, searched forward from the wave's current batch (g only
        // grows, so it is almost always mb or mb + 1; a backward search from the newest
        // loaded batch cost one dependent LDS round trip per batch posted ahead: ~10 per
        // batch change when a run's 20 batches are all inline).  Slot header {base, count,
        // done, stop} in one 16-byte read.
        for (uint32_t b = lo; b < L; ++b) {
            const SvcSlot &s = s_svc[b % kSvcRing];
            const uint4 h = *reinterpret_cast<const uint4 *>(&s);
            const uint32_t base = wave_uniform(h.x);
            if ((int32_t)(g - base) < 0) break;   // before this batch: not loaded (cannot happen)
            if (wave_uniform(h.w)) return kSvcStop;
            const uint32_t count = wave_uniform(h.y);
            if (g - base >= count) continue;      // in a later batch
            t.recs = wave_uniform64(s.recs);
            t.bits = wave_uniform64(s.bits);
            t.n = wave_uniform64(s.n);
            t.stride = wave_uniform64(s.stride);
            t.tile0 = wave_uniform64(s.tile0);
            t.tile = t.tile0 + (g - base);
            t.b = b;
            t.base = base;
            t.count = count;
            mb = b;
            return kSvcFound;
        }
        // load batch L (one loader per block at a time)
        uint32_t r = 0;   // 1: loaded or someone else did, 2: not posted yet
        if (lane == 0) {
            uint32_t expect = 0;
            if (__hip_atomic_compare_exchange_strong(&s_svc_lock, &expect, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)) {
                r = 1;
                if (__hip_atomic_load(&s_svc_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == L &&
                    !svc_load(a, L, blocking))
                    r = 2;
                __hip_atomic_store(&s_svc_lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        r = wave_uniform(r);
        if (r == 2 || (r == 0 && !blocking)) return kSvcPending;
        if (r == 0) {
            // watchdog: the loader is bounded by idle_ticks; never wait much longer here
            const uint64_t now = memrealtime();
            if (!t_wait) t_wait = now;
            if (now - t_wait > 2 * a->idle_ticks + 100000000ull) {
                if (lane == 0)
                    __hip_atomic_store(&a->host->status, kSvcWatchdog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return kSvcStop;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
}

template <int KEYSEL>
__global__ __launch_bounds__(kBlock) void k_verify_service(const SvcArgs args)
{
    // the fields through the kernarg segment pointer (constant address space): no private copy
    // of the 3.3 KiB argument struct, and helpers take the pointer
    const KArgs a = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    const uint32_t lane = threadIdx.x & 63;
    SvcDev *dev = a->dev;
    UniformKey ukey(a->key0, a->key0_ok);
    const uint32_t inf_off = a->inf_off, hf_off = a->hf_off;
    if (threadIdx.x == 0) {
        s_svc_next = 0;
        s_svc_lock = 0;
        s_svc_tag = a->tag;
        s_svc_c0 = karg_cum(a, blockIdx.x);
        s_svc_c1 = karg_cum(a, blockIdx.x + 1);
        s_svc_w = karg_cum(a, gridDim.x);
    }
    if (threadIdx.x < 64) svc_load_inline(a, lane);   // the batches posted before the launch
    if (blockIdx.x == 0 && threadIdx.x == 64) dev->area[(a->launch + 1) & 1].block_waits = 0;   // next grid's
    // Block 0's last wave relays later-posted descriptors and forwards completions for the
    // grid's life.  It must not be alive at a barrier the other waves wait at (a wave still
    // running holds the barrier), so it passes the table-fill barrier without filling and
    // starts relaying right after it.
    const uint32_t nthr = blockIdx.x == 0 ? 1024 - 64 : 1024;   // threads filling the tables
    const bool relay = blockIdx.x == 0 && threadIdx.x >= nthr;
    fill_block<KEYSEL>(a->t0, a->tab, nthr);
    __syncthreads();
    if (threadIdx.x == 0) {
        dev->blk_start[blockIdx.x] = memrealtime();
        dev->blk_clk0[blockIdx.x] = __builtin_amdgcn_s_memtime();
    }
    if (relay) {   // no barrier follows: the block's other waves go on without it
        svc_relay(a, lane, gridDim.x);
        return;
    }
    const Lane l = lane_bases();
    // KEYSEL_ZERO with slot 0 empty: every packet fails closed (xdp.c:83-84)
    const bool keyok = KEYSEL != HFV_KEYSEL_ZERO || ukey.ok;
    const UniformKey *ukp = KEYSEL == HFV_KEYSEL_ZERO ? &ukey : nullptr;

    if (blockIdx.x == 0 && threadIdx.x == 0) {   // diagnostics: shader clock over the grid's life
        dev->run_clock[0] = __builtin_amdgcn_s_memtime();
        dev->run_clock[1] = memrealtime();
    }
    uint32_t mb = 0;
    SvcTile none;
    none.base = 0;
    none.count = 0;
    // The loop, per tile: wait for the tile's records (loaded one iteration ahead), claim the
    // next tile (LDS atomic, just in time: claiming one iteration ahead made K = 20 grids 2.1-2.4 %
    // longer, profiles/ab_index.md r03_ahead_ab), store the
    // verdict words of a batch the wave left in the previous
    // iteration (so their write acknowledgement arrives while this tile computes and is
    // covered by the next iteration's wait), map the next tile and issue its loads, compute.
    // (Measured with a phase-counter build on the loop this replaces -- claim at the top, store
    // and a vmcnt(0) drain when leaving a batch: claim/map/load 10 %, store/count drain 9-20 %
    // of a wave's cycles.)
    auto claim = [&]() -> uint32_t {
        uint32_t g = 0;
        if (lane == 0) g = __hip_atomic_fetch_add(&s_svc_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return g;
    };
    SvcTile cur;
    if (svc_map(a, lane, wave_uniform(claim()), true, mb, none, cur) != kSvcFound) return;
    // Verdict words of cur.b's tiles wait in a per-wave stash (lane j: the j-th word) and go
    // out as ONE scattered write-through store, issued at the top of the iteration after the
    // wave left the batch (or filled the stash).  A store per tile would sit in the wave's
    // in-order vmcnt queue in front of the next tile's record loads.  (Collecting a block's
    // words in LDS and writing 512 B chunks instead was not faster.)
    uint64_t st_word = 0, st_tile = 0, st_bits = 0;
    uint32_t stashed = 0;
    bool flush = false;              // the stash holds words to store at the next top
    uint32_t fl_b = 0, fl_count = 0, fl_k = 0;   // ... and the count they complete (fl_k = 0: none)
    uint32_t dc_b = 0, dc_count = 0, dc_k = 0;   // stored last iteration: count after this wait
    uint32_t pending = 0;            // verified tiles of cur.b not handed to a count yet
    auto count = [&](uint32_t b, uint32_t cnt, uint32_t k) {   // stores acknowledged (caller waited)
        if (k && lane == 0) {
            const uint32_t old =
                __hip_atomic_fetch_add(&s_svc[b % kSvcRing].done, k, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old + k == cnt) svc_complete(dev, a->tag, b);
        }
    };
    auto store_stash = [&]() {
        if (lane < stashed)
            __hip_atomic_store(reinterpret_cast<GlobalU64 *>(st_bits) + st_tile, st_word, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        stashed = 0;
    };
    RecWords rc = load_tile(cur, lane, inf_off, hf_off);
    svc_prefetch(a, lane, cur.b);
    for (;;) {
        // This tile's record words (and every earlier store) are complete.  An explicit wait
        // (a builtin, so the waitcnt pass sees it): without it the pass merges the loop's
        // entry paths and puts a vmcnt(0) AFTER the next tile's loads.
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
        count(dc_b, dc_count, dc_k);           // the stores of the previous iteration are acknowledged
        dc_k = 0;
        if (flush) {                           // the batch left in the previous iteration
            store_stash();
            dc_b = fl_b;
            dc_count = fl_count;
            dc_k = fl_k;
            flush = false;
        }
        const uint32_t g = wave_uniform(claim());
        SvcTile nx;
        SvcClaim c = svc_map(a, lane, g, false, mb, cur, nx);
        if (c != kSvcFound) nx = cur;
        RecWords rn = load_tile(nx, lane, inf_off, hf_off);
        uint64_t ballot = 0;   // KEYSEL_ZERO with slot 0 empty: every packet fails closed
        if (keyok) ballot = verify_tile<KEYSEL>(rc, cur.tile * 64 + lane < cur.n, l, ukp);
        if (lane == stashed) {
            st_word = ballot;
            st_tile = cur.tile;
        }
        st_bits = cur.bits;
        ++stashed;
        ++pending;
        const bool leave = c != kSvcFound || nx.b != cur.b;
        if (leave || stashed == 64) {
            flush = true;
            fl_b = cur.b;
            fl_count = cur.count;
            fl_k = leave ? pending : 0;
            if (leave) pending = 0;
        }
        if (c != kSvcFound) {
            // before waiting for the host (or leaving): store and count everything verified,
            // so a host that waits for those batches before posting the next never waits on us
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            count(dc_b, dc_count, dc_k);
            dc_k = 0;
            if (flush) {
                store_stash();
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                count(fl_b, fl_count, fl_k);
                flush = false;
            }
            if (c == kSvcPending) {
                c = svc_map(a, lane, g, true, mb, none, nx);
                if (c == kSvcFound) rn = load_tile(nx, lane, inf_off, hf_off);
            }
        }
        if (c == kSvcStop) break;
        if (nx.b != cur.b) svc_prefetch(a, lane, nx.b);
        cur = nx;
        rc = rn;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dev->run_clock[2] = __builtin_amdgcn_s_memtime();
        dev->run_clock[3] = memrealtime();
    }
}

int launch_verify_service(const LaunchGeom &g, int keysel, const SvcArgs &args, void *stream, void *ev_start,
                          void *ev_stop, unsigned *grid_out)
{
    auto k = keysel == HFV_KEYSEL_IFID ? k_verify_service<HFV_KEYSEL_IFID> : k_verify_service<HFV_KEYSEL_ZERO>;
    unsigned grid = g.svc_blocks > 0 && g.svc_blocks < g.num_cus ? (unsigned)g.svc_blocks : (unsigned)g.num_cus;
    if (grid > kSvcMaxBlocks) grid = kSvcMaxBlocks;
    *grid_out = grid;
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
                          (hipEvent_t)ev_stop, 0u, args);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// prepared macinputs: verify (xdp.c:77-91) or full tags (aes_cmac_16bytes)
// ---------------------------------------------------------------------------------------
template <int MODE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_macinputs(const DevKeyTable *__restrict__ tab,
                                                     const uint4 *__restrict__ mi, const uint2 *__restrict__ expected,
                                                     const uint8_t *__restrict__ kidx, uint64_t n,
                                                     uint64_t *__restrict__ bits, uint4 *__restrict__ tags)
{
    constexpr uint32_t kWaves = BLOCK / 64;
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform(blockIdx.x * kWaves + threadIdx.x / 64);
    const uint32_t nwaves = gridDim.x * kWaves;
    fill_ttab<2>();
    fill_keys(tab);
    __syncthreads();
    const Lane l = lane_bases();
    for (uint64_t t = wave; t < ntiles; t += nwaves) {
        uint64_t i = t * 64 + lane;
        bool in = i < n;
        uint4 m = in ? mi[i] : make_uint4(0, 0, 0, 0);
        uint32_t slot = (in && kidx) ? kidx[i] : 0u;
        const LdsKey key(slot);
        uint32_t w[4] = {m.x, m.y, m.z, m.w}, s[4];
        cmac_general<2>(w, key, l, s);
        if constexpr (MODE == kModeTags) {
            uint32_t o[4];
            round_last_full<2>(s, key.row(10), l, o);
            if (!key.ok()) o[0] = o[1] = o[2] = o[3] = 0;
            if (in) tags[i] = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            uint32_t t0, t1;
            round_last_48<2>(s, key.row(10), l, t0, t1);
            uint2 e = in ? expected[i] : make_uint2(0, 0);
            // actual = tag bytes 0..5 as LE u64 (upper 16 bits zero) == expected (xdp.c:89-90)
            bool pass = in && key.ok() && t0 == e.x && (t1 & 0xffffu) == e.y;
            uint64_t ballot = __ballot(pass);
            if (lane == 0) bits[t] = ballot;
        }
    }
}

// ---------------------------------------------------------------------------------------
// key expansion + CMAC subkey, one key per lane (aes.c:120-137, 298-325; br_loader.cpp:215-218)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sbox_g(uint32_t x) { return (c_t0[x & 0xff] >> 8) & 0xffu; }
__device__ __forceinline__ uint32_t sub_word_g(uint32_t w)
{
    return sbox_g(w) | sbox_g(w >> 8) << 8 | sbox_g(w >> 16) << 16 | sbox_g(w >> 24) << 24;
}
__device__ __forceinline__ uint32_t tg(int row, uint32_t x)
{
    uint32_t t = c_t0[x & 0xff];
    return row ? __builtin_amdgcn_alignbit(t, t, 32 - 8 * row) : t;
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__global__ __launch_bounds__(256) void k_expand_keys(const uint4 *__restrict__ raw, uint64_t n,
                                                     hop_key *__restrict__ out, DevKeyTable *__restrict__ tab,
                                                     uint32_t first_slot)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 k = raw[i];
    uint32_t w[44];
    w[0] = k.x; w[1] = k.y; w[2] = k.z; w[3] = k.w;
    uint32_t rcon = 1;
#pragma unroll
    for (int j = 4; j < 44; j += 4) {
        uint32_t t = sub_word_g(__builtin_amdgcn_alignbit(w[j - 1], w[j - 1], 8)) ^ rcon;   // RotWord = rotr8
        rcon = (rcon << 1) ^ ((rcon & 0x80u) ? 0x11bu : 0u);
        w[j] = w[j - 4] ^ t;
        w[j + 1] = w[j - 3] ^ w[j];
        w[j + 2] = w[j - 2] ^ w[j + 1];
        w[j + 3] = w[j - 1] ^ w[j + 2];
    }
    // L = E_K(0^128); K1 = dbl(L) (RFC 4493 2.3)
    uint32_t s[4] = {w[0], w[1], w[2], w[3]}, nn[4];
    for (int r = 1; r < 10; ++r) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
            nn[c] = tg(0, s[c]) ^ tg(1, s[(c + 1) & 3] >> 8) ^ tg(2, s[(c + 2) & 3] >> 16) ^ tg(3, s[(c + 3) & 3] >> 24) ^
                    w[4 * r + c];
#pragma unroll
        for (int c = 0; c < 4; ++c) s[c] = nn[c];
    }
    uint32_t L[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
        L[c] = (sbox_g(s[c]) | sbox_g(s[(c + 1) & 3] >> 8) << 8 | sbox_g(s[(c + 2) & 3] >> 16) << 16 |
                sbox_g(s[(c + 3) & 3] >> 24) << 24) ^ w[40 + c];
    // big-endian 128-bit shift: byte 0 is the most significant
    uint32_t q0 = bswap(L[0]), q1 = bswap(L[1]), q2 = bswap(L[2]), q3 = bswap(L[3]);
    uint32_t msb = q0 >> 31;
    q0 = (q0 << 1) | (q1 >> 31);
    q1 = (q1 << 1) | (q2 >> 31);
    q2 = (q2 << 1) | (q3 >> 31);
    q3 = (q3 << 1) ^ (msb ? 0x87u : 0u);
    uint32_t k1[4] = {bswap(q0), bswap(q1), bswap(q2), bswap(q3)};
    if (out) {
        uint4 *o = reinterpret_cast<uint4 *>(out + i);
#pragma unroll
        for (int r = 0; r < 11; ++r) o[r] = make_uint4(w[4 * r], w[4 * r + 1], w[4 * r + 2], w[4 * r + 3]);
        o[11] = make_uint4(k1[0], k1[1], k1[2], k1[3]);
    }
    if (tab) {   // compiled device image (hfv_tables.h), same as compile_dev_key on the host
        uint32_t slot = first_slot + (uint32_t)i;
        uint32_t k0[4] = {w[0] ^ k1[0], w[1] ^ k1[1], w[2] ^ k1[2], w[3] ^ k1[3]};
        uint32_t *row0 = tab->rows[0][slot];
        row0[0] = k0[0]; row0[1] = k0[1]; row0[2] = k0[2]; row0[3] = k0[3];
        for (int r = 1; r < 11; ++r) {   // rows 1..9 pre-rotated by 16 (hfv_tables.h)
            uint32_t *p = tab->rows[r][slot];
            int rot = r < 10 ? 16 : 0;
            for (int c = 0; c < 4; ++c) p[c] = rot ? __builtin_amdgcn_alignbit(w[4 * r + c], w[4 * r + c], 16) : w[4 * r + c];
        }
        uint32_t *p = tab->rows[11][slot];
        p[0] = w[4] ^ tg(0, k0[0]) ^ tg(3, k0[3] >> 24);
        p[1] = w[5] ^ tg(2, k0[3] >> 16);
        p[2] = w[6] ^ tg(0, k0[2]);
        p[3] = w[7] ^ tg(1, k0[0] >> 8);
        for (int r = 3; r <= 10; ++r)   // schedule words t_r = w[4r] ^ w[4r-4] (hfv_internal.h)
            tab->sched[(r - 3) >> 2][slot][(r - 3) & 3] = w[4 * r] ^ w[4 * r - 4];
        atomicOr(&tab->valid[slot >> 5], 1u << (slot & 31));
    }
}

// ---------------------------------------------------------------------------------------
// synthetic 64 B records (CPU twin: oracle orc_gen_records)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_gen_records(const DevKeyTable *__restrict__ tab, int keysel,
                                                       uint8_t *__restrict__ recs, uint64_t stride, uint64_t n,
                                                       uint64_t seed, uint64_t first_index)
{
    fill_ttab<2>();
    fill_keys(tab);
    __syncthreads();
    const Lane l = lane_bases();
    for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK) {
        uint64_t i = first_index + j;
        uint64_t r0 = splitmix_at(seed, 4 * i), r1 = splitmix_at(seed, 4 * i + 1);
        uint64_t r2 = splitmix_at(seed, 4 * i + 2), r3 = splitmix_at(seed, 4 * i + 3);
        uint32_t cons = (uint32_t)r0 & 1u;
        uint32_t beta = (uint32_t)(r0 >> 8) & 0xffffu;
        uint32_t ts_w = bswap((uint32_t)(r0 >> 32));
        uint32_t exp = (uint32_t)r1 & 0xffu;
        uint32_t ing = 1u + (uint32_t)((r1 >> 8) & 0xffffu) % 255u;
        uint32_t eg = 1u + (uint32_t)((r1 >> 24) & 0xffffu) % 255u;
        uint32_t hf0 = (exp << 8) | (bswap16(ing) << 16);
        uint32_t hf1 = bswap16(eg);
        uint32_t slot = keysel == HFV_KEYSEL_IFID ? ((cons ? ing : eg) & 0xffu) : 0u;
        const LdsKey key(slot);
        uint32_t w[4] = {bswap16(beta) << 16, ts_w, hf0, hf1}, s[4], tg4[4];
        cmac_general<2>(w, key, l, s);
        round_last_full<2>(s, key.row(10), l, tg4);
        uint32_t seg = cons ? beta : (beta ^ bswap16(tg4[0] & 0xffffu));
        uint64_t mac = (uint64_t)tg4[0] | ((uint64_t)(tg4[1] & 0xffffu) << 32);
        if ((r2 & 15u) == 0) mac ^= 1ull << ((r2 >> 4) % 48u);
        uint4 q0 = make_uint4(bswap((uint32_t)(r3 & 0xfffffu)), 0x04000f11u, 1u, 0x00ff0100u);
        uint4 q1 = make_uint4(0x10000000u, 0x00ff0100u, 0x11000000u, 0x0100000au);
        uint4 q2 = make_uint4(0x0200000au, 0x00100000u, cons | (bswap16(seg) << 16), ts_w);
        uint4 q3 = make_uint4(hf0, hf1 | ((uint32_t)mac << 16), (uint32_t)(mac >> 16), bswap((uint32_t)i));
        uint4 *o = reinterpret_cast<uint4 *>(recs + j * stride);
        o[0] = q0; o[1] = q1; o[2] = q2; o[3] = q3;
    }
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
constexpr int kBlockAux = 512;

static inline unsigned grid_for(uint64_t n, int block, int num_cus, int per_cu)
{
    uint64_t tiles = (n + 63) / 64;
    uint64_t blocks = (tiles + block / 64 - 1) / (block / 64);
    uint64_t cap = (uint64_t)num_cus * (uint64_t)(per_cu > 0 ? per_cu : 1);
    if (blocks > cap) blocks = cap;
    return (unsigned)(blocks ? blocks : 1);
}

static RecArgs rec_args(const DevKeyTable *host_keys)
{
    RecArgs ka;
    memset(&ka, 0, sizeof ka);
    if (host_keys) {
        for (int r = 0; r < kDevKeyRows; ++r) memcpy(&ka.key0[4 * r], host_keys->rows[r][0], 16);
        ka.key0_ok = host_keys->valid[0] & 1u;
    }
    memcpy(ka.t0, kTables.t0, sizeof ka.t0);
    return ka;
}

int launch_verify_records(const LaunchGeom &g, const DevKeyTable *tab, const DevKeyTable *host_keys, int keysel,
                          const uint8_t *recs,
                          size_t stride, size_t n, uint32_t inf_off, uint32_t hf_off, uint64_t *bits, void *stream,
                          void *ev_start, void *ev_stop, bool interleaved)
{
    // Records in device memory: the batch-list kernel with one batch (the same loop as a burst of
    // batches, hfv_verify_batches; its 32-bit lane offsets and tile numbers bound stride and n).
    if (!interleaved && stride <= ((size_t)1 << 24) && n <= ((size_t)1 << 36)) {
        BatchArgs a;
        memset(&a, 0, sizeof a);
        a.tab = tab;
        a.inf_off = inf_off;
        a.hf_off = hf_off;
        a.nb = 1;
        a.total = (uint32_t)((n + 63) / 64);
        a.cum[0] = 0;
        a.cum[1] = a.total;
        a.d[0] = {(uint64_t)(uintptr_t)recs, (uint64_t)(uintptr_t)bits, (uint64_t)n, (uint64_t)stride};
        const RecArgs ra = rec_args(host_keys);
        memcpy(a.key0, ra.key0, sizeof a.key0);
        a.key0_ok = ra.key0_ok;
        memcpy(a.t0, ra.t0, sizeof a.t0);
        return launch_verify_batches(g, keysel, a, stream, ev_start, ev_stop);
    }
    using K = void (*)(const DevKeyTable *, const uint8_t *, uint64_t, uint64_t, uint32_t, uint32_t, uint64_t *,
                       uint64_t *, const RecArgs);
    const bool ifid = keysel == HFV_KEYSEL_IFID;
    K k = interleaved ? (ifid ? k_verify_records<HFV_KEYSEL_IFID, 0> : k_verify_records<HFV_KEYSEL_ZERO, 0>)
                      : (ifid ? k_verify_records<HFV_KEYSEL_IFID, 1> : k_verify_records<HFV_KEYSEL_ZERO, 1>);
    const unsigned grid = grid_for(n, kBlock, g.num_cus, 1);
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
                          (hipEvent_t)ev_stop, 0u, tab, recs, (uint64_t)stride, (uint64_t)n, inf_off, hf_off, bits,
                          (uint64_t *)nullptr, rec_args(host_keys));
    return (int)hipGetLastError();
}

int launch_verify_stamped(const LaunchGeom &g, const DevKeyTable *tab, const DevKeyTable *host_keys, const uint8_t *recs,
                          size_t n, uint64_t *bits, uint64_t *stamps, void *stream)
{
    const unsigned grid = grid_for(n, kBlock, g.num_cus, 1);
    hipLaunchKernelGGL((k_verify_records<HFV_KEYSEL_ZERO, 1, 1>), dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, tab,
                       recs, (uint64_t)64, (uint64_t)n, (uint32_t)HFV_REC_INF_OFF, (uint32_t)HFV_REC_HF_OFF, bits,
                       stamps, rec_args(host_keys));
    return (int)hipGetLastError();
}

int launch_verify_macinputs(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint64_t *expected,
                            const uint8_t *kidx, size_t n, uint64_t *bits, void *stream)
{
    unsigned grid = grid_for(n, kBlockAux, g.num_cus, 2);
    hipLaunchKernelGGL((k_macinputs<kModeMacinputs, kBlockAux>), dim3(grid), dim3(kBlockAux), 0, (hipStream_t)stream,
                       tab, (const uint4 *)mi, (const uint2 *)expected, kidx, (uint64_t)n, bits, (uint4 *)nullptr);
    return (int)hipGetLastError();
}

int launch_cmac_tags(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint8_t *kidx, size_t n,
                     void *tags, void *stream)
{
    unsigned grid = grid_for(n, kBlockAux, g.num_cus, 2);
    hipLaunchKernelGGL((k_macinputs<kModeTags, kBlockAux>), dim3(grid), dim3(kBlockAux), 0, (hipStream_t)stream, tab,
                       (const uint4 *)mi, (const uint2 *)nullptr, kidx, (uint64_t)n, (uint64_t *)nullptr,
                       (uint4 *)tags);
    return (int)hipGetLastError();
}

int launch_expand_keys(const uint8_t *raw, size_t n, hop_key *out, DevKeyTable *tab, uint32_t first_slot,
                       void *stream)
{
    unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_expand_keys, dim3(grid ? grid : 1), dim3(256), 0, (hipStream_t)stream, (const uint4 *)raw,
                       (uint64_t)n, out, tab, first_slot);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// record_verdict for the verify-only paths (xdp.c:54-70): per AS-ingress interface (the
// KEYSEL_IFID slot, IFID & 0xff, xdp.c:151-157) the packets that verified and the packets
// dropped as VERDICT_INVALID_HF, from the records and a verdict bitmap of either verify path.
// One lane per record; a block histogram in LDS, added to the u64 counters with one global
// atomic per non-zero bin.  HBM-bound: the three bytes it reads lie in the record's 64-byte line.
// ---------------------------------------------------------------------------------------
constexpr int kCountBlock = 512;
__global__ __launch_bounds__(kCountBlock) void k_count_verdicts(const uint8_t *__restrict__ recs, uint64_t stride,
                                                                uint64_t n, uint32_t inf_off, uint32_t hf_off,
                                                                const uint64_t *__restrict__ bits,
                                                                unsigned long long *__restrict__ counters)
{
    __shared__ uint32_t h[512];
    for (uint32_t i = threadIdx.x; i < 512; i += kCountBlock) h[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kCountBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kCountBlock) {
        const uint8_t *r = recs + i * stride;
        // Cons ? ConsIngress : ConsEgress, low byte of the big-endian field (rec_key_slot)
        const uint32_t slot = (r[inf_off] & 1u) ? r[hf_off + 3] : r[hf_off + 5];
        const uint32_t pass = (uint32_t)(bits[i >> 6] >> (i & 63)) & 1u;
        atomicAdd(&h[slot * 2 + (pass ^ 1u)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 512; i += kCountBlock)
        if (h[i]) atomicAdd(counters + i, (unsigned long long)h[i]);
}

int launch_count_verdicts(const LaunchGeom &g, const uint8_t *recs, size_t stride, size_t n, uint32_t inf_off,
                          uint32_t hf_off, const uint64_t *bits, uint64_t *counters, void *stream)
{
    unsigned grid = grid_for(n, kCountBlock, g.num_cus, 1);
    hipLaunchKernelGGL(k_count_verdicts, dim3(grid), dim3(kCountBlock), 0, (hipStream_t)stream, recs, (uint64_t)stride,
                       (uint64_t)n, inf_off, hf_off, bits, (unsigned long long *)counters);
    return (int)hipGetLastError();
}

int launch_gen_records(const LaunchGeom &g, const DevKeyTable *tab, int keysel, uint8_t *recs, size_t stride,
                       size_t n, uint64_t seed, uint64_t first_index, void *stream)
{
    uint64_t blocks = (n + kBlockAux - 1) / kBlockAux;
    uint64_t cap = (uint64_t)g.num_cus * 2;
    unsigned grid = (unsigned)(blocks < cap ? (blocks ? blocks : 1) : cap);
    hipLaunchKernelGGL((k_gen_records<kBlockAux>), dim3(grid), dim3(kBlockAux), 0, (hipStream_t)stream, tab, keysel,
                       recs, (uint64_t)stride, (uint64_t)n, seed, first_index);
    return (int)hipGetLastError();
}

int query_geometry(int device, LaunchGeom *g)
{
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return (int)e;
    g->num_cus = prop.multiProcessorCount;
    g->svc_blocks = g->num_cus;
    // one 1024-thread block per CU must fit: the service's LDS (tables, config 3's key rows,
    // descriptor cache) is the largest of the verify kernels'
    int occ = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_verify_service<HFV_KEYSEL_IFID>, kBlock, 0);
    if (e != hipSuccess) return (int)e;
    if (occ < 1) return (int)hipErrorInvalidConfiguration;
    return 0;
}

}  // namespace hfv
