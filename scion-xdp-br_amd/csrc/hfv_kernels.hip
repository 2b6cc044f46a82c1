// hfv_kernels.hip -- gfx950 (MI355X) kernels for SCION hop-field AES-CMAC verification.
//
// Replaces the per-packet BPF call chain verify_hop_field -> aes_cmac_16bytes ->
// aes_cypher (br/src/bpf/xdp.c:77-91, aes/include/aes/aes.h:129-141, aes/src/aes.c:249-293)
// with one lane per packet:
//
//   * AES round tables live in LDS, replicated 32x so that lane L always reads copy L%32:
//     dword (x << 6) | (t << 5) | (L & 31) holds table t (0 = T0, 1 = T1 = rotl8(T0)) at
//     index x.  ds_read_b32 banks are (addr/4) % 32 over each 32-lane half, so every
//     lookup is bank-conflict free whatever the data.  T2/T3 are T0/T1 rotated by 16 and
//     are folded in with one v_alignbit per column.
//   * The LDS byte address of a lookup is built with ONE v_perm_b32: byte 1 <- the state
//     byte, byte 0 <- the lane's copy/table bits, bytes 2-3 <- 0.
//   * Round keys: a single key (KEYSEL_ZERO, the reference rule xdp.c:82) is wave-uniform
//     and stays in SGPRs; per-packet keys come from an LDS copy of the key table.
//   * Verdicts: one __ballot per wave = 64 pass bits, one 8-byte store by lane 0.
//   * Persistent grid (a few blocks per CU) so the 64 KiB table fill is paid once per
//     block; the next tile's record bytes are prefetched while the current tile computes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_ext.h>

#include "hfv_aes_dev.h"
#include "hfv_bitslice.h"
#include "hfv_internal.h"

namespace hfv {

// How the one-launch-per-batch kernel fills its LDS round tables: 3 (default) from T0 in its
// kernel arguments (RecArgs: the block prologue is one memory hop, the kernarg segment, with the
// slot-0 key rows alongside); 2 the compact image copied through VGPRs, its pieces issued
// before the first tile's records (TtabRegs); 1 LDS-DMA from the compact image after the
// records.  The resident service takes T0 and the key rows from its arguments too
// (HFV_SVC_FILL_DMA=1: LDS-DMA).  Measured round 4 (profiles/r04/fill_ab.log, span probe):
// the service's block prologue (entry -> fill barrier) took 4.1-4.5 us with the key rows and
// the LDS-DMA source behind a second hop (the 16 KiB compact image or round 3's 128 KiB: the
// same), 3.4 us with the keys in the arguments and LDS-DMA, 3.0 us with both in the arguments;
// 5.3 us with the tables computed in the block (GF(2^8) inversion in VALU; removed).
#ifndef HFV_FILL
#define HFV_FILL 3
#endif
// HFV_SVC_FILL_DMA = 1: the service fills its tables by LDS-DMA from the compact image (a second
// memory hop after the kernel arguments) instead of from T0 in its kernel arguments
#ifndef HFV_SVC_FILL_DMA
#define HFV_SVC_FILL_DMA 0
#endif

// Compact source of the LDS round tables (the fill_ttab_dma source), built once per ctx:
// 16 KiB, entry e (16 bytes = 4 copies of one table value) for the 128-byte run of LDS
// (32 lane copies of table t at index x) that starts at byte e * 128 of the LDS image.  Every
// lane of an LDS-DMA instruction fetches its 16 bytes from entry (LDS offset / 128), so a
// block moves 16 KiB from L2 instead of a 128 KiB replicated image (ttab_src, hfv_aes_dev.h).
__global__ void k_build_ttab_image(uint32_t *__restrict__ img)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int)kTtabImageDwords) return;
    const int e = i >> 2;
    const uint32_t t0 = c_t0[(e >> 1) & 255];
    const int t = (e & 1) | (((e >> 9) & 1) << 1);
    img[i] = t ? __builtin_amdgcn_alignbit(t0, t0, 32 - 8 * t) : t0;
}

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
// NT: non-temporal loads (records are read once per launch).  The resident service uses
// plain, cache-allocating loads instead: a batch re-posted from the same ring slots (the
// benchmark re-verifies one resident 64 MiB batch) is then served from the Infinity Cache
// (measured at 2^20: +8-10 %; neutral at 2^24, where the batch does not fit).
template <bool NT = true>
__device__ __forceinline__ RecWords load_rec(const uint8_t *recs, uint64_t stride, uint64_t i, uint64_t last,
                                             uint32_t inf_off, uint32_t hf_off)
{
    RecWords r;
    // global address space even when `recs` came out of memory (the service's descriptors),
    // so these are global_load (vmcnt only), not flat loads that also count in lgkmcnt
    const GlobalU8 *p = (const GlobalU8 *)(recs) + (i < last ? i : last) * stride;
    typedef const __attribute__((address_space(1))) u32x2 *P2;
    typedef const __attribute__((address_space(1))) uint32_t *P1;
    u32x2 a, b;
    if constexpr (NT) {
        a = __builtin_nontemporal_load(reinterpret_cast<P2>(p + inf_off));
        b = __builtin_nontemporal_load(reinterpret_cast<P2>(p + hf_off));
        r.hfb = __builtin_nontemporal_load(reinterpret_cast<P1>(p + hf_off + 8));
    } else {
        a = *reinterpret_cast<P2>(p + inf_off);
        b = *reinterpret_cast<P2>(p + hf_off);
        r.hfb = *reinterpret_cast<P1>(p + hf_off + 8);
    }
    r.inf = make_uint2(a.x, a.y);
    r.hfa = make_uint2(b.x, b.y);
    return r;
}

// Same words read with system-scope (L1/L2-bypassing, coherent) loads: what the resident
// service uses when it may not invalidate the caches per batch (HFV_SVC_ACQ == 2).
__device__ __forceinline__ RecWords load_rec_sys(const uint8_t *recs, uint64_t stride, uint64_t i, uint64_t last,
                                                 uint32_t inf_off, uint32_t hf_off)
{
    RecWords r;
    const uint8_t *p = recs + (i < last ? i : last) * stride;
    uint64_t a = __hip_atomic_load(reinterpret_cast<const uint64_t *>(p + inf_off), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t b = __hip_atomic_load(reinterpret_cast<const uint64_t *>(p + hf_off), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    r.inf = make_uint2((uint32_t)a, (uint32_t)(a >> 32));
    r.hfa = make_uint2((uint32_t)b, (uint32_t)(b >> 32));
    r.hfb = __hip_atomic_load(reinterpret_cast<const uint32_t *>(p + hf_off + 8), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
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

// One tile = 64 consecutive records = one wave.  A wave computes NP tiles at once (NP
// independent AES chains per lane, interleaved by the scheduler to hide LDS latency), and
// loads its next NP tiles while it computes the current ones (PF = prefetch depth in
// iterations).  Tiles of one wave: t, t + nwaves, t + 2*nwaves, ...
// RET = 1: return the ballots in ret[] instead of storing them (the resident service
// batches its verdict stores).
template <int KEYSEL, int TAB, int NP, int RET = 0>
__device__ __forceinline__ void verify_tiles(const RecWords (&cur)[NP], uint64_t t, uint64_t nwaves, uint64_t n,
                                             uint32_t lane, const Lane &l, const UniformKey *ukey,
                                             uint64_t *__restrict__ bits, uint64_t *ret = nullptr)
{
    uint32_t s[NP][4];
    uint32_t slot[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        uint32_t w[4];
        rec_macinput(cur[p], w);
        slot[p] = rec_key_slot(cur[p]);
        uint4 k0;
        if constexpr (KEYSEL == HFV_KEYSEL_ZERO) k0 = ukey->row(0);
        else k0 = LdsKey(slot[p]).row(0);
        s[p][0] = w[0] ^ k0.x; s[p][1] = w[1] ^ k0.y; s[p][2] = w[2] ^ k0.z; s[p][3] = w[3] ^ k0.w;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        if constexpr (KEYSEL == HFV_KEYSEL_ZERO) round1_macinput<TAB>(s[p], ukey->row(11), l);
        else round1_macinput<TAB>(s[p], LdsKey(slot[p]).row(11), l);
    }
#pragma unroll
    for (int r = 2; r < 10; ++r) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if constexpr (KEYSEL == HFV_KEYSEL_ZERO) round_full<TAB>(s[p], ukey->template rk<TAB>(r), l);
            else round_full<TAB>(s[p], LdsKey(slot[p]).template rk<TAB>(r), l);
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        uint32_t t0, t1;
        bool ok = (t + p * nwaves) * 64 + lane < n;
        if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
            round_last_48<TAB>(s[p], ukey->row(10), l, t0, t1);
        } else {
            const LdsKey key(slot[p]);
            round_last_48<TAB>(s[p], key.row(10), l, t0, t1);
            ok = ok && key.ok();
        }
        bool pass = ok && rec_tag_matches(cur[p], t0, t1);
        uint64_t ballot = __ballot(pass);
        if constexpr (RET)
            ret[p] = ballot;
        else if (lane == 0 && t + p * nwaves < (n + 63) / 64)
            ((GlobalU64 *)(bits))[t + p * nwaves] = ballot;
    }
}

// Per-interface keys gathered into VGPRs (GatherKey) with the 4-table LDS layout: an internal
// key-selection value for the kernels' template argument (the host still says
// HFV_KEYSEL_IFID; the slot rule is the same, xdp.c:151-157).
constexpr int kKeyselGather = 2;
// ... or with three LDS rows per slot and rounds 3..10's keys expanded per packet (SchedKey).
constexpr int kKeyselSched = 3;

// One tile with the per-lane key rows already issued (GatherKey::issue): the verdict ballot.
template <int TAB>
__device__ __forceinline__ uint64_t verify_tile_gather(const RecWords &r, uint64_t t, uint64_t n, uint32_t lane,
                                                       const Lane &l, const GatherKey &key)
{
    uint32_t w[4];
    rec_macinput(r, w);
    uint32_t t0, t1;
    cmac48_macinput<TAB>(w, key, l, t0, t1);
    const bool pass = t * 64 + lane < n && key.ok() && rec_tag_matches(r, t0, t1);
    return __ballot(pass);
}

__device__ __forceinline__ uint64_t verify_tile_sched(const RecWords &r, uint64_t t, uint64_t n, uint32_t lane,
                                                      const Lane &l)
{
    uint32_t w[4];
    rec_macinput(r, w);
    const uint32_t slot = rec_key_slot(r);
    uint32_t t0, t1;
    cmac48_sched(w, slot, l, t0, t1);
    const bool ok = (s_valid[slot >> 5] >> (slot & 31)) & 1u;
    const bool pass = t * 64 + lane < n && ok && rec_tag_matches(r, t0, t1);
    return __ballot(pass);
}

// STAMP = 1 is a diagnostic build: lane 0 of every wave records s_memrealtime (100 MHz,
// chip-wide) at entry, after the table fill, after each of its first 10 tiles (12 in the
// static variant) and at exit into stamps[wave * 16 + k]; the dynamic variant also records
// s_memtime after the fill and at exit (slots 12, 13) for the in-kernel clock.  Nothing
// else reads the stamps.
// Dynamic variant: block b owns the contiguous tile range [b*T/G, (b+1)*T/G) and its waves
// pull tiles from an LDS counter, so waves that the LDS arbiter serves less often simply
// take fewer tiles instead of finishing last (static assignment left the last ~20 % of the
// kernel with few waves active: scripts/stamps.py).  A wave claims its next tile before
// computing the current one, so the next tile's record loads still overlap the rounds.
template <int KEYSEL, int BLOCK, int TAB, int DMA, int STAMP>
__device__ __forceinline__ void verify_dynamic(const DevKeyTable *__restrict__ tab,
                                               const uint32_t *__restrict__ ttab_img,
                                               const uint8_t *__restrict__ recs, uint64_t stride, uint64_t n,
                                               uint32_t inf_off, uint32_t hf_off, uint64_t *__restrict__ bits,
                                               uint64_t *__restrict__ st, const RecArgs &ka)
{
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t b0 = ntiles * blockIdx.x / gridDim.x, b1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    const uint32_t count = (uint32_t)(b1 - b0);
    const uint64_t last = n - 1;
    const uint32_t kWaves = BLOCK / 64;
    // first tile of each wave is static (wave index); the queue hands out the rest
    uint32_t t = wave_uniform(threadIdx.x / 64);
    UniformKey ukey(ka.key0, ka.key0_ok);   // from the kernel arguments: no second memory hop
    if (threadIdx.x == 0) s_next_tile = kWaves;
    // The wave's first records and its share of the table pieces are in flight together;
    // one vmcnt(0) then covers both (the table must be complete before the barrier).
    // (Waiting at the barrier only for the table, and for the records after it, needs the
    // record loads pinned ahead of the barrier and the waitcnt pass told that the LDS-DMA
    // writes are done; every form tried made the compiler drain the prefetch each tile.)
    RecWords cur;
    if constexpr (DMA && BLOCK == 1024 && HFV_FILL == 3) {
        // the first tile's records, then the tables from T0 in the kernel arguments
        cur = load_rec(recs, stride, (b0 + t) * 64 + lane, last, inf_off, hf_off);
        fill_ttab_karg<TAB>(ka.t0, threadIdx.x >> 6, BLOCK / 64);
    } else if constexpr (DMA && BLOCK == 1024 && HFV_FILL == 2) {
        // table pieces first, then the first tile's records: the pieces land (in order) and are
        // written to LDS while the records are still on their way from HBM
        TtabRegs<TAB> tr;
        tr.issue(ttab_img, threadIdx.x >> 6, BLOCK / 64);
        cur = load_rec(recs, stride, (b0 + t) * 64 + lane, last, inf_off, hf_off);
        tr.commit(threadIdx.x >> 6, BLOCK / 64);
    } else {
        cur = load_rec(recs, stride, (b0 + t) * 64 + lane, last, inf_off, hf_off);
        if constexpr (DMA) {
            fill_ttab_dma_issue<TAB, BLOCK>(ttab_img);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            fill_ttab<TAB>();
        }
    }
    if constexpr (KEYSEL == HFV_KEYSEL_IFID) fill_keys(tab);
    __syncthreads();
    const Lane l = lane_bases();
    int nst = 0;
    if constexpr (STAMP) {
        if (lane == 0) {
            st[1] = __builtin_amdgcn_s_memrealtime();
            st[12] = __builtin_amdgcn_s_memtime();   // shader clock, for the in-kernel frequency
        }
    }
    const UniformKey *ukp = nullptr;
    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
        if (!ukey.ok) {   // no key in slot 0: every packet fails closed (xdp.c:83-84)
            for (uint32_t tt = t; tt < count; tt += kWaves)
                if (lane == 0) bits[b0 + tt] = 0;
            return;
        }
        ukp = &ukey;
    }
    // Verdict words wait in a per-wave stash (lane j: the wave's j-th tile) and go out as one
    // store per 64 tiles: a store per tile sits in the in-order vmcnt queue, and the loop
    // latch (which waits for the prefetched record words) would wait for its write
    // acknowledgement every tile.
    uint64_t st_word = 0;
    uint32_t st_tile = 0, stashed = 0;
    while (t < count) {
        uint32_t nt = 0;
        if (lane == 0) nt = atomicAdd(&s_next_tile, 1u);
        nt = wave_uniform(nt);
        RecWords nxt = load_rec(recs, stride, (b0 + nt) * 64 + lane, last, inf_off, hf_off);
        RecWords c1[1] = {cur};
        uint64_t ballot;
        verify_tiles<KEYSEL, TAB, 1, 1>(c1, b0 + t, 0, n, lane, l, ukp, nullptr, &ballot);
        if (lane == stashed) {
            st_word = ballot;
            st_tile = t;
        }
        if (++stashed == 64) {
            ((GlobalU64 *)bits)[b0 + st_tile] = st_word;
            stashed = 0;
        }
        if constexpr (STAMP) {
            if (lane == 0 && nst < 10) st[2 + nst] = __builtin_amdgcn_s_memrealtime();
            ++nst;
        }
        cur = nxt;
        t = nt;
    }
    if (lane < stashed) ((GlobalU64 *)bits)[b0 + st_tile] = st_word;
    if constexpr (STAMP) {
        if (lane == 0) {
            st[13] = __builtin_amdgcn_s_memtime();
            st[15] = __builtin_amdgcn_s_memrealtime();
            st[14] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                     ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
        }
    }
}

// ---------------------------------------------------------------------------------------
// bitsliced verify (hfv_bitslice.h): VALU-only AES for chunks of 512 records per wave
// ---------------------------------------------------------------------------------------
// Per-wave LDS staging of a chunk: 6 words per record (macinput w0..w3, expected MAC words
// e0 = mac0..3, e1 = mac4..5), quad q's 32 records at dword q * kBsQuadStride + 6 p.  The
// 4-dword pad per quad makes the transposing reads (lane (q, c) reads word c of record p of
// quad q, all lanes the same p) bank-conflict free: bank = (4 q + c + 6 p) % 32.
constexpr uint32_t kBsChunk = 512;                 // records per wave per chunk = 8 tiles
constexpr uint32_t kBsQuadStride = 32 * 6 + 4;     // dwords
constexpr uint32_t kBsWaveDwords = 16 * kBsQuadStride;
constexpr uint32_t kBsMaxWaves = 4;
static __shared__ uint32_t s_bs[kBsMaxWaves * kBsWaveDwords];   // 49 KiB
static __shared__ uint32_t s_fill_done;

// AddRoundKey + ShiftRows on the quad: row r of lane c comes from lane (c + r) % 4
// (DPP quad_perm on the XOR's first operand).
template <int R>
__device__ __forceinline__ uint32_t quad_rot(uint32_t v)
{
    constexpr int ctrl = R == 1 ? 0x39 : R == 2 ? 0x4e : 0x93;   // quad_perm [1230], [2301], [3012]
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xf, 0xf, false);
}
__device__ __forceinline__ void bs_ark_sr(uint32_t (&s)[32], uint32_t kk)
{
#pragma unroll
    for (int b = 0; b < 8; ++b) s[b] ^= bs::kmask(kk, b);
#pragma unroll
    for (int b = 0; b < 8; ++b) s[8 + b] = quad_rot<1>(s[8 + b]) ^ bs::kmask(kk, 8 + b);
#pragma unroll
    for (int b = 0; b < 8; ++b) s[16 + b] = quad_rot<2>(s[16 + b]) ^ bs::kmask(kk, 16 + b);
#pragma unroll
    for (int b = 0; b < 8; ++b) s[24 + b] = quad_rot<3>(s[24 + b]) ^ bs::kmask(kk, 24 + b);
}

// The lane's key column for the ARK+SR step before round r + 1 (r = 0..9): row 0 of the
// device key image is rk0 ^ K1, rows 1..9 are rot16 of rk1..rk9 (hfv_tables.h).  The row is
// a wave-uniform scalar load (K$), so the round loop need not be unrolled to keep keys in
// registers.
// The four candidate words are formed on the scalar unit; the lane picks its column with
// per-lane all-ones/all-zeros selectors (sel[k] = -(c == k)), so nothing branches on c.
struct BsLaneSel {
    uint32_t sel[4];
    __device__ __forceinline__ explicit BsLaneSel(uint32_t c)
    {
#pragma unroll
        for (int k = 0; k < 4; ++k) sel[k] = vconst(0) - (c == (uint32_t)k ? 1u : 0u);
    }
    __device__ __forceinline__ uint32_t pick(const uint32_t (&w)[4]) const
    {
        return (w[0] & sel[0]) | (w[1] & sel[1]) | (w[2] & sel[2]) | (w[3] & sel[3]);
    }
};
__device__ __forceinline__ uint32_t bs_round_key(const DevKeyTable *tab, uint32_t r, const BsLaneSel &ls)
{
    const uint32_t *p = tab->rows[r][0];
    uint32_t w[4] = {p[0], p[1], p[2], p[3]};
    if (r >= 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (w[i] >> 16) | (w[i] << 16);
    }
    uint32_t k[4];   // k[c] = the pre-shifted key column of lane c (bs::shifted_key_column)
#pragma unroll
    for (int c = 0; c < 4; ++c)
        k[c] = (w[c] & 0xffu) | (w[(c + 1) & 3] & 0xff00u) | (w[(c + 2) & 3] & 0xff0000u) | (w[(c + 3) & 3] & 0xff000000u);
    return ls.pick(k);
}
// column c of rk10, added after the last SubBytes (no shift)
__device__ __forceinline__ uint32_t bs_final_key(const DevKeyTable *tab, const BsLaneSel &ls)
{
    const uint32_t *p = tab->rows[10][0];
    const uint32_t w[4] = {p[0], p[1], p[2], p[3]};
    return ls.pick(w);
}

// One chunk of up to 512 records [base, base + 512) by one wave: coalesced record loads
// (8 tiles), macinput + expected words staged in the wave's LDS region, transposed into
// bit planes per quad, 10 bitsliced rounds, then the 48-bit compare (xdp.c:89-90) in the
// bitsliced domain: lane 0 of a quad holds tag bytes 0..3 (column 0), lane 1 bytes 4..5.
// Records >= limit get a 0 bit; words32 = number of 32-bit bitmap words that may be written.
__device__ __forceinline__ void bs_chunk(const uint8_t *__restrict__ recs, uint64_t stride, uint64_t base,
                                         uint64_t limit, uint32_t inf_off, uint32_t hf_off, uint32_t *lds,
                                         const DevKeyTable *__restrict__ tab, uint32_t *__restrict__ bits32, uint64_t words32,
                                         uint32_t lane)
{
    const uint64_t last = limit - 1;
    RecWords r[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) r[it] = load_rec(recs, stride, base + it * 64 + lane, last, inf_off, hf_off);
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        uint32_t w[4];
        rec_macinput(r[it], w);
        uint32_t e0 = __builtin_amdgcn_alignbit(r[it].hfb, r[it].hfa.y, 16), e1 = r[it].hfb >> 16;
        uint32_t *d = lds + (2 * it + (lane >> 5)) * kBsQuadStride + 6 * (lane & 31);
        *reinterpret_cast<uint2 *>(d) = make_uint2(w[0], w[1]);
        *reinterpret_cast<uint2 *>(d + 2) = make_uint2(w[2], w[3]);
        *reinterpret_cast<uint2 *>(d + 4) = make_uint2(e0, e1);
    }
    const uint32_t q = lane >> 2, c = lane & 3;
    const BsLaneSel ls(c);
    const uint32_t *src = lds + q * kBsQuadStride + c;
    uint32_t s[32];
#pragma unroll
    for (int p = 0; p < 32; ++p) s[p] = src[6 * p];
    bs::transpose32(s);
#pragma unroll 1
    for (uint32_t rd = 0; rd < 9; ++rd) {
        bs_ark_sr(s, bs_round_key(tab, rd, ls));
        bs::sub_bytes(s);
        bs::mix_columns(s);
    }
    bs_ark_sr(s, bs_round_key(tab, 9, ls));
    bs::sub_bytes(s);
    const uint32_t k10 = bs_final_key(tab, ls);
    uint32_t e[32];
    const uint32_t *es = lds + q * kBsQuadStride + 4 + (c & 1);
#pragma unroll
    for (int p = 0; p < 32; ++p) e[p] = es[6 * p];
    bs::transpose32(e);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) lo |= HFV_BOP3(s[i], e[i], bs::kmask(k10, i), 0x96);
#pragma unroll
    for (int i = 16; i < 32; ++i) hi |= HFV_BOP3(s[i], e[i], bs::kmask(k10, i), 0x96);
    uint32_t m = lo | (c == 0 ? hi : 0u);
    m |= (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x55, 0xf, 0xf, false);   // quad_perm [1111]: + lane 1
    const uint64_t first = base + 32 * q;
    uint32_t valid = first >= limit ? 0u : (limit - first >= 32 ? ~0u : ((1u << (limit - first)) - 1u));
    const uint64_t word = base / 32 + q;
    if (c == 0 && word < words32) bits32[word] = ~m & valid;
}

// Pure bitsliced verify (KEYSEL_ZERO): every wave works through 512-record chunks.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_verify_bs(const DevKeyTable *__restrict__ tab,
                                                     const uint32_t *__restrict__ ttab_img,
                                                     const uint8_t *__restrict__ recs, uint64_t stride, uint64_t n,
                                                     uint32_t inf_off, uint32_t hf_off, uint64_t *__restrict__ bits,
                                                     uint64_t *__restrict__ stamps, const RecArgs ka)
{
    static_assert(BLOCK / 64 <= (int)kBsMaxWaves, "LDS staging regions");
    const uint32_t lane = threadIdx.x & 63, wv = wave_uniform(threadIdx.x / 64);
    const uint64_t nchunks = (n + kBsChunk - 1) / kBsChunk, words32 = 2 * ((n + 63) / 64);
    const uint64_t nwaves = (uint64_t)gridDim.x * (BLOCK / 64);
    UniformKey ukey(tab);
    uint32_t *bits32 = reinterpret_cast<uint32_t *>(bits);
    if (!ukey.ok) {   // no key in slot 0: every packet fails closed (xdp.c:83-84)
        for (uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; w < words32; w += (uint64_t)gridDim.x * BLOCK)
            bits32[w] = 0;
        return;
    }
    uint32_t *lds = s_bs + wv * kBsWaveDwords;
    for (uint64_t ch = (uint64_t)blockIdx.x * (BLOCK / 64) + wv; ch < nchunks; ch += nwaves)
        bs_chunk(recs, stride, ch * kBsChunk, n, inf_off, hf_off, lds, tab, bits32, words32, lane);
}

// Hybrid verify (KEYSEL_ZERO): per block, NBS waves run the bitsliced VALU path on 512-record
// chunks while the other waves run the LDS T-table path on 64-record tiles, both pulling
// from the block's tile queue over its contiguous tile range.  Only the T-table waves wait
// for the table fill (an LDS counter, not a block barrier), so the bitsliced waves start at
// once.  A bitsliced wave stops claiming when fewer than kBsStop tiles would remain for the
// T-table waves, so the block does not end on a long bitsliced chunk.
template <int BLOCK, int NBS>
__global__ __launch_bounds__(BLOCK) void k_verify_hybrid(const DevKeyTable *__restrict__ tab,
                                                         const uint32_t *__restrict__ ttab_img,
                                                         const uint8_t *__restrict__ recs, uint64_t stride,
                                                         uint64_t n, uint32_t inf_off, uint32_t hf_off,
                                                         uint64_t *__restrict__ bits, uint64_t *__restrict__ stamps,
                                                         const RecArgs ka)
{
    static_assert(NBS >= 1 && NBS <= (int)kBsMaxWaves && NBS < BLOCK / 64, "wave roles");
    constexpr uint32_t kWaves = BLOCK / 64, kTT = kWaves - NBS;
    constexpr uint32_t kChunkTiles = kBsChunk / 64;
    constexpr uint32_t kBsStop = kChunkTiles + 2 * kTT;
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63, wv = wave_uniform(threadIdx.x / 64);
    const uint64_t b0 = ntiles * blockIdx.x / gridDim.x, b1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    const uint32_t count = (uint32_t)(b1 - b0);
    const uint64_t last = n - 1;
    UniformKey ukey(tab);
    RecWords cur = load_rec(recs, stride, (b0 + (wv < kTT ? wv : 0)) * 64 + lane, last, inf_off, hf_off);
    if (threadIdx.x == 0) {
        s_next_tile = kTT;   // tiles 0..kTT-1 are the T-table waves' first tiles
        s_fill_done = 0;
    }
    __syncthreads();
    if (!ukey.ok) {   // no key in slot 0: every packet fails closed (xdp.c:83-84)
        for (uint32_t t = wv; t < count; t += kWaves)
            if (lane == 0) bits[b0 + t] = 0;
        return;
    }
    if (wv >= kTT) {   // bitsliced waves
        uint32_t *lds = s_bs + (wv - kTT) * kBsWaveDwords;
        uint32_t *bits32 = reinterpret_cast<uint32_t *>(bits);
        for (;;) {
            uint32_t t0 = count;
            if (lane == 0) {
                uint32_t head = __hip_atomic_load(&s_next_tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (head + kBsStop <= count) t0 = atomicAdd(&s_next_tile, kChunkTiles);
            }
            t0 = wave_uniform(t0);
            if (t0 >= count) break;
            const uint32_t t1 = t0 + kChunkTiles < count ? t0 + kChunkTiles : count;
            const uint64_t lim = (b0 + t1) * 64 < n ? (b0 + t1) * 64 : n;
            bs_chunk(recs, stride, (b0 + t0) * 64, lim, inf_off, hf_off, lds, tab, bits32, 2 * (b0 + t1), lane);
        }
        return;
    }
    // T-table waves: share the table fill, then wait on the LDS counter (acquire) for all of it
    {
        const int nw = kTT;
        char *ldst = reinterpret_cast<char *>(s_tab64);
        for (int ch = wv; ch < 64; ch += nw) {
            const char *src = ttab_src(ttab_img, ch, lane);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(ldst + ch * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(&s_fill_done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&s_fill_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < kTT)
            __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_s_setprio(3);   // issue ahead of the bitsliced waves on a shared SIMD
    const Lane l = lane_bases();
    uint32_t t = wv;
    while (t < count) {
        uint32_t nt = 0;
        if (lane == 0) nt = atomicAdd(&s_next_tile, 1u);
        nt = wave_uniform(nt);
        RecWords nxt = load_rec(recs, stride, (b0 + nt) * 64 + lane, last, inf_off, hf_off);
        RecWords c1[1] = {cur};
        verify_tiles<HFV_KEYSEL_ZERO, 2, 1>(c1, b0 + t, 0, n, lane, l, &ukey, bits);
        cur = nxt;
        t = nt;
    }
}

template <int KEYSEL, int BLOCK, int PF, int TAB, int DMA, int NP, int STAMP = 0, int DYN = 0>
__global__ __launch_bounds__(BLOCK) void k_verify_records(const DevKeyTable *__restrict__ tab,
                                                          const uint32_t *__restrict__ ttab_img,
                                                          const uint8_t *__restrict__ recs, uint64_t stride,
                                                          uint64_t n, uint32_t inf_off, uint32_t hf_off,
                                                          uint64_t *__restrict__ bits, uint64_t *__restrict__ stamps,
                                                          const RecArgs ka)
{
    static_assert(PF == 1 || PF == 2, "prefetch depth");
    static_assert(NP == 1 || NP == 2, "packets per lane");
    static_assert(KEYSEL == HFV_KEYSEL_ZERO || TAB == 2, "per-lane keys need the 64 KiB table layout");
    constexpr uint32_t kWaves = BLOCK / 64;
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform(blockIdx.x * kWaves + threadIdx.x / 64);
    const uint64_t nwaves = gridDim.x * kWaves;
    uint64_t *st = STAMP ? stamps + (uint64_t)wave * 16 : nullptr;
    int nst = 0;
    if constexpr (STAMP) {
        if (lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
    }

    if constexpr (DYN) {
        verify_dynamic<KEYSEL, BLOCK, TAB, DMA, STAMP>(tab, ttab_img, recs, stride, n, inf_off, hf_off, bits, st, ka);
        return;
    }
    // First tiles' record loads go out before the table fill so the fill overlaps their
    // memory latency.
    const uint64_t last = n - 1;
    const uint64_t step = NP * nwaves;   // tiles consumed per iteration by the whole grid
    uint64_t t = wave;
    RecWords cur[NP], nx1[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) cur[p] = load_rec(recs, stride, (t + p * nwaves) * 64 + lane, last, inf_off, hf_off);
    if constexpr (PF == 2) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
            nx1[p] = load_rec(recs, stride, (t + step + p * nwaves) * 64 + lane, last, inf_off, hf_off);
    }
    UniformKey ukey(tab);

    if constexpr (DMA) {
        fill_ttab_dma_issue<TAB, BLOCK>(ttab_img);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        fill_ttab<TAB>();
    }
    if constexpr (KEYSEL == HFV_KEYSEL_IFID) fill_keys(tab);
    __syncthreads();
    const Lane l = lane_bases();
    if constexpr (STAMP) {
        if (lane == 0) st[1] = __builtin_amdgcn_s_memrealtime();
    }

    const UniformKey *ukp = nullptr;
    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
        if (!ukey.ok) {   // no key in slot 0: every packet fails closed (xdp.c:83-84)
            for (uint64_t tt = wave; tt < ntiles; tt += nwaves)
                if (lane == 0) bits[tt] = 0;
            return;
        }
        ukp = &ukey;
    }
    for (; t < ntiles; t += step) {
        RecWords nxt[NP];
#pragma unroll
        for (int p = 0; p < NP; ++p)
            nxt[p] = load_rec(recs, stride, (t + PF * step + p * nwaves) * 64 + lane, last, inf_off, hf_off);
        verify_tiles<KEYSEL, TAB, NP>(cur, t, nwaves, n, lane, l, ukp, bits);
        if constexpr (STAMP) {
            if (lane == 0 && nst < 12) st[2 + nst] = __builtin_amdgcn_s_memrealtime();
            ++nst;
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if constexpr (PF == 2) {
                cur[p] = nx1[p];
                nx1[p] = nxt[p];
            } else {
                cur[p] = nxt[p];
            }
        }
    }
    if constexpr (STAMP) {
        if (lane == 0) {
            st[15] = __builtin_amdgcn_s_memrealtime();
            // placement: HW_REG_HW_ID (hwreg 4, all 32 bits) and HW_REG_XCC_ID (hwreg 20)
            st[14] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                     ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
        }
    }
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

#ifndef HFV_SVC_ACQ
#define HFV_SVC_ACQ 1   // 0: none, 1: acquire fence per loaded batch, 2: system-scope record loads
#endif
// HFV_SVC_PROF = 1: diagnostic build; every wave sums the shader cycles (s_memtime) it spends
// in each phase of the service loop and adds them to host->prof[] at exit:
//   0 waiting for the current tile's records at the top of the loop, 1 claim + map + next
//   tile's loads, 2 the tile's AES rounds and verdict, 3 verdict stores + completion count,
//   4 blocking waits for a descriptor, 5 tiles verified, 6 the wave's whole loop.
#ifndef HFV_SVC_PROF
#define HFV_SVC_PROF 0
#endif
// HFV_SVC_SPAN = 1: diagnostic build; block entry, table-fill and wave exit stamps
// (s_memrealtime, 100 MHz) into dev->span_* (hfv_debug_service_span)
#ifndef HFV_SVC_SPAN
#define HFV_SVC_SPAN 0
#endif
// HFV_SVC_AHEAD = 1: the next tile's number is claimed one iteration early (a wave then holds
// three tiles: the one it computes, the one whose records are loading, the claimed one); 0 (the
// default): it is claimed at the top of the iteration that loads its records, so a wave holds
// two and the block's last tiles go to whichever waves are free one tile-time later: K = 20
// grids 2.1-2.4 % shorter (profiles/r03/ahead_ab/), the claim's LDS latency is not missed.
#ifndef HFV_SVC_AHEAD
#define HFV_SVC_AHEAD 0
#endif
// Only wave 1 of every block samples (s_memtime from every wave of a CU slowed the loop
// many times over); the other waves run the plain loop beside it.
struct SvcProf {
    uint64_t c[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t t = 0;
    bool on = false;
    __device__ __forceinline__ void start()
    {
        if constexpr (HFV_SVC_PROF) {
            on = wave_uniform(threadIdx.x >> 6) == 1;
            if (on) t = __builtin_amdgcn_s_memtime();
        }
    }
    __device__ __forceinline__ void mark(int k)
    {
        if constexpr (HFV_SVC_PROF) {
            if (!on) return;
            uint64_t now = __builtin_amdgcn_s_memtime();
            c[k] += now - t;
            t = now;
        }
    }
    __device__ __forceinline__ void flush(SvcShared *host, uint32_t lane, uint64_t t0)
    {
        if constexpr (HFV_SVC_PROF) {
            if (!on) return;
            c[6] = __builtin_amdgcn_s_memtime() - t0;
            if (lane == 0)
                for (int k = 0; k < 7; ++k)
                    __hip_atomic_fetch_add(&host->prof[k], c[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
};

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
#if HFV_SVC_ACQ == 1
    // the batch's records were written (by a kernel or a copy into device memory) before the
    // host posted it: drop this CU's stale L1 lines (agent scope, buffer_inv sc1)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#elif HFV_SVC_ACQ == 3
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope (buffer_inv sc0 sc1: L1 and L2)
#endif
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

template <int KEYSEL, int TAB>
__global__ __launch_bounds__(1024) void k_verify_service(const SvcArgs args)
{
    // the fields through the kernarg segment pointer (constant address space): no private copy
    // of the 2.4 KB argument struct, and helpers take the pointer
    const KArgs a = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    (void)args;
    const uint32_t lane = threadIdx.x & 63;
    SvcDev *dev = a->dev;
    if (HFV_SVC_SPAN && threadIdx.x == 0) dev->span_entry[blockIdx.x] = memrealtime();
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
#if HFV_SVC_FILL_DMA
    if (!relay) fill_ttab_dma_issue_n<TAB>(a->ttab_img, threadIdx.x >> 6, nthr >> 6);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
    if (!relay) fill_ttab_karg<TAB>(a->t0, threadIdx.x >> 6, nthr >> 6);
#endif
    if constexpr (KEYSEL == HFV_KEYSEL_IFID) {
        if (!relay) fill_keys(a->tab, nthr);
    } else if constexpr (KEYSEL == kKeyselGather) {
        fill_valid(a->tab);
    } else if constexpr (KEYSEL == kKeyselSched) {
        if (!relay) fill_keys3(a->tab, nthr);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        dev->blk_start[blockIdx.x] = memrealtime();
        dev->blk_clk0[blockIdx.x] = __builtin_amdgcn_s_memtime();
    }
    if (HFV_SVC_SPAN && threadIdx.x == 0) dev->span_fill[blockIdx.x] = memrealtime();
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
    // next tile (LDS atomic; HFV_SVC_AHEAD = 1 claimed it one iteration earlier still), store the
    // verdict words of a batch the wave left in the previous
    // iteration (so their write acknowledgement arrives while this tile computes and is
    // covered by the next iteration's wait), map the next tile and issue its loads, compute.
    // Measured with the HFV_SVC_PROF build on the loop this replaces (claim at the top, store
    // and a vmcnt(0) drain when leaving a batch): claim/map/load 10 %, store/count drain
    // 9-20 % of a wave's cycles.
    auto claim = [&]() -> uint32_t {
        uint32_t g = 0;
        if (lane == 0) g = __hip_atomic_fetch_add(&s_svc_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return g;
    };
    SvcTile cur;
    if (svc_map(a, lane, wave_uniform(claim()), true, mb, none, cur) != kSvcFound) return;
    uint32_t gq = HFV_SVC_AHEAD ? claim() : 0u;   // the next tile's number (lane 0), read one iteration later
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
    SvcProf prof;
    const uint64_t prof_t0 = HFV_SVC_PROF ? __builtin_amdgcn_s_memtime() : 0;
    prof.start();
    for (;;) {
        // This tile's record words (and every earlier store) are complete.  An explicit wait
        // (a builtin, so the waitcnt pass sees it): without it the pass merges the loop's
        // entry paths and puts a vmcnt(0) AFTER the next tile's loads.
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
        count(dc_b, dc_count, dc_k);           // the stores of the previous iteration are acknowledged
        dc_k = 0;
        prof.mark(0);
        if (flush) {                           // the batch left in the previous iteration
            store_stash();
            dc_b = fl_b;
            dc_count = fl_count;
            dc_k = fl_k;
            flush = false;
        }
        // per-interface keys: this tile's key rows, issued BEFORE the next tile's record loads
        // (vmcnt retires in order: a row wait must not also wait for those HBM loads)
        GatherKey gk;
        if constexpr (KEYSEL == kKeyselGather) gk.issue(a->tab, rec_key_slot(rc));
        uint32_t g;
        if constexpr (HFV_SVC_AHEAD) {
            g = wave_uniform(gq);
            gq = claim();
        } else {
            g = wave_uniform(claim());
        }
        SvcTile nx;
        SvcClaim c = svc_map(a, lane, g, false, mb, cur, nx);
        if (c != kSvcFound) nx = cur;
        RecWords rn = load_tile(nx, lane, inf_off, hf_off);
        prof.mark(1);
        uint64_t ballot = 0;   // KEYSEL_ZERO with slot 0 empty: every packet fails closed
        if constexpr (KEYSEL == kKeyselGather) {
            ballot = verify_tile_gather<TAB>(rc, cur.tile, cur.n, lane, l, gk);
        } else if constexpr (KEYSEL == kKeyselSched) {
            ballot = verify_tile_sched(rc, cur.tile, cur.n, lane, l);
        } else if (keyok) {
            RecWords c1[1] = {rc};
            verify_tiles<KEYSEL, TAB, 1, 1>(c1, cur.tile, 0, cur.n, lane, l, ukp, nullptr, &ballot);
        }
        if constexpr (HFV_SVC_PROF) prof.c[5] += 1;
        prof.mark(2);
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
        prof.mark(3);
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
        prof.mark(4);
        if (c == kSvcStop) break;
        if (nx.b != cur.b) svc_prefetch(a, lane, nx.b);
        cur = nx;
        rc = rn;
    }
    prof.flush(a->host, lane, prof_t0);
    if (HFV_SVC_SPAN && lane == 0) dev->span_exit[blockIdx.x * 16 + (threadIdx.x >> 6)] = memrealtime();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dev->run_clock[2] = __builtin_amdgcn_s_memtime();
        dev->run_clock[3] = memrealtime();
    }
}

// Diagnostics (hfv_debug_publish_delay): hold a stream for `us` microseconds, bounded by the
// 100 MHz s_memrealtime, so a test can queue a key-table publish behind it deterministically.
__global__ void k_debug_spin(uint32_t us)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(8);
}

int launch_debug_spin(void *stream, uint32_t us)
{
    if (us > 1000000u) us = 1000000u;
    hipLaunchKernelGGL(k_debug_spin, dim3(1), dim3(64), 0, (hipStream_t)stream, us);
    return (int)hipGetLastError();
}

int launch_verify_service(const LaunchGeom &g, int keysel, const SvcArgs &args, void *stream, void *ev_start,
                          void *ev_stop, unsigned *grid_out)
{
    // Per-interface keys (config 3).  Default: three LDS rows per slot beside all four round
    // tables, rounds 3..10's keys expanded per packet (SchedKey): bank-conflict cycles 1.37 M ->
    // 0.38 M per 2^20 batch, LDS-active cycles -6 %, 0.5-2.6 % faster (profiles/r03/pmc/,
    // ifid_ab/).  HFV_SVC_IFID=lds: the round-2 layout (48 KiB key image beside two tables and
    // a 16-bit rotation per column).  HFV_SVC_IFID=gather: each packet's key rows gathered from
    // L2 into VGPRs beside all four tables -- 2x slower (31 vs 63 Gpkt/s, profiles/r03/ifid_gather/):
    // 11 scattered 16-byte loads per lane per tile hold the vector-memory path ~100 cycles each.
    static const char *iv = getenv("HFV_SVC_IFID");
    static const int ifv = !iv ? 2 : !strcmp(iv, "gather") ? 1 : !strcmp(iv, "lds") ? 0 : 2;
    auto k = keysel != HFV_KEYSEL_IFID ? k_verify_service<HFV_KEYSEL_ZERO, 4>
             : ifv == 1               ? k_verify_service<kKeyselGather, 4>
             : ifv == 2               ? k_verify_service<kKeyselSched, 4>
                                      : k_verify_service<HFV_KEYSEL_IFID, 2>;
    const char *ge = getenv("HFV_SVC_GRID");   // experiments only: fewer blocks than CUs
    unsigned grid = ge && atoi(ge) > 0 && atoi(ge) < g.num_cus ? (unsigned)atoi(ge) : (unsigned)g.num_cus;
    if (grid > kSvcMaxBlocks) grid = kSvcMaxBlocks;
    *grid_out = grid;
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(1024), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
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
        uint32_t(*g)[4] = tab->gather[slot];   // slot-major copy (hfv_internal.h)
        for (int c = 0; c < 4; ++c) {
            g[0][c] = k0[c];
            g[1][c] = p[c];
            g[10][c] = w[40 + c];
        }
        for (int r = 2; r < 10; ++r)
            for (int c = 0; c < 4; ++c) g[r][c] = w[4 * r + c];
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

using VerifyKernel = void (*)(const DevKeyTable *, const uint32_t *, const uint8_t *, uint64_t, uint64_t, uint32_t,
                              uint32_t, uint64_t *, uint64_t *, const RecArgs);

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

// Record-verify variants (tuning knobs; the default is chosen by scripts/sweep.py data).
template <int KEYSEL>
static VerifyKernel pick_verify(const KernelVariant &v)
{
    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {   // bitsliced paths: one key for all lanes
        if (v.bs == kBsOnly) return v.block == 256 ? k_verify_bs<256> : nullptr;
        if (v.bs > 0) {
            if (v.block != 1024 || !v.dma || v.tab != 2 || v.np != 1) return nullptr;
            if (v.bs == 1) return k_verify_hybrid<1024, 1>;
            if (v.bs == 2) return k_verify_hybrid<1024, 2>;
            if (v.bs == 3) return k_verify_hybrid<1024, 3>;
            if (v.bs == 4) return k_verify_hybrid<1024, 4>;
            return nullptr;
        }
    } else {
        if (v.bs) return nullptr;
    }
#define HFV_V(B, P, T)                                                                          \
    if (v.block == B && v.pf == P && v.tab == T && v.dma && v.np == 1 && v.dyn)                        \
        return k_verify_records<KEYSEL, B, P, T, 1, 1, 0, 1>;                                           \
    if (v.block == B && v.pf == P && v.tab == T && v.dma && v.np == 1) return k_verify_records<KEYSEL, B, P, T, 1, 1>; \
    if (v.block == B && v.pf == P && v.tab == T && v.dma && v.np == 2) return k_verify_records<KEYSEL, B, P, T, 1, 2>; \
    if (v.block == B && v.pf == P && v.tab == T && !v.dma && v.np == 1) return k_verify_records<KEYSEL, B, P, T, 0, 1>;
    HFV_V(1024, 1, 2) HFV_V(1024, 2, 2) HFV_V(768, 1, 2) HFV_V(512, 1, 2)
    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
        HFV_V(1024, 1, 4) HFV_V(768, 1, 4)
    }
#undef HFV_V
    return nullptr;
}

int launch_verify_records(const LaunchGeom &g, const DevKeyTable *tab, const DevKeyTable *host_keys, int keysel,
                          const uint8_t *recs,
                          size_t stride, size_t n, uint32_t inf_off, uint32_t hf_off, uint64_t *bits, void *stream,
                          void *ev_start, void *ev_stop, bool interleaved)
{
    KernelVariant v = keysel == HFV_KEYSEL_IFID ? g.multi : g.single;
    if (interleaved && v.bs == 0) v.dyn = 0;   // the static kernel walks the tiles grid-stride
    VerifyKernel k = keysel == HFV_KEYSEL_IFID ? pick_verify<HFV_KEYSEL_IFID>(v) : pick_verify<HFV_KEYSEL_ZERO>(v);
    if (!k) return (int)hipErrorInvalidConfiguration;
    unsigned grid = grid_for(n, v.block, g.num_cus, v.blocks_per_cu);
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(v.block), 0, (hipStream_t)stream, (hipEvent_t)ev_start,
                          (hipEvent_t)ev_stop, 0u, tab, (const uint32_t *)g.ttab_img, recs, (uint64_t)stride,
                          (uint64_t)n, inf_off, hf_off, bits, (uint64_t *)nullptr, rec_args(host_keys));
    return (int)hipGetLastError();
}

int launch_verify_stamped(const LaunchGeom &g, const DevKeyTable *tab, const DevKeyTable *host_keys, const uint8_t *recs,
                          size_t n,
                          uint64_t *bits, uint64_t *stamps, void *stream)
{
    const KernelVariant &v = g.single;
    unsigned grid = grid_for(n, 1024, g.num_cus, v.blocks_per_cu);
    auto k = v.tab == 4 ? (v.dyn ? k_verify_records<HFV_KEYSEL_ZERO, 1024, 1, 4, 1, 1, 1, 1>
                                 : k_verify_records<HFV_KEYSEL_ZERO, 1024, 1, 4, 1, 1, 1, 0>)
                        : (v.dyn ? k_verify_records<HFV_KEYSEL_ZERO, 1024, 1, 2, 1, 1, 1, 1>
                                 : k_verify_records<HFV_KEYSEL_ZERO, 1024, 1, 2, 1, 1, 1, 0>);
    hipLaunchKernelGGL(k, dim3(grid), dim3(1024), 0,
                       (hipStream_t)stream, tab, (const uint32_t *)g.ttab_img, recs, (uint64_t)64, (uint64_t)n,
                       (uint32_t)HFV_REC_INF_OFF, (uint32_t)HFV_REC_HF_OFF, bits, stamps, rec_args(host_keys));
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

// Persistent-grid geometry.  Defaults: see DESIGN.md section 4 (measured with
// scripts/sweep.py).  HFV_KVARIANT="block=768,pf=2,tab=2,bpc=2" overrides the KEYSEL_ZERO
// kernel and HFV_KVARIANT_IFID the per-lane-key kernel; blocks per CU are capped by the LDS
// a block needs and by the occupancy query.
static void parse_variant(const char *env, KernelVariant *v)
{
    if (!env) return;
    const char *p = env;
    while (*p) {
        int val = 0;
        if (sscanf(p, "block=%d", &val) == 1) v->block = val;
        else if (sscanf(p, "pf=%d", &val) == 1) v->pf = val;
        else if (sscanf(p, "tab=%d", &val) == 1) v->tab = val;
        else if (sscanf(p, "bpc=%d", &val) == 1) v->blocks_per_cu = val;
        else if (sscanf(p, "dma=%d", &val) == 1) v->dma = val;
        else if (sscanf(p, "np=%d", &val) == 1) v->np = val;
        else if (sscanf(p, "dyn=%d", &val) == 1) v->dyn = val;
        else if (sscanf(p, "bs=%d", &val) == 1) v->bs = val;
        const char *c = strchr(p, ',');
        if (!c) break;
        p = c + 1;
    }
}

static int finish_variant(int keysel, KernelVariant *v)
{
    VerifyKernel k = keysel == HFV_KEYSEL_IFID ? pick_verify<HFV_KEYSEL_IFID>(*v) : pick_verify<HFV_KEYSEL_ZERO>(*v);
    if (!k) return (int)hipErrorInvalidConfiguration;
    int lds = (v->tab == 4 ? 131072 : 65536) + (keysel == HFV_KEYSEL_IFID ? (int)sizeof(uint4) * kDevKeyRows * HFV_MAX_KEYS + 32 : 0);
    if (v->bs == kBsOnly) lds = (int)sizeof(s_bs);
    else if (v->bs > 0) lds += (int)sizeof(s_bs);
    int by_lds = (160 * 1024) / lds;
    int by_waves = 32 / (v->block / 64);
    int occ = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, v->block, 0);
    if (e != hipSuccess) return (int)e;
    int cap = by_lds < by_waves ? by_lds : by_waves;
    if (occ > 0 && occ < cap) cap = occ;
    if (cap < 1) cap = 1;
    if (v->blocks_per_cu <= 0 || v->blocks_per_cu > cap) v->blocks_per_cu = cap;
    return 0;
}

int build_ttab_image(uint32_t *img, void *stream)
{
    hipLaunchKernelGGL(k_build_ttab_image, dim3(kTtabImageDwords / 256), dim3(256), 0, (hipStream_t)stream, img);
    return (int)hipGetLastError();
}

int query_geometry(int device, LaunchGeom *g)
{
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return (int)e;
    g->num_cus = prop.multiProcessorCount;
    g->single = KernelVariant{1024, 1, 4, 1, 1, 1, 1, 0};
    g->multi = KernelVariant{1024, 1, 2, 1, 1, 1, 1, 0};
    parse_variant(getenv("HFV_KVARIANT"), &g->single);
    parse_variant(getenv("HFV_KVARIANT_IFID"), &g->multi);
    int rc = finish_variant(HFV_KEYSEL_ZERO, &g->single);
    if (rc) return rc;
    return finish_variant(HFV_KEYSEL_IFID, &g->multi);
}

}  // namespace hfv
