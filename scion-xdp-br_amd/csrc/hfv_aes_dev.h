// hfv_aes_dev.h -- device-side AES-128 / CMAC building blocks shared by the gfx950 kernels
// (record verify in hfv_kernels.hip, full border-router path in hfv_br_kernel.hip).
// Each translation unit gets its own copy of the LDS arrays and the constant T0 table
// (internal linkage); a kernel's LDS allocation counts only the arrays it touches.
#pragma once
#include <hip/hip_runtime.h>

#include "hfv_internal.h"

namespace hfv {
// ---------------------------------------------------------------------------------------
// tables
// ---------------------------------------------------------------------------------------
#define T0V(i) kTables.t0[i]
#define T0V8(i) T0V(i), T0V(i + 1), T0V(i + 2), T0V(i + 3), T0V(i + 4), T0V(i + 5), T0V(i + 6), T0V(i + 7)
#define T0V64(i) T0V8(i), T0V8(i + 8), T0V8(i + 16), T0V8(i + 24), T0V8(i + 32), T0V8(i + 40), T0V8(i + 48), T0V8(i + 56)
static __constant__ uint32_t c_t0[256] = {T0V64(0), T0V64(64), T0V64(128), T0V64(192)};
#undef T0V64
#undef T0V8
#undef T0V


// Round tables in LDS.  Layout (byte address of table t at index x for lane L):
//   (x << 8) | ((t & 1) << 7) | ((L & 31) << 2) | ((t >> 1) << 16)
// TAB = 2 keeps T0/T1 (64 KiB) and derives T2/T3 by a 16-bit rotation; TAB = 4 stores all
// four (128 KiB) and needs no rotation.
static __shared__ uint32_t s_tab64[16384];
static __shared__ uint32_t s_tab128[32768];
// TAB = 3: T0/T1 with kTab3Copies lane copies (4: 8 KiB) for kernels where AES is a small
// part of the work and LDS is needed for other things (the router kernel): byte address
//   (t << (10 + log2 copies)) | (x << (2 + log2 copies)) | ((L % copies) << 2)
// formed with a shift instead of v_perm.  The table bit sits above the bank bits, so the
// lanes that share a copy spread over 32 / copies banks by x (at 4 copies: 8 lanes of a
// 32-lane half over 8 banks); lanes of one copy still conflict when their x differ in the
// bank bits' range.  A translation unit may define HFV_TAB3_COPIES before including this header.
#ifndef HFV_TAB3_COPIES
#define HFV_TAB3_COPIES 16
#endif
constexpr uint32_t kTab3Copies = HFV_TAB3_COPIES;
constexpr uint32_t kTab3Log = kTab3Copies == 32 ? 5 : kTab3Copies == 16 ? 4 : kTab3Copies == 8 ? 3 : kTab3Copies == 4 ? 2 : 99;
static_assert(kTab3Log < 8, "HFV_TAB3_COPIES must be 4, 8, 16 or 32");
static __shared__ uint32_t s_tab32[256 * 2 * kTab3Copies];
static __shared__ uint4 s_keys[kDevKeyRows * HFV_MAX_KEYS];   // 48 KiB, round-major
static __shared__ uint32_t s_valid[8];
static __shared__ uint32_t s_next_tile;   // DYN: the block's tile queue head

// v_perm selector for state byte k: address byte 0 <- base byte 0 (copy + T0/T1 bit),
// byte 1 <- state byte k, byte 2 <- base byte 2 (T2/T3 bit), byte 3 <- 0.
constexpr uint32_t sel_byte(int k) { return 0x0c020400u | (uint32_t(k) << 8); }
constexpr uint32_t SEL_B0 = sel_byte(0), SEL_B1 = sel_byte(1), SEL_B2 = sel_byte(2), SEL_B3 = sel_byte(3);

__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }

// Round-table lookup of state byte K of w in the table whose lane-copy base is `base`.  The
// LDS byte address is one v_perm_b32: state byte K -> address byte 1, the lane's copy/table
// bits -> byte 0 (and byte 2 for T2/T3).  v_perm issues at half the rate of v_bitop3 on
// gfx950 (scripts/ubench/valu_rate.hip), but the full-rate alternative (a shift + a
// (v & 0xff00) | base bitop3 per byte: 7 issue slots per state word instead of 8) measured
// slower in the kernel (2^24 records: 257.5 vs 235.5 us, profiles/r01/addr_bitop3.log): the
// verify loop is bound by LDS issue and the lookup chain's latency, not by VALU throughput,
// and the second dependent instruction lengthens the address -> ds_read chain.
struct Lane;
template <int TAB, int K>
__device__ __forceinline__ uint32_t tlu(uint32_t w, uint32_t base, const Lane &l);

template <int TAB>
__device__ __forceinline__ void fill_ttab()
{
    if constexpr (TAB == 3) {
#pragma unroll 4
        for (int e = threadIdx.x; e < (int)(256 * 2 * kTab3Copies); e += blockDim.x) {
            uint32_t t = c_t0[(e >> kTab3Log) & 255];
            s_tab32[e] = (e >> (kTab3Log + 8)) ? __builtin_amdgcn_alignbit(t, t, 24) : t;   // T1 = rotl8(T0)
        }
        return;
    }
    constexpr int kDwords = TAB == 4 ? 32768 : 16384;
    uint32_t *dst = TAB == 4 ? s_tab128 : s_tab64;
#pragma unroll 4
    for (int e = threadIdx.x; e < kDwords; e += blockDim.x) {
        uint32_t t = c_t0[(e >> 6) & 255];
        int rot = 8 * (((e >> 5) & 1) | ((e >> 13) & 2));   // table index * 8
        dst[e] = rot ? __builtin_amdgcn_alignbit(t, t, 32 - rot) : t;
    }
}

// The tables written from T0 in the kernel arguments (constant address space, one memory hop
// with the rest of the arguments): every filling lane loads T0 of its chunks' runs and writes
// 16-byte pieces (4 copies of the table value) with ds_write_b128.
template <int TAB, class P>
__device__ __forceinline__ void fill_ttab_karg(P t0, uint32_t wave, uint32_t nw)
{
    constexpr uint32_t kChunks = (TAB == 4 ? 131072 : 65536) / 1024;
    constexpr int kMax = (int)((kChunks + 14) / 15);   // at least 15 filling waves
    const uint32_t lane = threadIdx.x & 63;
    char *lds = TAB == 4 ? reinterpret_cast<char *>(s_tab128) : reinterpret_cast<char *>(s_tab64);
    uint32_t v[kMax];
#pragma unroll
    for (int k = 0; k < kMax; ++k) {
        const uint32_t c = wave + k * nw;
        const uint32_t e = (c << 3) + (lane >> 3);   // 128-byte run of table t at index x
        v[k] = c < kChunks ? t0[(e >> 1) & 255u] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kMax; ++k) {
        const uint32_t c = wave + k * nw;
        if (c < kChunks) {
            const uint32_t e = (c << 3) + (lane >> 3);
            const uint32_t t = (e & 1u) | (((e >> 9) & 1u) << 1);
            const uint32_t x = t ? __builtin_amdgcn_alignbit(v[k], v[k], 32 - 8 * t) : v[k];
            *reinterpret_cast<uint4 *>(lds + c * 1024 + lane * 16) = make_uint4(x, x, x, x);
        }
    }
}

// nthr: the block's threads 0..nthr-1 share the copy (0: all of them)
__device__ __forceinline__ void fill_keys(const DevKeyTable *tab, uint32_t nthr = 0)
{
    const uint32_t n = nthr ? nthr : blockDim.x;
    const uint4 *src = reinterpret_cast<const uint4 *>(tab->rows);
    for (uint32_t e = threadIdx.x; e < kDevKeyRows * HFV_MAX_KEYS; e += n) s_keys[e] = src[e];
    if (threadIdx.x < 8) s_valid[threadIdx.x] = tab->valid[threadIdx.x];
}

// ---------------------------------------------------------------------------------------
// AES rounds on a column-word state (s[c] = LE u32 of column c)
// ---------------------------------------------------------------------------------------
struct Lane {
    uint32_t b0, b1, b2, b3;   // LDS byte offsets of this lane's copies of T0..T3
    uint32_t s0, s1, s2, s3;   // v_perm selectors SEL_B0..SEL_B3, held in VGPRs
    uint32_t f01, f23;         // final-round byte-gather selectors
};

template <int TAB, int K>
__device__ __forceinline__ uint32_t tlu(uint32_t w, uint32_t base, const Lane &l)
{
    static_assert(K >= 0 && K < 4, "state byte");
    if constexpr (TAB == 3) {
        const uint32_t a3 = (__builtin_amdgcn_ubfe(w, 8 * K, 8) << (kTab3Log + 2)) | base;
        return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_tab32) + a3);
    }
    const uint32_t a = __builtin_amdgcn_perm(w, base, K == 0 ? l.s0 : K == 1 ? l.s1 : K == 2 ? l.s2 : l.s3);
    const char *t = TAB == 4 ? reinterpret_cast<const char *>(s_tab128) : reinterpret_cast<const char *>(s_tab64);
    return *reinterpret_cast<const uint32_t *>(t + a);
}

// Materialise a constant in a VGPR.  v_perm_b32 (VOP3 on gfx9) takes no literal, so its
// selectors would otherwise occupy SGPRs; the SGPR-resident round keys already bring the
// kernel close to the 80-SGPR line above which a SIMD holds fewer than 8 waves.
__device__ __forceinline__ uint32_t vconst(uint32_t c)
{
    uint32_t r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "i"(c));
    return r;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // v_bitop3_b32 (gfx950)
}

// One full round.  TAB = 2 expects the round key pre-rotated by 16 (device key image rows
// 1..9) and folds it into the rotated half: 2 x xor3 + 1 rotate per column; TAB = 4 expects
// the plain round key: 2 x xor3 per column.
template <int TAB, bool PIN = false>
__device__ __forceinline__ void round_full(uint32_t s[4], const uint4 &rk, const Lane &l)
{
    const uint32_t r[4] = {rk.x, rk.y, rk.z, rk.w};
    uint32_t n[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t a = tlu<TAB, 0>(s[c], l.b0, l);
        uint32_t b = tlu<TAB, 1>(s[(c + 1) & 3], l.b1, l);
        if constexpr (TAB == 4) {
            uint32_t x = tlu<TAB, 2>(s[(c + 2) & 3], l.b2, l);
            uint32_t d = tlu<TAB, 3>(s[(c + 3) & 3], l.b3, l);
            n[c] = xor3(xor3(a, b, x), d, r[c]);
        } else {
            uint32_t x = tlu<TAB, 2>(s[(c + 2) & 3], l.b0, l);
            uint32_t d = tlu<TAB, 3>(s[(c + 3) & 3], l.b1, l);
            n[c] = xor3(a, b, rot16(xor3(x, d, r[c])));
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] = n[c];
    if constexpr (TAB == 4 && PIN) {
        // the round's issue order pinned: its 16 v_perm addresses, its 16 reads, its 8 xor3.
        // Taken by the one-launch-per-batch kernel only: 17.2 against 17.8-19.1 us per 2^20
        // batch there, neutral to slightly slower in the service (profiles/r05/s7/ab_sched_vk.log)
        __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);   // VALU
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);   // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);    // VALU
    }
}

// Round 1 for a whitened macinput whose bytes 0,1,8,14,15 are key-only: the five lookups
// they feed are folded into rk1' (device key row 11, see hfv_tables.h).
template <int TAB>
__device__ __forceinline__ void round1_macinput(uint32_t s[4], const uint4 &rk1p, const Lane &l)
{
    uint32_t n0, n1, n2, n3;
    if constexpr (TAB == 4) {
        n0 = xor3(tlu<TAB, 1>(s[1], l.b1, l), tlu<TAB, 2>(s[2], l.b2, l), rk1p.x);
        n1 = xor3(xor3(tlu<TAB, 0>(s[1], l.b0, l), tlu<TAB, 1>(s[2], l.b1, l), tlu<TAB, 3>(s[0], l.b3, l)), rk1p.y, 0u);
        n2 = xor3(xor3(tlu<TAB, 1>(s[3], l.b1, l), tlu<TAB, 2>(s[0], l.b2, l), tlu<TAB, 3>(s[1], l.b3, l)), rk1p.z, 0u);
        n3 = xor3(xor3(tlu<TAB, 0>(s[3], l.b0, l), tlu<TAB, 2>(s[1], l.b2, l), tlu<TAB, 3>(s[2], l.b3, l)), rk1p.w, 0u);
    } else {
        n0 = xor3(tlu<TAB, 1>(s[1], l.b1, l), rot16(tlu<TAB, 2>(s[2], l.b0, l)), rk1p.x);
        n1 = xor3(tlu<TAB, 0>(s[1], l.b0, l), tlu<TAB, 1>(s[2], l.b1, l), rk1p.y) ^ rot16(tlu<TAB, 3>(s[0], l.b1, l));
        n2 = xor3(tlu<TAB, 1>(s[3], l.b1, l), rot16(tlu<TAB, 2>(s[0], l.b0, l) ^ tlu<TAB, 3>(s[1], l.b1, l)), rk1p.z);
        n3 = xor3(tlu<TAB, 0>(s[3], l.b0, l), rot16(tlu<TAB, 2>(s[1], l.b0, l) ^ tlu<TAB, 3>(s[2], l.b1, l)), rk1p.w);
    }
    s[0] = n0; s[1] = n1; s[2] = n2; s[3] = n3;
}

// Final round, S(x) taken from byte 1 of T0[x].  All four output columns:
template <int TAB>
__device__ __forceinline__ void round_last_full(uint32_t s[4], const uint4 &rk, const Lane &l, uint32_t out[4])
{
    const uint32_t r[4] = {rk.x, rk.y, rk.z, rk.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t a = tlu<TAB, 0>(s[c], l.b0, l);
        uint32_t b = tlu<TAB, 1>(s[(c + 1) & 3], l.b0, l);
        uint32_t x = tlu<TAB, 2>(s[(c + 2) & 3], l.b0, l);
        uint32_t d = tlu<TAB, 3>(s[(c + 3) & 3], l.b0, l);
        out[c] = xor3(__builtin_amdgcn_perm(b, a, l.f01), __builtin_amdgcn_perm(d, x, l.f23), r[c]);
    }
}

// Final round, only the 48 bits the verifier compares (tag bytes 0..5, xdp.c:89):
// column 0 whole, column 1 bytes 0-1 (upper half of the result is don't-care).
template <int TAB>
__device__ __forceinline__ void round_last_48(const uint32_t s[4], const uint4 &rk, const Lane &l, uint32_t &t0,
                                              uint32_t &t1)
{
    uint32_t a = tlu<TAB, 0>(s[0], l.b0, l), b = tlu<TAB, 1>(s[1], l.b0, l);
    uint32_t x = tlu<TAB, 2>(s[2], l.b0, l), d = tlu<TAB, 3>(s[3], l.b0, l);
    t0 = xor3(__builtin_amdgcn_perm(b, a, l.f01), __builtin_amdgcn_perm(d, x, l.f23), rk.x);
    uint32_t a1 = tlu<TAB, 0>(s[1], l.b0, l), b1 = tlu<TAB, 1>(s[2], l.b0, l);
    t1 = __builtin_amdgcn_perm(b1, a1, l.f01) ^ rk.y;
}

// ---------------------------------------------------------------------------------------
// key sources
// ---------------------------------------------------------------------------------------
// Key sources.  row(r) is the device key image row as stored (hfv_tables.h); rk<TAB>(r) is
// the form round_full<TAB> takes for rounds 1..9 (image rows are pre-rotated for TAB = 2).
struct UniformKey {          // slot 0 for every lane, kept in SGPRs
    uint4 k[kDevKeyRows];
    bool ok;
    __device__ __forceinline__ explicit UniformKey(const DevKeyTable *tab)
    {
#pragma unroll
        for (int r = 0; r < kDevKeyRows; ++r) {
            const uint32_t *p = tab->rows[r][0];
            k[r] = make_uint4(p[0], p[1], p[2], p[3]);
        }
        ok = tab->valid[0] & 1u;
    }
    // the rows from the kernel arguments (constant address space: scalar loads); P is the
    // kernarg pointer type (address space 4, or generic into a by-value kernel argument, which
    // the compiler keeps in the kernarg segment)
    template <class P>
    __device__ __forceinline__ UniformKey(P rows, uint32_t valid)
    {
#pragma unroll
        for (int r = 0; r < kDevKeyRows; ++r) k[r] = make_uint4(rows[4 * r], rows[4 * r + 1], rows[4 * r + 2], rows[4 * r + 3]);
        ok = valid & 1u;
    }
    __device__ __forceinline__ uint4 row(int r) const { return k[r]; }
    template <int TAB>
    __device__ __forceinline__ uint4 rk(int r) const
    {
        if constexpr (TAB == 2 || TAB == 3) {
            return k[r];
        } else {   // undo the image's rotation; uniform operands, so these stay scalar
            auto u = [](uint32_t x) { return (x >> 16) | (x << 16); };
            return make_uint4(u(k[r].x), u(k[r].y), u(k[r].z), u(k[r].w));
        }
    }
};

struct LdsKey {              // per-lane slot from the LDS copy of the table
    uint32_t slot;
    __device__ __forceinline__ explicit LdsKey(uint32_t s) : slot(s) {}
    __device__ __forceinline__ uint4 row(int r) const { return s_keys[r * HFV_MAX_KEYS + slot]; }
    template <int TAB>
    __device__ __forceinline__ uint4 rk(int r) const
    {
        static_assert(TAB == 2, "per-lane keys use the 64 KiB two-table layout");
        return row(r);
    }
    __device__ __forceinline__ bool ok() const { return (s_valid[slot >> 5] >> (slot & 31)) & 1u; }
};

// ---------------------------------------------------------------------------------------
// Per-interface keys (config 3, KEYSEL_IFID): five 16-byte rows per slot in LDS beside all
// four round tables -- row 0 (rk0 ^ K1), row 11 (round 1 folded), rk2, and the key-schedule
// words t_r = SubWord(RotWord(w_{4r-1})) ^ Rcon_r of rounds 3..6 and 7..10 (DevKeyTable::sched,
// aes.c:120-137) -- 20 KiB for 256 slots.  Round key r then follows from round key r - 1 by
// XOR alone (w_{4r} = w_{4r-4} ^ t_r, w_{4r+j} = w_{4r+j-4} ^ w_{4r+j-1}): per packet five
// random-slot ds_read_b128 (each ~3 LDS cycles per 16-lane group: 16 lanes over 16 quad-banks)
// and no S-box lookup for the schedule.  Round 4 expanded rounds 3..10 per packet from rk2 with
// four conflict-free T-table reads per step (32 lookups and 16 v_perm per packet, three rows):
// 186.8 LDS instructions per 64-packet tile against 150.7 for one key.
constexpr int kSchedRows = 5;
static __shared__ uint4 s_keys5[kSchedRows * HFV_MAX_KEYS];

__device__ __forceinline__ void fill_keys5(const DevKeyTable *tab, uint32_t nthr)
{
    // image rows 0 and 11 as stored; rk2 (image row 2, stored rotated by 16) unrotated; the
    // two schedule rows as stored
    for (uint32_t e = threadIdx.x; e < kSchedRows * HFV_MAX_KEYS; e += nthr) {
        const uint32_t j = e / HFV_MAX_KEYS, k = e % HFV_MAX_KEYS;
        const uint32_t *p = j < 3 ? tab->rows[j == 0 ? 0 : j == 1 ? 11 : 2][k] : tab->sched[j - 3][k];
        uint4 v = make_uint4(p[0], p[1], p[2], p[3]);
        if (j == 2) v = make_uint4(rot16(v.x), rot16(v.y), rot16(v.z), rot16(v.w));
        s_keys5[e] = v;
    }
    if (threadIdx.x < 8) s_valid[threadIdx.x] = tab->valid[threadIdx.x];
}

// One AES-128 key-schedule step from its precomputed word t = SubWord(RotWord(w3)) ^ Rcon.
__device__ __forceinline__ uint4 next_round_key(const uint4 &rk, uint32_t t)
{
    uint4 n;
    n.x = rk.x ^ t;
    n.y = rk.y ^ n.x;
    n.z = rk.z ^ n.y;
    n.w = rk.w ^ n.z;
    return n;
}

__device__ __forceinline__ bool slot_valid(uint32_t slot) { return (s_valid[slot >> 5] >> (slot & 31)) & 1u; }

// Tag words 0..1 of a record-derived macinput for the slot's key (s_keys5).
__device__ __forceinline__ void cmac48_sched(const uint32_t w[4], uint32_t slot, const Lane &l, uint32_t &t0,
                                             uint32_t &t1)
{
    const uint4 k0 = s_keys5[slot];
    const uint4 r1 = s_keys5[HFV_MAX_KEYS + slot];
    uint4 rk = s_keys5[2 * HFV_MAX_KEYS + slot];   // rk2
    const uint4 ta = s_keys5[3 * HFV_MAX_KEYS + slot], tb = s_keys5[4 * HFV_MAX_KEYS + slot];
    const uint32_t t[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    uint32_t s[4] = {w[0] ^ k0.x, w[1] ^ k0.y, w[2] ^ k0.z, w[3] ^ k0.w};
    round1_macinput<4>(s, r1, l);
    round_full<4>(s, rk, l);
#pragma unroll
    for (int r = 3; r < 10; ++r) {
        rk = next_round_key(rk, t[r - 3]);
        round_full<4>(s, rk, l);
    }
    rk = next_round_key(rk, t[7]);                 // rk10
    round_last_48<4>(s, rk, l, t0, t1);
}

// Tag words 0..1 for a record-derived macinput w[] (bytes 0,1,8,14,15 zero).
template <int TAB, class K, bool PIN = false>
__device__ __forceinline__ void cmac48_macinput(const uint32_t w[4], const K &key, const Lane &l, uint32_t &t0,
                                                uint32_t &t1)
{
    uint4 k0 = key.row(0);
    uint32_t s[4] = {w[0] ^ k0.x, w[1] ^ k0.y, w[2] ^ k0.z, w[3] ^ k0.w};
    round1_macinput<TAB>(s, key.row(11), l);
#pragma unroll
    for (int r = 2; r < 10; ++r) round_full<TAB, PIN>(s, key.template rk<TAB>(r), l);
    round_last_48<TAB>(s, key.row(10), l, t0, t1);
}

template <int TAB, class K>
__device__ __forceinline__ void cmac_general(const uint32_t w[4], const K &key, const Lane &l, uint32_t s[4])
{
    uint4 k0 = key.row(0);
    s[0] = w[0] ^ k0.x; s[1] = w[1] ^ k0.y; s[2] = w[2] ^ k0.z; s[3] = w[3] ^ k0.w;
#pragma unroll
    for (int r = 1; r < 10; ++r) round_full<TAB>(s, key.template rk<TAB>(r), l);
}

__device__ __forceinline__ Lane lane_bases()
{
    uint32_t lane = threadIdx.x & 63;
    Lane l;
    l.s0 = vconst(SEL_B0); l.s1 = vconst(SEL_B1); l.s2 = vconst(SEL_B2); l.s3 = vconst(SEL_B3);
    l.f01 = vconst(0x0c0c0501u); l.f23 = vconst(0x05010c0cu);
    l.b0 = (lane & 31) << 2;
    l.b1 = l.b0 | 0x80u;
    l.b2 = l.b0 | 0x10000u;
    l.b3 = l.b1 | 0x10000u;
    return l;
}

// Lane bases for the TAB = 3 layout (b0: T0, b1: T1; b2/b3 unused: T2/T3 are rotations).
__device__ __forceinline__ Lane lane_bases3()
{
    Lane l = lane_bases();
    l.b0 = (threadIdx.x & (kTab3Copies - 1)) << 2;
    l.b1 = l.b0 | (1u << (kTab3Log + 10));
    l.b2 = l.b0;
    l.b3 = l.b1;
    return l;
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
}  // namespace hfv
