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
#include <stdlib.h>

#include "hfv_internal.h"

namespace hfv {

// ---------------------------------------------------------------------------------------
// tables
// ---------------------------------------------------------------------------------------
#define T0V(i) kTables.t0[i]
#define T0V8(i) T0V(i), T0V(i + 1), T0V(i + 2), T0V(i + 3), T0V(i + 4), T0V(i + 5), T0V(i + 6), T0V(i + 7)
#define T0V64(i) T0V8(i), T0V8(i + 8), T0V8(i + 16), T0V8(i + 24), T0V8(i + 32), T0V8(i + 40), T0V8(i + 48), T0V8(i + 56)
__constant__ uint32_t c_t0[256] = {T0V64(0), T0V64(64), T0V64(128), T0V64(192)};
#undef T0V64
#undef T0V8
#undef T0V

constexpr int kTabDwords = 256 * 64;            // 64 KiB
__shared__ uint32_t s_ttab[kTabDwords];
__shared__ uint4 s_keys[kDevKeyRows * HFV_MAX_KEYS];   // 48 KiB, round-major
__shared__ uint32_t s_valid[8];

// v_perm selectors: address byte 1 <- state byte k, byte 0 <- base byte 0
constexpr uint32_t SEL_B0 = 0x0c0c0400u, SEL_B1 = 0x0c0c0500u, SEL_B2 = 0x0c0c0600u, SEL_B3 = 0x0c0c0700u;

__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }

__device__ __forceinline__ uint32_t tlu(uint32_t w, uint32_t base, uint32_t sel)
{
    uint32_t a = __builtin_amdgcn_perm(w, base, sel);
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_ttab) + a);
}

__device__ __forceinline__ void fill_ttab()
{
    for (int e = threadIdx.x; e < kTabDwords; e += blockDim.x) {
        uint32_t t = c_t0[e >> 6];
        s_ttab[e] = (e & 32) ? ((t << 8) | (t >> 24)) : t;
    }
}

__device__ __forceinline__ void fill_keys(const DevKeyTable *tab)
{
    const uint4 *src = reinterpret_cast<const uint4 *>(tab->rows);
    for (int e = threadIdx.x; e < kDevKeyRows * HFV_MAX_KEYS; e += blockDim.x) s_keys[e] = src[e];
    if (threadIdx.x < 8) s_valid[threadIdx.x] = tab->valid[threadIdx.x];
}

// ---------------------------------------------------------------------------------------
// AES rounds on a column-word state (s[c] = LE u32 of column c)
// ---------------------------------------------------------------------------------------
struct Lane {
    uint32_t b0, b1;   // LDS byte offsets of this lane's T0 / T1 copies
};

__device__ __forceinline__ void round_full(uint32_t s[4], const uint4 &rk, const Lane &l)
{
    const uint32_t r[4] = {rk.x, rk.y, rk.z, rk.w};
    uint32_t n[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t a = tlu(s[c], l.b0, SEL_B0);
        uint32_t b = tlu(s[(c + 1) & 3], l.b1, SEL_B1);
        uint32_t x = tlu(s[(c + 2) & 3], l.b0, SEL_B2);
        uint32_t d = tlu(s[(c + 3) & 3], l.b1, SEL_B3);
        n[c] = a ^ b ^ r[c] ^ rot16(x ^ d);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) s[c] = n[c];
}

// Round 1 for a whitened macinput whose bytes 0,1,8,14,15 are key-only: the five lookups
// they feed are folded into rk1' (device key row 11, see hfv_tables.h).
__device__ __forceinline__ void round1_macinput(uint32_t s[4], const uint4 &rk1p, const Lane &l)
{
    uint32_t n0 = tlu(s[1], l.b1, SEL_B1) ^ rot16(tlu(s[2], l.b0, SEL_B2)) ^ rk1p.x;
    uint32_t n1 = tlu(s[1], l.b0, SEL_B0) ^ tlu(s[2], l.b1, SEL_B1) ^ rot16(tlu(s[0], l.b1, SEL_B3)) ^ rk1p.y;
    uint32_t n2 = tlu(s[3], l.b1, SEL_B1) ^ rot16(tlu(s[0], l.b0, SEL_B2) ^ tlu(s[1], l.b1, SEL_B3)) ^ rk1p.z;
    uint32_t n3 = tlu(s[3], l.b0, SEL_B0) ^ rot16(tlu(s[1], l.b0, SEL_B2) ^ tlu(s[2], l.b1, SEL_B3)) ^ rk1p.w;
    s[0] = n0; s[1] = n1; s[2] = n2; s[3] = n3;
}

// Final round, S(x) taken from byte 1 of T0[x].  All four output columns:
__device__ __forceinline__ void round_last_full(uint32_t s[4], const uint4 &rk, const Lane &l, uint32_t out[4])
{
    const uint32_t r[4] = {rk.x, rk.y, rk.z, rk.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t a = tlu(s[c], l.b0, SEL_B0);
        uint32_t b = tlu(s[(c + 1) & 3], l.b0, SEL_B1);
        uint32_t x = tlu(s[(c + 2) & 3], l.b0, SEL_B2);
        uint32_t d = tlu(s[(c + 3) & 3], l.b0, SEL_B3);
        out[c] = __builtin_amdgcn_perm(b, a, 0x0c0c0501u) ^ __builtin_amdgcn_perm(d, x, 0x05010c0cu) ^ r[c];
    }
}

// Final round, only the 48 bits the verifier compares (tag bytes 0..5, xdp.c:89):
// column 0 whole, column 1 bytes 0-1 (upper half of the result is don't-care).
__device__ __forceinline__ void round_last_48(const uint32_t s[4], const uint4 &rk, const Lane &l, uint32_t &t0,
                                              uint32_t &t1)
{
    uint32_t a = tlu(s[0], l.b0, SEL_B0), b = tlu(s[1], l.b0, SEL_B1);
    uint32_t x = tlu(s[2], l.b0, SEL_B2), d = tlu(s[3], l.b0, SEL_B3);
    t0 = __builtin_amdgcn_perm(b, a, 0x0c0c0501u) ^ __builtin_amdgcn_perm(d, x, 0x05010c0cu) ^ rk.x;
    uint32_t a1 = tlu(s[1], l.b0, SEL_B0), b1 = tlu(s[2], l.b0, SEL_B1);
    t1 = __builtin_amdgcn_perm(b1, a1, 0x0c0c0501u) ^ rk.y;
}

// ---------------------------------------------------------------------------------------
// key sources
// ---------------------------------------------------------------------------------------
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
    __device__ __forceinline__ uint4 row(int r) const { return k[r]; }
};

struct LdsKey {              // per-lane slot from the LDS copy of the table
    uint32_t slot;
    __device__ __forceinline__ explicit LdsKey(uint32_t s) : slot(s) {}
    __device__ __forceinline__ uint4 row(int r) const { return s_keys[r * HFV_MAX_KEYS + slot]; }
    __device__ __forceinline__ bool ok() const { return (s_valid[slot >> 5] >> (slot & 31)) & 1u; }
};

// Tag words 0..1 for a record-derived macinput w[] (bytes 0,1,8,14,15 zero).
template <class K>
__device__ __forceinline__ void cmac48_macinput(const uint32_t w[4], const K &key, const Lane &l, uint32_t &t0,
                                                uint32_t &t1)
{
    uint4 k0 = key.row(0);
    uint32_t s[4] = {w[0] ^ k0.x, w[1] ^ k0.y, w[2] ^ k0.z, w[3] ^ k0.w};
    round1_macinput(s, key.row(11), l);
#pragma unroll
    for (int r = 2; r < 10; ++r) round_full(s, key.row(r), l);
    round_last_48(s, key.row(10), l, t0, t1);
}

template <class K>
__device__ __forceinline__ void cmac_general(const uint32_t w[4], const K &key, const Lane &l, uint32_t s[4])
{
    uint4 k0 = key.row(0);
    s[0] = w[0] ^ k0.x; s[1] = w[1] ^ k0.y; s[2] = w[2] ^ k0.z; s[3] = w[3] ^ k0.w;
#pragma unroll
    for (int r = 1; r < 10; ++r) round_full(s, key.row(r), l);
}

__device__ __forceinline__ Lane lane_bases()
{
    uint32_t lane = threadIdx.x & 63;
    Lane l;
    l.b0 = (lane & 31) << 2;
    l.b1 = l.b0 | 0x80u;
    return l;
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// ---------------------------------------------------------------------------------------
// record verify: macinput from INF/HF (path_processing.h:39-81), CMAC, 48-bit compare
// ---------------------------------------------------------------------------------------
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct RecWords {
    uint2 inf;    // INF bytes 0-7: flags rsv segid[2] | ts[4]
    uint2 hfa;    // HF bytes 0-7: flags exp ing[2] | eg[2] mac0 mac1
    uint32_t hfb; // HF bytes 8-11: mac2..mac5
};

// Unconditional loads (no branch around them, so the compiler can keep a counted vmcnt for
// the prefetch): lanes past the end re-read the last record and are masked off later.
__device__ __forceinline__ RecWords load_rec(const uint8_t *recs, uint64_t stride, uint64_t i, uint64_t last,
                                             uint32_t inf_off, uint32_t hf_off)
{
    RecWords r;
    const uint8_t *p = recs + (i < last ? i : last) * stride;
    u32x2 a = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(p + inf_off));
    u32x2 b = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(p + hf_off));
    r.inf = make_uint2(a.x, a.y);
    r.hfa = make_uint2(b.x, b.y);
    r.hfb = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p + hf_off + 8));
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

template <int KEYSEL, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_verify_records(const DevKeyTable *__restrict__ tab,
                                                          const uint8_t *__restrict__ recs, uint64_t stride,
                                                          uint64_t n, uint32_t inf_off, uint32_t hf_off,
                                                          uint64_t *__restrict__ bits)
{
    constexpr uint32_t kWaves = BLOCK / 64;
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform(blockIdx.x * kWaves + threadIdx.x / 64);
    const uint32_t nwaves = gridDim.x * kWaves;

    fill_ttab();
    if constexpr (KEYSEL == HFV_KEYSEL_IFID) fill_keys(tab);
    __syncthreads();
    const Lane l = lane_bases();

    if constexpr (KEYSEL == HFV_KEYSEL_ZERO) {
        const UniformKey key(tab);
        if (!key.ok) {   // no key in slot 0: every packet fails closed (xdp.c:83-84)
            for (uint64_t t = wave; t < ntiles; t += nwaves)
                if (lane == 0) bits[t] = 0;
            return;
        }
        uint64_t t = wave;
        RecWords cur = load_rec(recs, stride, t * 64 + lane, n - 1, inf_off, hf_off);
        for (; t < ntiles; t += nwaves) {
            RecWords nxt = load_rec(recs, stride, (t + nwaves) * 64 + lane, n - 1, inf_off, hf_off);
            uint32_t w[4], t0, t1;
            rec_macinput(cur, w);
            cmac48_macinput(w, key, l, t0, t1);
            bool pass = rec_tag_matches(cur, t0, t1) && (t * 64 + lane < n);
            uint64_t ballot = __ballot(pass);
            if (lane == 0) bits[t] = ballot;
            cur = nxt;
        }
    } else {
        uint64_t t = wave;
        RecWords cur = load_rec(recs, stride, t * 64 + lane, n - 1, inf_off, hf_off);
        for (; t < ntiles; t += nwaves) {
            RecWords nxt = load_rec(recs, stride, (t + nwaves) * 64 + lane, n - 1, inf_off, hf_off);
            const LdsKey key(rec_key_slot(cur));
            uint32_t w[4], t0, t1;
            rec_macinput(cur, w);
            cmac48_macinput(w, key, l, t0, t1);
            bool pass = rec_tag_matches(cur, t0, t1) && key.ok() && (t * 64 + lane < n);
            uint64_t ballot = __ballot(pass);
            if (lane == 0) bits[t] = ballot;
            cur = nxt;
        }
    }
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
    fill_ttab();
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
        cmac_general(w, key, l, s);
        if constexpr (MODE == kModeTags) {
            uint32_t o[4];
            round_last_full(s, key.row(10), l, o);
            if (!key.ok()) o[0] = o[1] = o[2] = o[3] = 0;
            if (in) tags[i] = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            uint32_t t0, t1;
            round_last_48(s, key.row(10), l, t0, t1);
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
        for (int r = 1; r < 11; ++r) {
            uint32_t *p = tab->rows[r][slot];
            p[0] = w[4 * r]; p[1] = w[4 * r + 1]; p[2] = w[4 * r + 2]; p[3] = w[4 * r + 3];
        }
        uint32_t *p = tab->rows[11][slot];
        p[0] = w[4] ^ tg(0, k0[0]) ^ tg(3, k0[3] >> 24);
        p[1] = w[5] ^ tg(2, k0[3] >> 16);
        p[2] = w[6] ^ tg(0, k0[2]);
        p[3] = w[7] ^ tg(1, k0[0] >> 8);
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
    fill_ttab();
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
        cmac_general(w, key, l, s);
        round_last_full(s, key.row(10), l, tg4);
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
constexpr int kBlockRec = 1024;
constexpr int kBlockAux = 512;

static inline unsigned grid_for(uint64_t n, int block, int num_cus, int per_cu)
{
    uint64_t tiles = (n + 63) / 64;
    uint64_t blocks = (tiles + block / 64 - 1) / (block / 64);
    uint64_t cap = (uint64_t)num_cus * (uint64_t)(per_cu > 0 ? per_cu : 1);
    if (blocks > cap) blocks = cap;
    return (unsigned)(blocks ? blocks : 1);
}

int launch_verify_records(const LaunchGeom &g, const DevKeyTable *tab, int keysel, const uint8_t *recs,
                          size_t stride, size_t n, uint32_t inf_off, uint32_t hf_off, uint64_t *bits, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    if (keysel == HFV_KEYSEL_IFID) {
        unsigned grid = grid_for(n, kBlockRec, g.num_cus, g.blocks_per_cu_multi);
        hipLaunchKernelGGL((k_verify_records<HFV_KEYSEL_IFID, kBlockRec>), dim3(grid), dim3(kBlockRec), 0, st, tab,
                           recs, (uint64_t)stride, (uint64_t)n, inf_off, hf_off, bits);
    } else {
        unsigned grid = grid_for(n, kBlockRec, g.num_cus, g.blocks_per_cu_single);
        hipLaunchKernelGGL((k_verify_records<HFV_KEYSEL_ZERO, kBlockRec>), dim3(grid), dim3(kBlockRec), 0, st, tab,
                           recs, (uint64_t)stride, (uint64_t)n, inf_off, hf_off, bits);
    }
    return (int)hipGetLastError();
}

int launch_verify_macinputs(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint64_t *expected,
                            const uint8_t *kidx, size_t n, uint64_t *bits, void *stream)
{
    unsigned grid = grid_for(n, kBlockAux, g.num_cus, 2 * g.blocks_per_cu_multi);
    hipLaunchKernelGGL((k_macinputs<kModeMacinputs, kBlockAux>), dim3(grid), dim3(kBlockAux), 0, (hipStream_t)stream,
                       tab, (const uint4 *)mi, (const uint2 *)expected, kidx, (uint64_t)n, bits, (uint4 *)nullptr);
    return (int)hipGetLastError();
}

int launch_cmac_tags(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint8_t *kidx, size_t n,
                     void *tags, void *stream)
{
    unsigned grid = grid_for(n, kBlockAux, g.num_cus, 2 * g.blocks_per_cu_multi);
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

// Persistent-grid size: blocks per CU for the record-verify kernels.  One 16-wave block per
// CU pays the 64 KiB table fill once per CU; HFV_BLOCKS_PER_CU overrides it (capped by the
// occupancy query, which on ROCm 7.2 can over-report for SGPR-heavy kernels).
int query_geometry(int device, LaunchGeom *g)
{
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return (int)e;
    g->num_cus = prop.multiProcessorCount;
    int want = 1;
    if (const char *env = getenv("HFV_BLOCKS_PER_CU")) want = atoi(env) > 0 ? atoi(env) : 1;
    int b = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_verify_records<HFV_KEYSEL_ZERO, kBlockRec>, kBlockRec, 0);
    if (e != hipSuccess) return (int)e;
    g->blocks_per_cu_single = b > 0 ? (want < b ? want : b) : 1;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_verify_records<HFV_KEYSEL_IFID, kBlockRec>, kBlockRec, 0);
    if (e != hipSuccess) return (int)e;
    g->blocks_per_cu_multi = b > 0 ? (want < b ? want : b) : 1;
    return 0;
}

}  // namespace hfv
