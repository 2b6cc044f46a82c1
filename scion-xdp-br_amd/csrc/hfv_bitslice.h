// hfv_bitslice.h -- bitsliced AES-128 for the hop-field verify kernel: VALU-only AES that
// runs beside the LDS T-table waves (hfv_aes_dev.h) so that the verify kernel uses both the
// vector ALUs and the LDS, instead of leaving the ALUs half idle behind 145 LDS lookups per
// packet.
//
// Layout ("quad" bitslicing).  A quad of 4 lanes holds the AES states of 32 packets; lane c
// of the quad holds state column c: 32 bit planes s[8*r + b] = bit b of state byte (row r,
// column c) of the 32 packets (packet p in bit p).  Per round each lane then computes
//   * AddRoundKey + ShiftRows together: rows 1..3 come from lane (c + r) % 4 of the quad
//     (a DPP quad_perm on the XOR's first operand), each plane XORed with an all-0/all-1
//     mask made from the lane's pre-shifted round-key column (v_bfe_i32);
//   * SubBytes: 4 S-box circuits (hfv_bitslice_sbox.h, 84 v_bitop3 nodes each);
//   * MixColumns: column-local, 76 XOR/XOR3 on 32 planes.
// ShiftRows is applied before SubBytes (they commute), so a round is ARK+SR, SB, MC.
// The per-lane code is plain __host__ __device__ C++ except for the quad exchange, so the
// CPU self-test (csrc/bs_selftest.cpp) runs the same round code for 4 emulated lanes.
#pragma once
#include <stdint.h>

#if defined(__HIP_DEVICE_COMPILE__)
#define HFV_BS_FN __device__ __forceinline__
#define HFV_BOP3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
#else
#define HFV_BS_FN static inline
#define HFV_BOP3(a, b, c, tt) ::hfv::bs::bop3_host((a), (b), (c), (tt))
#endif

namespace hfv {
namespace bs {
// v_bitop3_b32 semantics: result bit = tt bit ((a << 2) | (b << 1) | c)
static inline uint32_t bop3_host(uint32_t a, uint32_t b, uint32_t c, uint32_t tt)
{
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i)
        if ((tt >> i) & 1) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
}
}  // namespace bs
}  // namespace hfv

#include "hfv_bitslice_sbox.h"

namespace hfv {
namespace bs {

// MixColumns on one column's planes a[8*r + b] (rows r = 0..3), in place:
//   out_r = 2 a_r ^ 3 a_{r+1} ^ a_{r+2} ^ a_{r+3} = a_{r+1} ^ u_{r+2} ^ xtime(u_r),
//   u_r = a_r ^ a_{r+1};  xtime(u)[0] = u[7], [1] = u[0]^u[7], [2] = u[1], [3] = u[2]^u[7],
//   [4] = u[3]^u[7], [5..7] = u[4..6]  (reduction polynomial 0x11b).
HFV_BS_FN void mix_columns(uint32_t (&a)[32])
{
    uint32_t u[32], o[32];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int b = 0; b < 8; ++b) u[8 * r + b] = a[8 * r + b] ^ a[8 * ((r + 1) & 3) + b];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t *ur = u + 8 * r, *u2 = u + 8 * ((r + 2) & 3), *a1 = a + 8 * ((r + 1) & 3);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint32_t x = HFV_BOP3(a1[b], u2[b], b ? ur[b - 1] : ur[7], 0x96);
            if (b == 1 || b == 3 || b == 4) x ^= ur[7];
            o[8 * r + b] = x;
        }
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = o[i];
}

HFV_BS_FN void sub_bytes(uint32_t (&s)[32])
{
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint32_t x[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) x[b] = s[8 * r + b];
        sbox(x);
#pragma unroll
        for (int b = 0; b < 8; ++b) s[8 * r + b] = x[b];
    }
}

// byte permute: result byte i = byte sel_i of the 8-byte value {hi:lo} (v_perm_b32 order)
HFV_BS_FN uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xff) << (8 * i);
    return r;
#endif
}

// 32 x 32 bit transpose in place: afterwards bit p of x[i] = bit i of the old x[p].
// Stages 16 and 8 move whole bytes (one v_perm_b32 per output word); stages 4, 2, 1 are
// shift + bit-field-insert pairs.
HFV_BS_FN void transpose32(uint32_t (&x)[32])
{
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        uint32_t a = x[k], b = x[k + 16];
        x[k] = perm(b, a, 0x05040100u);
        x[k + 16] = perm(b, a, 0x07060302u);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        if (k & 8) continue;
        uint32_t a = x[k], b = x[k + 8];
        x[k] = perm(b, a, 0x06020400u);
        x[k + 8] = perm(b, a, 0x07030501u);
    }
    constexpr uint32_t m4 = 0x0f0f0f0fu, m2 = 0x33333333u, m1 = 0x55555555u;
#pragma unroll
    for (int st = 0; st < 3; ++st) {
        const int j = 4 >> st;
        const uint32_t m = j == 4 ? m4 : j == 2 ? m2 : m1;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (k & j) continue;
            uint32_t a = x[k], b = x[k + j];
            x[k] = (a & m) | ((b << j) & ~m);
            x[k + j] = ((a >> j) & m) | (b & ~m);
        }
    }
}

// all-ones / all-zeros plane for key bit `bit` of the lane's key column word
HFV_BS_FN uint32_t kmask(uint32_t kk, int bit)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_amdgcn_sbfe((int)kk, bit, 1);
#else
    return 0u - ((kk >> bit) & 1u);
#endif
}

// The lane's key column for the ARK+SR step: row r of the pre-shifted key, i.e. byte r of
// round-key column (c + r) % 4.  rk[] = the four LE column words of the round key.
// (Selects, not an indexed register array: c differs per lane.)
HFV_BS_FN uint32_t shifted_key_column(const uint32_t rk[4], uint32_t c)
{
    uint32_t k = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t i = (c + r) & 3u;
        const uint32_t w = i == 0 ? rk[0] : i == 1 ? rk[1] : i == 2 ? rk[2] : rk[3];
        k |= w & (0xffu << (8 * r));
    }
    return k;
}

}  // namespace bs
}  // namespace hfv
