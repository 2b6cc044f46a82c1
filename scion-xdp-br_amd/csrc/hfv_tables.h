// hfv_tables.h -- compile-time AES tables shared by the host control-plane code and the
// gfx950 kernels.  Nothing here is transcribed: the S-box is generated from its FIPS-197
// definition (inverse in GF(2^8) via log/antilog tables of the generator 3, then the
// affine map), and the round table T0 from the S-box and the MixColumns matrix.
//
// Word convention (aes/include/aes/aes.h:48-82): a column of the AES state is the
// little-endian u32 of its four bytes, row r in byte r.  T0[x] is the MixColumns image of
// S(x) entering in row 0: bytes (2S, S, S, 3S).  Row r's table is T0 rotated left by 8r.
#pragma once
#include <stdint.h>

namespace hfv {

constexpr uint8_t xtime(uint8_t x) { return uint8_t((x << 1) ^ ((x & 0x80) ? 0x1b : 0x00)); }

struct Tables {
    uint8_t sbox[256];
    uint32_t t0[256];
};

constexpr Tables make_tables()
{
    Tables t{};
    uint8_t exp3[256] = {};
    uint8_t log3[256] = {};
    uint8_t p = 1;
    for (int i = 0; i < 255; ++i) {      // 3 generates GF(2^8)*: exp3[i] = 3^i
        exp3[i] = p;
        log3[p] = uint8_t(i);
        p = uint8_t(p ^ xtime(p));
    }
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = x ? exp3[(255 - log3[x]) % 255] : 0;
        uint8_t s = inv;
        uint8_t r = inv;
        for (int k = 0; k < 4; ++k) {        // s = inv ^ rotl1 ^ rotl2 ^ rotl3 ^ rotl4
            r = uint8_t((r << 1) | (r >> 7));
            s ^= r;
        }
        t.sbox[x] = uint8_t(s ^ 0x63);
    }
    for (int x = 0; x < 256; ++x) {
        uint8_t s = t.sbox[x], s2 = xtime(s), s3 = uint8_t(s2 ^ s);
        t.t0[x] = uint32_t(s2) | uint32_t(s) << 8 | uint32_t(s) << 16 | uint32_t(s3) << 24;
    }
    return t;
}

constexpr Tables kTables = make_tables();

static_assert(kTables.sbox[0x00] == 0x63 && kTables.sbox[0x01] == 0x7c && kTables.sbox[0x53] == 0xed &&
                  kTables.sbox[0xff] == 0x16,
              "S-box generation (FIPS-197 Figure 7 spot values)");

constexpr uint32_t rotl32(uint32_t x, int s) { return s & 31 ? (x << (s & 31)) | (x >> (32 - (s & 31))) : x; }

// Device key image consumed by the kernels (192 B = 12 x 16 B), compiled from a hop_key:
//   row 0      k0x   = rk0 ^ K1          (CMAC whitening folded into round 0)
//   rows 1..9  rot16(rk1) .. rot16(rk9)  (the two-table round adds its key inside the
//                      16-bit-rotated half: n = T0 ^ T1 ^ rot16(T0' ^ T1' ^ rot16(rk)),
//                      two 3-input XORs and one rotate per column)
//   row 10     rk10  (final round)
//   row 11     rk1'  = rk1 ^ the five round-1 table terms whose inputs are the constant-zero
//                      macinput bytes 0,1,8,14,15 (scion.h:122-132), i.e. key-only values.
// Row 11 is only valid for inputs with those bytes zero (records built by the verifier).
constexpr int kDevKeyRows = 12;

}  // namespace hfv
