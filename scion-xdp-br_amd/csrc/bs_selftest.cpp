// bs_selftest.cpp -- CPU check of the bitsliced AES formulation used by the verify kernel
// (hfv_bitslice.h): the same per-lane round code, run for the 4 lanes of a quad emulated on
// the host (the DPP quad exchange becomes an array read), against the library's T-table
// AES (hfv::encrypt_block) on random blocks and keys.  Also checks the device key image
// handling (row 0 = rk0 ^ K1, rows 1..9 rotated by 16) by computing full CMAC tags
// (aes.h:129-141) through compile_dev_key.
//
//   bs_selftest [iterations]   -> prints "ok <n> blocks" or the first mismatch, exit 0/1
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hfv_bitslice.h"
#include "hfv_internal.h"

using namespace hfv;

static uint64_t g_state = 0x5C1000BEEFull;
static uint32_t rnd32()
{
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}

// Quad of 4 emulated lanes; lane c holds column c of 32 packets.
struct Quad {
    uint32_t s[4][32];
};

// ARK + ShiftRows: lane c row r <- lane (c + r) % 4 row r, XOR the lane's key column mask.
static void ark_sr(Quad &q, const uint32_t kk[4])
{
    Quad o;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            for (int b = 0; b < 8; ++b)
                o.s[c][8 * r + b] = q.s[(c + r) & 3][8 * r + b] ^ bs::kmask(kk[c], 8 * r + b);
    q = o;
}

static uint32_t rot16(uint32_t x) { return (x >> 16) | (x << 16); }

int main(int argc, char **argv)
{
    int iters = argc > 1 ? atoi(argv[1]) : 64;
    long checked = 0;
    for (int it = 0; it < iters; ++it) {
        uint8_t key[16];
        for (int i = 0; i < 16; i += 4) {
            uint32_t r = rnd32();
            memcpy(key + i, &r, 4);
        }
        hop_key hk;
        hop_key_from_key(key, &hk);
        uint32_t dk[4 * kDevKeyRows];
        compile_dev_key(&hk, dk);
        // round keys as the kernel forms them: row 0 = rk0 ^ K1; rows 1..9 un-rotated; row 10
        uint32_t rk[11][4];
        for (int r = 0; r < 11; ++r)
            for (int c = 0; c < 4; ++c) rk[r][c] = (r >= 1 && r <= 9) ? rot16(dk[4 * r + c]) : dk[4 * r + c];

        uint32_t blk[32][4];
        for (int p = 0; p < 32; ++p)
            for (int c = 0; c < 4; ++c) blk[p][c] = rnd32();

        Quad q;
        for (int c = 0; c < 4; ++c) {
            uint32_t x[32];
            for (int p = 0; p < 32; ++p) x[p] = blk[p][c];
            bs::transpose32(x);
            memcpy(q.s[c], x, sizeof x);
        }
        for (int r = 0; r < 10; ++r) {
            uint32_t kk[4];
            for (int c = 0; c < 4; ++c) kk[c] = bs::shifted_key_column(rk[r], (uint32_t)c);
            ark_sr(q, kk);
            for (int c = 0; c < 4; ++c) {
                bs::sub_bytes(q.s[c]);
                if (r < 9) bs::mix_columns(q.s[c]);
            }
        }
        for (int c = 0; c < 4; ++c) {
            for (int i = 0; i < 32; ++i) q.s[c][i] ^= bs::kmask(rk[10][c], i);
            bs::transpose32(q.s[c]);   // planes -> per-packet words (the transpose is an involution)
        }
        for (int p = 0; p < 32; ++p) {
            // reference: CMAC of one full block = AES_K(m ^ K1) (aes.h:129-141)
            uint32_t in[4], out[4];
            for (int c = 0; c < 4; ++c) in[c] = blk[p][c] ^ hk.subkey.w[c];
            encrypt_block(hk.key.w, in, out);
            for (int c = 0; c < 4; ++c) {
                if (q.s[c][p] != out[c]) {
                    printf("mismatch iter %d packet %d column %d: bitsliced %08x, reference %08x\n", it, p, c,
                           q.s[c][p], out[c]);
                    return 1;
                }
            }
            ++checked;
        }
    }
    printf("ok %ld blocks\n", checked);
    return 0;
}
