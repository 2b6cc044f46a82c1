// hfv_aes_host.cpp -- host side of the control plane: the reference's aes.h API
// (aes/src/aes.c, re-exported by libscionhfv.so for br_loader-style callers), the base64
// key decoder of br-loader, the scalar verify_hop_field, and the host compiler of the
// device key image.  Word-oriented T-table implementation built on hfv_tables.h.
#include <errno.h>
#include <string.h>

#include "hfv_internal.h"

extern "C" const uint8_t AES_SBox[256] = {
#define S(i) hfv::kTables.sbox[i]
#define S8(i) S(i), S(i + 1), S(i + 2), S(i + 3), S(i + 4), S(i + 5), S(i + 6), S(i + 7)
#define S64(i) S8(i), S8(i + 8), S8(i + 16), S8(i + 24), S8(i + 32), S8(i + 40), S8(i + 48), S8(i + 56)
    S64(0), S64(64), S64(128), S64(192)
#undef S64
#undef S8
#undef S
};

namespace hfv {

static inline uint32_t ld_le(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }   // x86-64: LE
static inline void st_le(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline uint32_t sub_word(uint32_t w)
{
    return uint32_t(kTables.sbox[w & 0xff]) | uint32_t(kTables.sbox[(w >> 8) & 0xff]) << 8 |
           uint32_t(kTables.sbox[(w >> 16) & 0xff]) << 16 | uint32_t(kTables.sbox[w >> 24]) << 24;
}

void expand_key(const uint8_t key[16], uint32_t w[44])
{
    for (int i = 0; i < 4; ++i) w[i] = ld_le(key + 4 * i);
    uint32_t rcon = 1;
    for (int i = 4; i < 44; i += 4) {
        uint32_t t = sub_word(rotl32(w[i - 1], 24)) ^ rcon;   // RotWord moves byte 1 to byte 0
        rcon = xtime(uint8_t(rcon));
        w[i] = w[i - 4] ^ t;
        w[i + 1] = w[i - 3] ^ w[i];
        w[i + 2] = w[i - 2] ^ w[i + 1];
        w[i + 3] = w[i - 1] ^ w[i + 2];
    }
}

void encrypt_block(const uint32_t rk[44], const uint32_t in[4], uint32_t out[4])
{
    uint32_t s[4], n[4];
    for (int c = 0; c < 4; ++c) s[c] = in[c] ^ rk[c];
    for (int r = 1; r < 10; ++r) {
        for (int c = 0; c < 4; ++c)
            n[c] = kTables.t0[s[c] & 0xff] ^ rotl32(kTables.t0[(s[(c + 1) & 3] >> 8) & 0xff], 8) ^
                   rotl32(kTables.t0[(s[(c + 2) & 3] >> 16) & 0xff], 16) ^
                   rotl32(kTables.t0[s[(c + 3) & 3] >> 24], 24) ^ rk[4 * r + c];
        memcpy(s, n, sizeof s);
    }
    for (int c = 0; c < 4; ++c)
        out[c] = (uint32_t(kTables.sbox[s[c] & 0xff]) | uint32_t(kTables.sbox[(s[(c + 1) & 3] >> 8) & 0xff]) << 8 |
                  uint32_t(kTables.sbox[(s[(c + 2) & 3] >> 16) & 0xff]) << 16 |
                  uint32_t(kTables.sbox[s[(c + 3) & 3] >> 24]) << 24) ^
                 rk[40 + c];
}

// RFC 4493 doubling in GF(2^128), big-endian bit order over the 16 bytes
static void cmac_double(uint8_t b[16])
{
    uint8_t carry = 0;
    for (int i = 15; i >= 0; --i) {
        uint8_t nb = uint8_t(b[i] >> 7);
        b[i] = uint8_t((b[i] << 1) | carry);
        carry = nb;
    }
    if (carry) b[15] ^= 0x87;
}

void hop_key_from_key(const uint8_t key[16], hop_key *hk)
{
    uint32_t w[44];
    expand_key(key, w);
    for (int i = 0; i < 44; ++i) hk->key.w[i] = w[i];
    uint32_t zero[4] = {0, 0, 0, 0}, l[4];
    encrypt_block(w, zero, l);
    uint8_t k1[16];
    for (int c = 0; c < 4; ++c) st_le(k1 + 4 * c, l[c]);
    cmac_double(k1);
    memcpy(hk->subkey.b, k1, 16);
}

void compile_dev_key(const hop_key *hk, uint32_t dk[4 * kDevKeyRows])
{
    const uint32_t *rk = hk->key.w;
    for (int c = 0; c < 4; ++c) dk[c] = rk[c] ^ hk->subkey.w[c];
    for (int i = 4; i < 44; ++i) dk[i] = rk[i];
    // Round-1 terms fed only by the zero macinput bytes 0,1 (col 0), 8 (col 2), 14,15 (col 3):
    // after whitening those state bytes equal the k0x bytes themselves.
    const uint32_t *k = dk;
    auto T = [](int row, uint32_t x) { return rotl32(kTables.t0[x & 0xff], 8 * row); };
    dk[44] = rk[4] ^ T(0, k[0]) ^ T(3, k[3] >> 24);          // col 0: row0 <- byte 0, row3 <- byte 15
    dk[45] = rk[5] ^ T(2, k[3] >> 16);                          // col 1: row2 <- byte 14
    dk[46] = rk[6] ^ T(0, k[2]);                                // col 2: row0 <- byte 8
    dk[47] = rk[7] ^ T(1, k[0] >> 8);                           // col 3: row1 <- byte 1
    for (int i = 4; i < 40; ++i) dk[i] = rotl32(dk[i], 16);    // rows 1..9 pre-rotated (hfv_tables.h)
}

// Key-schedule words of rounds 3..10 (DevKeyTable::sched): t_r = SubWord(RotWord(w[4r-1])) ^
// Rcon[r] = w[4r] ^ w[4r-4] (aes.c:120-137).
void compile_dev_sched(const hop_key *hk, uint32_t t[8])
{
    const uint32_t *w = hk->key.w;
    for (int r = 3; r <= 10; ++r) t[r - 3] = w[4 * r] ^ w[4 * r - 4];
}

}  // namespace hfv

// ---------------------------------------------------------------------------------------
// aes.h surface (aes/include/aes/aes.h:85-119)
// ---------------------------------------------------------------------------------------
extern "C" {

void aes_key_expansion(const struct aes_key *key, struct aes_key_schedule *key_schedule)
{
    hfv::expand_key(key->b, key_schedule->w);
}

int aes_cypher(const struct aes_block *input, const struct aes_key_schedule *key_schedule,
               struct aes_block *output)
{
    uint32_t in[4], out[4];
    memcpy(in, input->w, 16);
    hfv::encrypt_block(key_schedule->w, in, out);
    memcpy(output->w, out, 16);
    return 0;
}

void aes_cmac_subkeys(const struct aes_key_schedule *key_schedule, struct aes_block subkeys[2])
{
    struct aes_block zero;
    memset(&zero, 0, sizeof zero);
    aes_cypher(&zero, key_schedule, &subkeys[0]);
    hfv::cmac_double(subkeys[0].b);
    subkeys[1] = subkeys[0];
    hfv::cmac_double(subkeys[1].b);
}

// One CBC-MAC chain over `nfull` whole blocks, then a final block holding `tail` bytes
// (0..16) at data + 16*nfull, padded with 10* and whitened with K2 when tail < 16.
static void cmac_chain(const uint8_t *data, size_t nfull, size_t tail, const struct aes_key_schedule *ks,
                       const struct aes_block subkeys[2], struct aes_cmac *mac)
{
    struct aes_block x;
    memset(&x, 0, sizeof x);
    for (size_t b = 0; b < nfull; ++b) {
        for (int i = 0; i < 16; ++i) x.b[i] ^= data[16 * b + i];
        aes_cypher(&x, ks, &x);
    }
    const uint8_t *last = data + 16 * nfull;
    for (size_t i = 0; i < tail; ++i) x.b[i] ^= last[i];
    const struct aes_block *sk = &subkeys[0];
    if (tail < 16) {
        x.b[tail] ^= 0x80;
        sk = &subkeys[1];
    }
    for (int i = 0; i < 16; ++i) x.b[i] ^= sk->b[i];
    aes_cypher(&x, ks, &x);
    memcpy(mac->b, x.b, 16);
}

void aes_cmac(const uint8_t *data, size_t len, const struct aes_key_schedule *key_schedule,
              const struct aes_block subkeys[2], struct aes_cmac *mac)
{
    // RFC 4493: the last block is the final (possibly partial, possibly empty) block
    size_t nblocks = len == 0 ? 1 : (len + 15) / 16;
    cmac_chain(data, nblocks - 1, len - 16 * (nblocks - 1), key_schedule, subkeys, mac);
}

void aes_cmac_no_loops(const uint8_t *data, size_t len, const struct aes_key_schedule *key_schedule,
                       const struct aes_block subkeys[2], struct aes_cmac *mac)
{
    // Reference behaviour (aes.c:384-431): at most three whole blocks precede the final
    // block, whose size is still taken from len % 16, so inputs over 64 B are truncated.
    size_t nblocks = len == 0 ? 1 : (len + 15) / 16;
    size_t tail = len == 0 ? 0 : (len % 16 ? len % 16 : 16);
    size_t nfull = nblocks > 4 ? 3 : nblocks - 1;
    cmac_chain(data, nfull, tail, key_schedule, subkeys, mac);
}

int hfv_verify_macinput(const struct macinput *mi, uint64_t expected, const struct hop_key *key)
{
    if (!mi || !key) return 0;                         // xdp.c:79,84
    struct aes_block x;
    memcpy(x.b, mi, 16);
    for (int i = 0; i < 16; ++i) x.b[i] ^= key->subkey.b[i];
    aes_cypher(&x, &key->key, &x);
    uint64_t actual;
    memcpy(&actual, x.b, 8);
    return (actual & 0xffffffffffffull) == expected;   // xdp.c:89-90
}

int hfv_decode_key_b64(const char *base64, struct aes_key *key)
{
    // br_loader.cpp:65-73: exactly 24 characters; the trailing "==" carries no key bits
    if (!base64 || !key) return hfv::fail(-EINVAL, "null argument");
    if (strlen(base64) != 24) return hfv::fail(-EINVAL, "Key has invalid length");
    uint32_t acc = 0;
    int nbits = 0;
    size_t out = 0;
    uint8_t buf[16];
    for (int i = 0; i < 22; ++i) {
        char ch = base64[i];
        int v;
        if (ch >= 'A' && ch <= 'Z') v = ch - 'A';
        else if (ch >= 'a' && ch <= 'z') v = ch - 'a' + 26;
        else if (ch >= '0' && ch <= '9') v = ch - '0' + 52;
        else if (ch == '+') v = 62;
        else if (ch == '/') v = 63;
        else return hfv::fail(-EINVAL, "invalid base64 character");
        acc = (acc << 6) | uint32_t(v);
        nbits += 6;
        if (nbits >= 8 && out < 16) {
            nbits -= 8;
            buf[out++] = uint8_t(acc >> nbits);
        }
    }
    memcpy(key->b, buf, 16);
    return 0;
}

}  // extern "C"
