/*
 * hfv_oracle.c -- TEST INFRASTRUCTURE ONLY (see hfv_oracle.h).
 *
 * A plain, byte-at-a-time restatement of the reference AES-128 / AES-CMAC
 * (aes/src/aes.c) and of the BR hop-field verify step (br/src/bpf/xdp.c:77-91,
 * br/src/bpf/path_processing.h:39-81).  It is deliberately written for clarity,
 * not speed: it is the checker the HIP kernels are compared against.
 *
 * The S-box is not transcribed from the reference table (aes.c:69-86); it is derived
 * here from its FIPS-197 definition (multiplicative inverse in GF(2^8) followed by the
 * affine map) and the KAT vectors in tests/golden/kat.json pin the result.
 */
#include "hfv_oracle.h"

#include <pthread.h>
#include <string.h>

/* ---------------------------------------------------------------------------------- */
/* GF(2^8) and the S-box (FIPS-197 5.1.1; reference table at aes.c:69-86)             */
/* ---------------------------------------------------------------------------------- */

static uint8_t g_sbox[256];
static int g_sbox_ready = 0;

/* aes.c:208-211 */
static uint8_t xtime(uint8_t p) { return (uint8_t)((p << 1) ^ ((p & 0x80) ? 0x1b : 0x00)); }

static uint8_t gf_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

static uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }

static void sbox_init(void)
{
    if (g_sbox_ready) return;
    for (int x = 0; x < 256; ++x) {
        /* inverse = x^254 (0 maps to 0) */
        uint8_t inv = 0;
        if (x) {
            uint8_t acc = 1, base = (uint8_t)x;
            int e = 254;
            while (e) {
                if (e & 1) acc = gf_mul(acc, base);
                base = gf_mul(base, base);
                e >>= 1;
            }
            inv = acc;
        }
        g_sbox[x] = (uint8_t)(inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63);
    }
    g_sbox_ready = 1;
}

const uint8_t *orc_sbox(void)
{
    sbox_init();
    return g_sbox;
}

/* ---------------------------------------------------------------------------------- */
/* Key expansion (aes.c:98-137): 44 little-endian words, Rcon in the low byte          */
/* ---------------------------------------------------------------------------------- */

static uint32_t ld32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
static void st32(uint8_t *p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }

void orc_key_expansion(const uint8_t key[16], uint8_t sched[176])
{
    sbox_init();
    uint32_t w[44];
    for (int i = 0; i < 4; ++i) w[i] = ld32(key + 4 * i);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; ++i) {
        uint32_t t = w[i - 1];
        if ((i & 3) == 0) {
            t = (t >> 8) | (t << 24);                         /* rot_word, aes.c:109-115 */
            t = (uint32_t)g_sbox[t & 0xff] | (uint32_t)g_sbox[(t >> 8) & 0xff] << 8 |
                (uint32_t)g_sbox[(t >> 16) & 0xff] << 16 | (uint32_t)g_sbox[t >> 24] << 24; /* sub_word */
            t ^= rcon;                                         /* AES_Rcon[i/4], aes.c:88-90 */
            rcon = xtime(rcon);
        }
        w[i] = w[i - 4] ^ t;
    }
    for (int i = 0; i < 44; ++i) st32(sched + 4 * i, w[i]);
}

/* ---------------------------------------------------------------------------------- */
/* Cipher (aes.c:141-293): state b[row + 4*col]                                        */
/* ---------------------------------------------------------------------------------- */

static void add_round_key(uint8_t s[16], const uint8_t *rk)
{
    for (int i = 0; i < 16; ++i) s[i] ^= rk[i];
}

static void sub_shift(uint8_t s[16])
{
    uint8_t t[16];
    /* ShiftRows: new[r][c] = old[r][(c + r) mod 4] (aes.c:174-205) after SubBytes */
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            t[r + 4 * c] = g_sbox[s[r + 4 * ((c + r) & 3)]];
    memcpy(s, t, 16);
}

static void mix_columns(uint8_t s[16])
{
    for (int c = 0; c < 4; ++c) {
        uint8_t *col = s + 4 * c;
        uint8_t a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
        col[0] = (uint8_t)(gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3);
        col[1] = (uint8_t)(a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3);
        col[2] = (uint8_t)(a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3));
        col[3] = (uint8_t)(gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2));
    }
}

void orc_cypher(const uint8_t in[16], const uint8_t sched[176], uint8_t out[16])
{
    sbox_init();
    uint8_t s[16];
    memcpy(s, in, 16);
    add_round_key(s, sched);
    for (int round = 1; round < 10; ++round) {
        sub_shift(s);
        mix_columns(s);
        add_round_key(s, sched + 16 * round);
    }
    sub_shift(s);
    add_round_key(s, sched + 160);
    memcpy(out, s, 16);
}

/* ---------------------------------------------------------------------------------- */
/* CMAC (RFC 4493; aes.c:298-434)                                                      */
/* ---------------------------------------------------------------------------------- */

static void dbl(uint8_t b[16])   /* generate_subkey_helper, aes.c:298-308 */
{
    uint8_t msb = b[0] >> 7;
    for (int i = 0; i < 15; ++i) b[i] = (uint8_t)((b[i] << 1) | (b[i + 1] >> 7));
    b[15] = (uint8_t)(b[15] << 1);
    if (msb) b[15] ^= 0x87;
}

void orc_cmac_subkeys(const uint8_t sched[176], uint8_t k1[16], uint8_t k2[16])
{
    uint8_t z[16] = {0};
    orc_cypher(z, sched, k1);
    dbl(k1);
    memcpy(k2, k1, 16);
    dbl(k2);
}

void orc_cmac(const uint8_t *data, size_t len, const uint8_t sched[176],
              const uint8_t k1[16], const uint8_t k2[16], uint8_t mac[16])
{
    uint8_t x[16] = {0};
    size_t nblk = len ? (len + 15) / 16 : 1;
    for (size_t b = 0; b < nblk; ++b) {
        size_t off = 16 * b;
        size_t take = len - off < 16 ? len - off : 16;
        if (len == 0) take = 0;
        for (size_t i = 0; i < take; ++i) x[i] ^= data[off + i];
        if (b + 1 == nblk) {
            const uint8_t *sk = k1;
            if (take < 16) { x[take] ^= 0x80; sk = k2; }
            for (int i = 0; i < 16; ++i) x[i] ^= sk[i];
        }
        orc_cypher(x, sched, x);
    }
    memcpy(mac, x, 16);
}

/* aes_cmac_no_loops keeps the reference's structure on purpose: for more than four
 * blocks the switch's default label falls into "case 4", so only the first three full
 * blocks plus a final block sized from len % 16 are processed (aes.c:394-431). */
void orc_cmac_no_loops(const uint8_t *data, size_t len, const uint8_t sched[176],
                       const uint8_t k1[16], const uint8_t k2[16], uint8_t mac[16])
{
    size_t blocks = 1, last = 0;
    if (len > 0) {
        blocks = (len + 15) / 16;
        last = len % 16;
        if (last == 0) last = 16;
    }
    size_t full = blocks >= 4 ? 3 : blocks - 1;
    uint8_t x[16] = {0};
    size_t off = 0;
    for (size_t b = 0; b < full; ++b) {
        for (int i = 0; i < 16; ++i) x[i] ^= data[off + i];
        orc_cypher(x, sched, x);
        off += 16;
    }
    for (size_t i = 0; i < last; ++i) x[i] ^= data[off + i];
    const uint8_t *sk = k1;
    if (last < 16) { x[last] ^= 0x80; sk = k2; }
    for (int i = 0; i < 16; ++i) x[i] ^= sk[i];
    orc_cypher(x, sched, x);
    memcpy(mac, x, 16);
}

/* ---------------------------------------------------------------------------------- */
/* hop-field layer                                                                     */
/* ---------------------------------------------------------------------------------- */

void orc_hop_key_from_key(const uint8_t key[16], orc_hop_key *hk)
{
    uint8_t k2[16];
    orc_key_expansion(key, hk->sched);
    orc_cmac_subkeys(hk->sched, hk->k1, k2);
}

void orc_cmac16(const uint8_t mi[16], const orc_hop_key *key, uint8_t tag[16])
{
    /* aes_cmac_16bytes (aes.h:129-141): data ^ K1, then one cipher call */
    uint8_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = mi[i] ^ key->k1[i];
    orc_cypher(x, key->sched, tag);
}

uint64_t orc_macinput_beta(const uint8_t inf[8], const uint8_t hf[12], uint16_t beta, uint8_t mi[16])
{
    /* struct macinput (scion.h:122-132), filled as in path_processing.h:45-53 */
    memset(mi, 0, 16);
    mi[2] = (uint8_t)(beta >> 8);          /* htons(beta) */
    mi[3] = (uint8_t)beta;
    memcpy(mi + 4, inf + 4, 4);            /* ts, wire order */
    mi[9] = hf[1];                         /* exp */
    memcpy(mi + 10, hf + 2, 2);            /* ingress, wire order */
    memcpy(mi + 12, hf + 4, 2);            /* egress, wire order */
    uint64_t expected = 0;                 /* memcpy(&mac[which], hop->mac, 6) on LE */
    for (int i = 0; i < 6; ++i) expected |= (uint64_t)hf[6 + i] << (8 * i);
    return expected;
}

uint64_t orc_macinput_ingress(const uint8_t inf[8], const uint8_t hf[12], uint8_t mi[16])
{
    /* path_processing.h:73-77: beta = ntohs(SegID); if !Cons, beta ^= mac[0]<<8 | mac[1] */
    uint16_t beta = (uint16_t)(inf[2] << 8 | inf[3]);
    if (!(inf[0] & 0x01)) beta ^= (uint16_t)(hf[6] << 8 | hf[7]);
    return orc_macinput_beta(inf, hf, beta, mi);
}

int orc_verify_hop_field(const uint8_t mi[16], uint64_t expected, const orc_hop_key *key)
{
    if (!mi || !key) return 0;                       /* xdp.c:79,84: fail closed */
    uint8_t tag[16];
    orc_cmac16(mi, key, tag);
    uint64_t actual = 0;                             /* *(u64*)mac.w & 0xffffffffffff */
    for (int i = 0; i < 6; ++i) actual |= (uint64_t)tag[i] << (8 * i);
    return actual == expected;
}

uint32_t orc_record_key_index(const uint8_t *rec, int keysel)
{
    if (keysel != ORC_KEYSEL_IFID) return 0;
    const uint8_t *inf = rec + ORC_REC_INF_OFF, *hf = rec + ORC_REC_HF_OFF;
    uint16_t ifid = (inf[0] & 1) ? (uint16_t)(hf[2] << 8 | hf[3]) : (uint16_t)(hf[4] << 8 | hf[5]);
    return ifid & 0xff;
}

static int verify_one_record(const uint8_t *rec, const orc_hop_key *keys, const uint32_t valid[8], int keysel)
{
    uint32_t idx = orc_record_key_index(rec, keysel);
    const orc_hop_key *key = ((valid[idx >> 5] >> (idx & 31)) & 1) ? &keys[idx] : NULL;
    uint8_t mi[16];
    uint64_t expected = orc_macinput_ingress(rec + ORC_REC_INF_OFF, rec + ORC_REC_HF_OFF, mi);
    return orc_verify_hop_field(mi, expected, key);
}

void orc_verify_records(const uint8_t *recs, size_t stride, size_t n,
                        const orc_hop_key *keys, const uint32_t valid[8], int keysel,
                        uint64_t *pass_bits)
{
    size_t words = (n + 63) / 64;
    for (size_t w = 0; w < words; ++w) {
        uint64_t bits = 0;
        for (size_t j = 0; j < 64 && 64 * w + j < n; ++j)
            if (verify_one_record(recs + (64 * w + j) * stride, keys, valid, keysel)) bits |= 1ull << j;
        pass_bits[w] = bits;
    }
}

typedef struct {
    const uint8_t *recs; size_t stride, n0, n1;
    const orc_hop_key *keys; const uint32_t *valid; int keysel; uint64_t *bits;
} mt_job;

static void *mt_worker(void *p)
{
    mt_job *j = (mt_job *)p;
    if (j->n1 > j->n0)
        orc_verify_records(j->recs + j->n0 * j->stride, j->stride, j->n1 - j->n0, j->keys, j->valid,
                           j->keysel, j->bits + j->n0 / 64);
    return NULL;
}

void orc_verify_records_mt(const uint8_t *recs, size_t stride, size_t n,
                           const orc_hop_key *keys, const uint32_t valid[8], int keysel,
                           uint64_t *pass_bits, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    mt_job jobs[256];
    size_t words = (n + 63) / 64;
    for (int t = 0; t < nthreads; ++t) {
        size_t w0 = words * (size_t)t / (size_t)nthreads, w1 = words * (size_t)(t + 1) / (size_t)nthreads;
        size_t n0 = 64 * w0, n1 = 64 * w1 < n ? 64 * w1 : n;
        jobs[t] = (mt_job){recs, stride, n0, n1, keys, valid, keysel, pass_bits};
        pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* ---------------------------------------------------------------------------------- */
/* Synthetic records                       */
/* ---------------------------------------------------------------------------------- */

#define GOLDEN 0x9E3779B97F4A7C15ull

uint64_t orc_splitmix_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1) * GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_gen_key_table(uint64_t seed, uint32_t nkeys, uint8_t keys[][16])
{
    for (uint32_t k = 0; k < nkeys; ++k) {
        uint64_t a = orc_splitmix_at(seed, 2ull * k), b = orc_splitmix_at(seed, 2ull * k + 1);
        for (int i = 0; i < 8; ++i) { keys[k][i] = (uint8_t)(a >> (8 * i)); keys[k][8 + i] = (uint8_t)(b >> (8 * i)); }
    }
}

static void be16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void be32(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v; }

void orc_gen_records(uint8_t *recs, size_t stride, size_t n, uint64_t seed, uint64_t first_index,
                     const orc_hop_key *keys, int keysel)
{
    for (size_t j = 0; j < n; ++j) {
        uint64_t i = first_index + j;
        uint64_t r0 = orc_splitmix_at(seed, 4 * i), r1 = orc_splitmix_at(seed, 4 * i + 1);
        uint64_t r2 = orc_splitmix_at(seed, 4 * i + 2), r3 = orc_splitmix_at(seed, 4 * i + 3);
        uint8_t *p = recs + j * stride;
        memset(p, 0, 64);
        /* SCION common header (scion.h:26-50) */
        be32(p + 0, (uint32_t)(r3 & 0xfffff));  /* version 0, TC 0, flow id */
        p[4] = 17;                               /* NextHdr = UDP */
        p[5] = 15;                               /* HdrLen = 60 B / 4 */
        be16(p + 6, 4);                          /* payload length */
        p[8] = 1;                                /* PathType = SCION */
        p[9] = 0;                                /* DT/DL/ST/SL: IPv4 hosts */
        be16(p + 12, 1); p[14] = 0xff; p[19] = 0x10;  /* dst ISD-AS 1-ff00:0:110 */
        be16(p + 20, 1); p[22] = 0xff; p[27] = 0x11;  /* src ISD-AS 1-ff00:0:111 */
        be32(p + 28, 0x0a000001u); be32(p + 32, 0x0a000002u);
        be32(p + 36, 1u << 12);                  /* PathMeta: CurrINF 0, CurrHF 0, Seg0Len 1 */
        uint8_t *inf = p + ORC_REC_INF_OFF, *hf = p + ORC_REC_HF_OFF;
        int cons = (int)(r0 & 1);
        uint16_t beta = (uint16_t)(r0 >> 8);
        inf[0] = (uint8_t)cons;
        be32(inf + 4, (uint32_t)(r0 >> 32));     /* timestamp */
        hf[0] = 0;
        hf[1] = (uint8_t)r1;                     /* exp */
        be16(hf + 2, (uint16_t)(1 + ((r1 >> 8) & 0xffff) % 255));   /* ConsIngress in [1,255] */
        be16(hf + 4, (uint16_t)(1 + ((r1 >> 24) & 0xffff) % 255));  /* ConsEgress in [1,255] */
        /* MAC with beta_i, then the wire SegID: beta_i if Cons, else beta_i ^ MAC[0:2] */
        uint32_t kidx = 0;
        if (keysel == ORC_KEYSEL_IFID) {
            uint16_t ifid = cons ? (uint16_t)(hf[2] << 8 | hf[3]) : (uint16_t)(hf[4] << 8 | hf[5]);
            kidx = ifid & 0xff;
        }
        uint8_t mi[16], tag[16];
        orc_macinput_beta(inf, hf, beta, mi);
        orc_cmac16(mi, &keys[kidx], tag);
        memcpy(hf + 6, tag, 6);
        uint16_t seg = cons ? beta : (uint16_t)(beta ^ (uint16_t)(tag[0] << 8 | tag[1]));
        be16(inf + 2, seg);
        if ((r2 & 15) == 0) {                    /* ~1/16 corrupted: flip one MAC bit */
            unsigned bit = (unsigned)((r2 >> 4) % 48);
            hf[6 + bit / 8] ^= (uint8_t)(1u << (bit % 8));
        }
        be32(p + 60, (uint32_t)i);               /* payload */
    }
}
