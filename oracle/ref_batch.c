/*
 * ref_batch.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Batch driver around the REFERENCE's own AES library: this file is compiled together
 * with /root/reference/aes/src/aes.c and aes_hw_accel.c (unmodified, read in place) by
 * oracle/Makefile into oracle/_ref/libaesref.so.  It lets the tests and the bench's
 * cpu_baseline leg run the reference arithmetic over the same 64 B records the GPU path
 * verifies:
 *   - soft path  = aes_cmac()               (aes/src/aes.c:333-368), the arithmetic XDP runs
 *   - AES-NI path = aes_cmac_unaligned128() (aes/src/aes_hw_accel.c:187-223)
 * The per-record logic (macinput + beta + 48-bit compare) restates
 * br/src/bpf/path_processing.h:39-81 and br/src/bpf/xdp.c:77-91 (BPF-only in the reference).
 */
#include "aes/aes.h"
#include "aes/aes_hw_accel.h"

#include <pthread.h>
#include <stdalign.h>
#include <string.h>

/* hop_key = { aes_key_schedule key; aes_block subkey; } (br/src/bpf/common.h:87-91) */
void ref_hop_key(const uint8_t key_bytes[16], uint8_t out[192])
{
    struct aes_key key;
    memcpy(key.b, key_bytes, 16);
    struct aes_key_schedule sched;
    aes_key_expansion(&key, &sched);
    struct aes_block subkeys[2];
    aes_cmac_subkeys(&sched, subkeys);        /* br_loader.cpp:215-218 keeps K1 */
    memcpy(out, sched.b, 176);
    memcpy(out + 176, subkeys[0].b, 16);
}

static uint64_t build_macinput(const uint8_t *rec, uint8_t mi[16])
{
    const uint8_t *inf = rec + 40, *hf = rec + 48;
    uint16_t beta = (uint16_t)(inf[2] << 8 | inf[3]);
    if (!(inf[0] & 1)) beta ^= (uint16_t)(hf[6] << 8 | hf[7]);
    memset(mi, 0, 16);
    mi[2] = (uint8_t)(beta >> 8); mi[3] = (uint8_t)beta;
    memcpy(mi + 4, inf + 4, 4);
    mi[9] = hf[1];
    memcpy(mi + 10, hf + 2, 4);
    uint64_t e = 0;
    for (int i = 0; i < 6; ++i) e |= (uint64_t)hf[6 + i] << (8 * i);
    return e;
}

static uint32_t key_index(const uint8_t *rec, int keysel)
{
    if (keysel != 1) return 0;
    const uint8_t *inf = rec + 40, *hf = rec + 48;
    uint16_t ifid = (inf[0] & 1) ? (uint16_t)(hf[2] << 8 | hf[3]) : (uint16_t)(hf[4] << 8 | hf[5]);
    return ifid & 0xff;
}

typedef struct {
    const uint8_t *recs; size_t stride, n0, n1;
    const uint8_t *keys192; const uint32_t *valid; int keysel; int aesni;
    const __m128i *ni_sched; const __m128i *ni_sub;   /* [256][11], [256][2] */
    uint64_t *bits;
} job_t;

static void run_range(job_t *j)
{
    for (size_t w = j->n0 / 64; 64 * w < j->n1; ++w) {
        uint64_t bits = 0;
        for (size_t b = 0; b < 64 && 64 * w + b < j->n1; ++b) {
            const uint8_t *rec = j->recs + (64 * w + b) * j->stride;
            uint32_t idx = key_index(rec, j->keysel);
            if (!((j->valid[idx >> 5] >> (idx & 31)) & 1)) continue;   /* xdp.c:84 */
            uint8_t mi[16];
            uint64_t expected = build_macinput(rec, mi);
            struct aes_cmac mac;
            if (j->aesni) {
                aes_cmac_unaligned128(mi, 16, j->ni_sched + 11 * idx, j->ni_sub + 2 * idx, &mac);
            } else {
                const uint8_t *hk = j->keys192 + 192 * (size_t)idx;
                struct aes_block sub[2];
                memcpy(sub[0].b, hk + 176, 16);
                memset(sub[1].b, 0, 16);             /* K2 unused for a 16-byte message */
                aes_cmac(mi, 16, (const struct aes_key_schedule *)hk, sub, &mac);
            }
            uint64_t actual = 0;
            memcpy(&actual, mac.b, 8);
            if ((actual & 0xffffffffffffull) == expected) bits |= 1ull << b;
        }
        j->bits[w] = bits;
    }
}

static void *worker(void *p) { run_range((job_t *)p); return NULL; }

/* keys192: nkeys x 192 B hop_key images (ref_hop_key output); raw_keys: nkeys x 16 B (AES-NI
 * schedule is derived from the raw key with aes_key_expansion_128). */
int ref_verify_records(const uint8_t *recs, size_t stride, size_t n, const uint8_t *keys192,
                       const uint8_t *raw_keys, uint32_t nkeys, const uint32_t valid[8], int keysel,
                       uint64_t *pass_bits, int nthreads, int aesni)
{
    static alignas(16) __m128i ni_sched[256 * 11];
    static alignas(16) __m128i ni_sub[256 * 2];
    if (nkeys > 256) return -1;
    if (aesni) {
        for (uint32_t k = 0; k < nkeys; ++k) {
            __m128i kr = _mm_loadu_si128((const __m128i_u *)(raw_keys + 16 * k));
            aes_key_expansion_128(kr, ni_sched + 11 * k);
            aes_cmac_subkeys_128(ni_sched + 11 * k, ni_sub + 2 * k);
        }
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    size_t words = (n + 63) / 64;
    for (int t = 0; t < nthreads; ++t) {
        size_t w0 = words * (size_t)t / (size_t)nthreads, w1 = words * (size_t)(t + 1) / (size_t)nthreads;
        jobs[t] = (job_t){recs, stride, 64 * w0, 64 * w1 < n ? 64 * w1 : n, keys192, valid, keysel, aesni,
                          ni_sched, ni_sub, pass_bits};
        if (nthreads == 1) run_range(&jobs[t]);
        else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}
