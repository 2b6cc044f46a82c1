/*
 * hfv_aes.h -- the reference's host AES / AES-CMAC API, re-exported by libscionhfv.so.
 *
 * Drop-in for aes/include/aes/aes.h:47-119 (non-BPF half): same function names, argument
 * meaning, struct layouts (16 B blocks in FIPS-197 column-major order with a little-endian
 * u32 view; 176 B key schedule = key + 10 round keys) and error behaviour (no error
 * returns; aes_cypher always returns 0).  The BR control plane links these unchanged
 * (br/src/br_loader.cpp:215-217 key install, br/src/maps.cpp:86 AES_SBox).
 *
 * These are control-plane helpers.  The per-packet data path (the BPF-only
 * aes_cmac_16bytes, aes.h:129-141, called from verify_hop_field, xdp.c:77-91) is served by
 * the MI355X kernels behind scion_hfv.h, never by these host functions.
 */
#ifndef HFV_AES_H
#define HFV_AES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AES_KEY_LENGTH 4
#define AES_BLOCK_SIZE 4
#define AES_ROUNDS 10
#define AES_SCHED_SIZE ((AES_ROUNDS + 1) * AES_BLOCK_SIZE)
#define AES_CMAC_NO_LOOP_MAX_BYTES (4 * (4 * AES_BLOCK_SIZE))

struct aes_block { union { uint8_t b[16]; uint32_t w[4]; }; };            /* aes.h:48-54 */
struct aes_key { union { uint8_t b[16]; uint32_t w[4]; }; };              /* aes.h:57-63 */
struct aes_key_schedule {                                                  /* aes.h:66-73 */
    union { uint8_t b[176]; uint32_t w[44]; struct aes_key k[11]; };
};
struct aes_cmac { union { uint8_t b[16]; uint32_t w[4]; }; };             /* aes.h:76-82 */

/* FIPS-197 S-box, replaces aes.c:69-86 (exported for maps.cpp:83-88-style consumers) */
extern const uint8_t AES_SBox[256];

/* aes.c:120-137 */
void aes_key_expansion(const struct aes_key *key, struct aes_key_schedule *key_schedule);
/* aes.c:249-293; returns 0 */
int aes_cypher(const struct aes_block *input, const struct aes_key_schedule *key_schedule,
               struct aes_block *output);
/* aes.c:313-325: subkeys[0] = K1, subkeys[1] = K2 */
void aes_cmac_subkeys(const struct aes_key_schedule *key_schedule, struct aes_block subkeys[2]);
/* aes.c:333-368, RFC 4493 */
void aes_cmac(const uint8_t *data, size_t len, const struct aes_key_schedule *key_schedule,
              const struct aes_block subkeys[2], struct aes_cmac *mac);
/* aes.c:377-434, including its >64 B behaviour (at most 4 blocks are processed) */
void aes_cmac_no_loops(const uint8_t *data, size_t len, const struct aes_key_schedule *key_schedule,
                       const struct aes_block subkeys[2], struct aes_cmac *mac);

#ifdef __cplusplus
}
#endif
#endif
