/*
 * hfv_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's hop-field AES-CMAC verify path, used as the
 * parity checker for the MI355X kernels.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product library never links it.
 *
 * Parity pinning: the restatement is checked against
 *   (1) the known-answer vectors in the reference's aes/src/test/aes_test.cpp:33-245
 *       (transcribed as data into tests/golden/kat.json), and
 *   (2) the reference's own aes/src/aes.c compiled from /root/reference by
 *       oracle/Makefile into oracle/_ref/libaesref.so (tests/test_oracle.py and
 *       tests/golden/make_golden.py), plus OpenSSL CMAC as an independent third party.
 *
 * Byte/word conventions follow aes/include/aes/aes.h:48-82: a block is 16 bytes in
 * FIPS-197 column-major order, and "words" are little-endian views of 4 bytes.
 */
#ifndef HFV_ORACLE_H
#define HFV_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- AES-128 / AES-CMAC (aes/src/aes.c) ---------------------------------------- */
void orc_key_expansion(const uint8_t key[16], uint8_t sched[176]);          /* aes.c:120-137 */
void orc_cypher(const uint8_t in[16], const uint8_t sched[176], uint8_t out[16]); /* aes.c:249-293 */
void orc_cmac_subkeys(const uint8_t sched[176], uint8_t k1[16], uint8_t k2[16]);  /* aes.c:298-325 */
void orc_cmac(const uint8_t *data, size_t len, const uint8_t sched[176],
              const uint8_t k1[16], const uint8_t k2[16], uint8_t mac[16]);       /* aes.c:333-368 */
void orc_cmac_no_loops(const uint8_t *data, size_t len, const uint8_t sched[176],
                       const uint8_t k1[16], const uint8_t k2[16], uint8_t mac[16]); /* aes.c:377-434 */
const uint8_t *orc_sbox(void);

/* ---- hop_key (br/src/bpf/common.h:87-91): 176 B schedule + 16 B K1 ------------- */
typedef struct orc_hop_key {
    uint8_t sched[176];
    uint8_t k1[16];
} orc_hop_key;

/* br_loader.cpp:213-218: expansion, subkeys, keep K1 only */
void orc_hop_key_from_key(const uint8_t key[16], orc_hop_key *hk);

/* ---- hop-field layer (br/src/bpf/path_processing.h, xdp.c) ---------------------- */
/* defer_verify_hop_field (path_processing.h:39-58) with the AS-ingress beta rule
 * (path_processing.h:73-81).  inf = 8 wire bytes, hf = 12 wire bytes.
 * Writes the 16-byte struct macinput (include/bpf/scion.h:122-132) and returns the
 * expected 48-bit MAC as the little-endian u64 of hf->mac[0..5]. */
uint64_t orc_macinput_ingress(const uint8_t inf[8], const uint8_t hf[12], uint8_t mi[16]);
/* Same, with an explicit beta in host order (used by the egress rule, path_processing.h:136-142) */
uint64_t orc_macinput_beta(const uint8_t inf[8], const uint8_t hf[12], uint16_t beta, uint8_t mi[16]);

/* verify_hop_field (xdp.c:77-91): NULL key => fail closed */
int orc_verify_hop_field(const uint8_t mi[16], uint64_t expected, const orc_hop_key *key);

/* CMAC tag of one 16-byte block = aes_cmac_16bytes (aes.h:129-141) */
void orc_cmac16(const uint8_t mi[16], const orc_hop_key *key, uint8_t tag[16]);

/* ---- 64 B synthetic SCION record batch -------------------- */
enum { ORC_KEYSEL_ZERO = 0, ORC_KEYSEL_IFID = 1 };
#define ORC_REC_INF_OFF 40
#define ORC_REC_HF_OFF 48

/* Key index for a record: 0 (xdp.c:82) or the AS-ingress IFID & 0xff
 * (Cons ? HF.ConsIngress : HF.ConsEgress, xdp.c:151-157). */
uint32_t orc_record_key_index(const uint8_t *rec, int keysel);

/* Verify n records; bit i of pass_bits[i/64] = 1 iff record i's HF MAC verifies.
 * keys[idx] is used only when valid bit idx is set (missing key => fail closed).
 * pass_bits must hold ceil(n/64) words; unused high bits are cleared. */
void orc_verify_records(const uint8_t *recs, size_t stride, size_t n,
                        const orc_hop_key *keys, const uint32_t valid[8], int keysel,
                        uint64_t *pass_bits);
/* Same, split over nthreads pthreads (static contiguous partition, word-aligned). */
void orc_verify_records_mt(const uint8_t *recs, size_t stride, size_t n,
                           const orc_hop_key *keys, const uint32_t valid[8], int keysel,
                           uint64_t *pass_bits, int nthreads);

/* Synthetic generator (counter-based splitmix64; exact spec in DESIGN.md section 3). */
uint64_t orc_splitmix_at(uint64_t seed, uint64_t k);
void orc_gen_key_table(uint64_t seed, uint32_t nkeys, uint8_t keys[][16]);
void orc_gen_records(uint8_t *recs, size_t stride, size_t n, uint64_t seed, uint64_t first_index,
                     const orc_hop_key *keys, int keysel);

/* ---- full BR per-packet path (config 4), hfv_br_oracle.c -------------------------------- */
/* cfg: struct hfv_br_config (include/scion_hfv.h); key0: mac_key_map[0] or NULL.  Same
 * outputs as hfv_br_process; stats may be NULL. */
void orc_br_process(uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                    const void *cfg, const orc_hop_key *key0, uint8_t *action, uint8_t *verdict,
                    int32_t *egress_ifindex, uint64_t *stats);
/* feat_off: build options switched off (br/CMakeLists.txt:5-7) -- ENABLE_IPV4, ENABLE_IPV6,
 * ENABLE_SCION_PATH; the same bits as HFV_BR_NO_* in include/scion_hfv.h. */
#define ORC_BR_NO_IPV4 1u
#define ORC_BR_NO_IPV6 2u
#define ORC_BR_NO_SCION_PATH 4u
void orc_br_process_feat(uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                         const void *cfg, const orc_hop_key *key0, uint8_t *action, uint8_t *verdict,
                         int32_t *egress_ifindex, uint64_t *stats, int hf_check, uint32_t feat_off);
/* hf_check = 0: the ENABLE_HF_CHECK=OFF router (no hop-field MAC check). */
void orc_br_process_ex(uint8_t *pkts, size_t slot, const uint16_t *len, const uint32_t *ingress_ifindex, size_t n,
                       const void *cfg, const orc_hop_key *key0, uint8_t *action, uint8_t *verdict,
                       int32_t *egress_ifindex, uint64_t *stats, int hf_check);

#ifdef __cplusplus
}
#endif
#endif
