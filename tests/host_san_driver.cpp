// The product's host-side C++ (csrc/hfv_aes_host.cpp: the aes.h API the control plane
// links, verify_hop_field's scalar form and the br-loader base64 key decode;
// csrc/hfv_keymap.cpp and csrc/hfv_statsmap.cpp: the pinned key and counter maps)
// built with AddressSanitizer + UBSan and exercised here (tests/test_sanitize.py).  Expected
// values: FIPS-197 appendix B and the RFC 4493 CMAC vectors, which the reference's
// aes_test.cpp:33-245 also checks (tests/golden/kat.json).  Any failure aborts.
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "hfv_aes.h"
#include "scion_hfv.h"

namespace hfv {
// the library's error sink lives in hfv_api.cpp (not built here)
int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    char buf[256];
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return code;
}
}  // namespace hfv

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
            abort();                                                    \
        }                                                               \
    } while (0)

static void hex(const char *s, uint8_t *out, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        unsigned v;
        CHECK(sscanf(s + 2 * i, "%2x", &v) == 1);
        out[i] = (uint8_t)v;
    }
}

int main()
{
    // ---- aes.h host API -----------------------------------------------------------------
    aes_key key;
    hex("2b7e151628aed2a6abf7158809cf4f3c", key.b, 16);
    aes_key_schedule ks;
    aes_key_expansion(&key, &ks);
    aes_block in, out, want;
    hex("3243f6a8885a308d313198a2e0370734", in.b, 16);
    hex("3925841d02dc09fbdc118597196a0b32", want.b, 16);
    CHECK(aes_cypher(&in, &ks, &out) == 0 && !memcmp(out.b, want.b, 16));
    aes_block sub[2];
    aes_cmac_subkeys(&ks, sub);
    uint8_t k1[16], k2[16];
    hex("fbeed618357133667c85e08f7236a8de", k1, 16);
    hex("f7ddac306ae266ccf90bc11ee46d513b", k2, 16);
    CHECK(!memcmp(sub[0].b, k1, 16) && !memcmp(sub[1].b, k2, 16));
    uint8_t msg[64];
    hex("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
        "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710", msg, 64);
    const struct { size_t len; const char *tag; } rfc[] = {
        {0, "bb1d6929e95937287fa37d129b756746"}, {16, "070a16b46b4d4144f79bdd9dd04a287c"},
        {40, "dfa66747de9ae63030ca32611497c827"}, {64, "51f0bebf7e3b9d92fc49741779363cfe"}};
    for (const auto &v : rfc) {
        struct aes_cmac m1, m2;
        uint8_t t[16];
        hex(v.tag, t, 16);
        aes_cmac(msg, v.len, &ks, sub, &m1);
        aes_cmac_no_loops(msg, v.len, &ks, sub, &m2);
        CHECK(!memcmp(m1.b, t, 16) && !memcmp(m2.b, t, 16));
    }
    std::mt19937 rng(7);
    uint8_t buf[256];
    for (size_t len = 0; len < sizeof buf; ++len) {   // every length, exact-size heap copies
        for (size_t i = 0; i < len; ++i) buf[i] = (uint8_t)rng();
        uint8_t *heap = (uint8_t *)malloc(len ? len : 1);
        memcpy(heap, buf, len);
        struct aes_cmac m1, m2;
        aes_cmac(heap, len, &ks, sub, &m1);
        aes_cmac_no_loops(heap, len, &ks, sub, &m2);
        if (len <= AES_CMAC_NO_LOOP_MAX_BYTES) CHECK(!memcmp(m1.b, m2.b, 16));
        free(heap);
    }

    // ---- verify_hop_field's scalar form and the br-loader key decode ----------------------
    // the BR key convention (run_tests:113) and a hop-field macinput whose tag starts
    // a6 40 53 45 fa 79 (SURVEY 8c golden sample, OpenSSL-checked)
    aes_key bk;
    CHECK(hfv_decode_key_b64("MTExMTExMTExMTExMTExMQ==", &bk) == 0);
    for (int i = 0; i < 16; ++i) CHECK(bk.b[i] == '1');
    CHECK(hfv_decode_key_b64("MTEx", &bk) != 0);
    hop_key bhk;
    aes_key_expansion(&bk, &bhk.key);
    aes_block bsub[2];
    aes_cmac_subkeys(&bhk.key, bsub);
    bhk.subkey = bsub[0];
    macinput mi;
    hex("000012345f5e1000003f000100020000", reinterpret_cast<uint8_t *>(&mi), 16);
    const uint64_t expected = 0x79fa455340a6ull;   // LE u64 of tag bytes 0..5
    CHECK(hfv_verify_macinput(&mi, expected, &bhk) == 1);
    CHECK(hfv_verify_macinput(&mi, expected ^ 1, &bhk) == 0);
    CHECK(hfv_verify_macinput(&mi, expected, nullptr) == 0);   // missing key fails closed

    // ---- pinned key map and counter map ---------------------------------------------------
    if (!getenv("HFV_PIN_DIR")) {   // the test passes its own temporary directory
        static char dir[] = "/tmp/hfv_san_XXXXXX";
        CHECK(mkdtemp(dir) != nullptr);
        setenv("HFV_PIN_DIR", dir, 1);
    }
    char path[512];
    CHECK(hfv_keymap_path("br1", path, sizeof path) == 0);
    CHECK(hfv_keymap_path("../etc", path, sizeof path) != 0);
    CHECK(hfv_keymap_path("br1", path, sizeof path) == 0);
    hop_key hk;
    memset(&hk, 0, sizeof hk);
    hk.key = ks;
    hk.subkey = sub[0];
    CHECK(hfv_keymap_update(path, 0, &hk) == 0);
    CHECK(hfv_keymap_update(path, 200, &hk) == 0);
    CHECK(hfv_keymap_update(path, HFV_MAX_KEYS, &hk) != 0);
    hop_key *slots = (hop_key *)calloc(HFV_MAX_KEYS, sizeof(hop_key));
    uint32_t valid[8];
    CHECK(hfv_keymap_read(path, slots, valid) == 0);
    CHECK(valid[0] == 1u && valid[6] == (1u << 8) && !memcmp(&slots[200], &hk, sizeof hk));
    CHECK(hfv_keymap_erase(path, 200) == 0);
    CHECK(hfv_keymap_erase(path, 200) != 0);   // erase of a missing element fails (Map::erase)
    CHECK(hfv_keymap_read(path, slots, valid) == 0 && valid[6] == 0);
    free(slots);
    char spath[512];
    CHECK(hfv_statsmap_path("br1", spath, sizeof spath) == 0);
    const size_t nst = HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS;
    uint64_t *st = (uint64_t *)calloc(nst, 8), *rd = (uint64_t *)calloc(nst, 8);
    for (size_t i = 0; i < nst; ++i) st[i] = i;
    CHECK(hfv_statsmap_add(spath, st) == 0 && hfv_statsmap_add(spath, st) == 0);
    CHECK(hfv_statsmap_read(spath, rd) == 0);
    for (size_t i = 0; i < nst; ++i) CHECK(rd[i] == 2 * i);
    free(st);
    free(rd);
    printf("host san ok\n");
    return 0;
}
