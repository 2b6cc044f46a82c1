#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (where /root/reference exists) after `make -C oracle`:

    python tests/golden/make_golden.py

Sources of truth, in order:
  * kat.json: the known-answer vectors of the reference's aes/src/test/aes_test.cpp:33-245
    (key expansion, FIPS-197 blocks, RFC 4493 CMAC at len 0/16/40/64), transcribed as data;
    the three AESCMAC payloads of aes/test/test.py:121-126 with their tags computed by the
    reference library; the aes_cmac_no_loops >64 B quirk (aes.c:394-431) computed by the
    reference; and the BR key convention of br/test/run_tests:113.
  * hf_*.npz: synthetic 64 B SCION records whose CMAC tags and verify
    bitmaps are computed by the REFERENCE aes.c (oracle/_ref/libaesref.so: aes_cmac soft
    path and aes_cmac_unaligned128 AES-NI path), cross-checked with OpenSSL's CMAC and
    with our restatement (oracle/libhfvoracle.so).  Any disagreement aborts.
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
ORC = ctypes.CDLL(os.path.join(ROOT, "oracle", "libhfvoracle.so"))
REF = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libaesref.so"))
SSL = ctypes.CDLL("libcrypto.so.3")

SEED_RECORDS = 0x5C100001
SEED_KEYS = 0x5C100100
KEY_1111 = b"1111111111111111"  # base64 MTExMTExMTExMTExMTExMQ== (br/test/run_tests:113)


def le_words_to_bytes(words):
    return b"".join(int(w).to_bytes(4, "little") for w in words)


# ---- aes_test.cpp vectors (data only) --------------------------------------------------
KEY_2B7E = le_words_to_bytes([0x16157E2B, 0xA6D2AE28, 0x8815F7AB, 0x3C4FCF09])
EXPANSION = [
    0x16157E2B, 0xA6D2AE28, 0x8815F7AB, 0x3C4FCF09, 0x17FEFAA0, 0xB12C5488, 0x3939A323, 0x05766C2A,
    0xF295C2F2, 0x43B9967A, 0x7A803559, 0x7FF65973, 0x7D47803D, 0x3EFE1647, 0x447E231E, 0x3B887A6D,
    0x41A544EF, 0x7F5B52A8, 0x3B2571B6, 0x00AD0BDB, 0xF8C6D1D4, 0x879D837C, 0xBCB8F2CA, 0xBC15F911,
    0x7AA3886D, 0xFD3E0B11, 0x4186F9DB, 0xFD9300CA, 0x0EF7544E, 0xF3C95F5F, 0xB24FA684, 0x4FDCA64E,
    0x2173D2EA, 0xD2BA8DB5, 0x60F52B31, 0x2F298D7F, 0xF36677AC, 0x21DCFA19, 0x4129D128, 0x6E005C57,
    0xA8F914D0, 0x8925EEC9, 0xC80C3FE1, 0xA60C63B6,
]
BLOCKS = [
    (KEY_2B7E, "3243f6a8885a308d313198a2e0370734", "3925841d02dc09fbdc118597196a0b32"),
    (le_words_to_bytes([0x03020100, 0x07060504, 0x0B0A0908, 0x0F0E0D0C]),
     "00112233445566778899aabbccddeeff", "69c4e0d86a7b0430d8cdb78070b4c55a"),
]
CMAC_MSG = ("6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
            "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710")
CMAC_EXPECTED = {
    0: [0x29691DBB, 0x283759E9, 0x127DA37F, 0x4667759B],
    16: [0xB4160A07, 0x44414D6B, 0x9DDD9BF7, 0x7C284AD0],
    40: [0x4767A6DF, 0x30E69ADE, 0x6132CA30, 0x27C89714],
    64: [0xBFBEF051, 0x929D3B7E, 0x177449FC, 0xFE3C3679],
}
TESTPY_BLOCKS = ["00" * 16, "6bc1bee22e409f96e93d7e117393172a", "ff" * 16]  # aes/test/test.py:122-126


def ref_sched(key):
    s = ctypes.create_string_buffer(176)
    REF.aes_key_expansion(key, s)
    return s


def ref_subkeys(sched):
    sk = ctypes.create_string_buffer(32)
    REF.aes_cmac_subkeys(sched, sk)
    return sk.raw[:16], sk.raw[16:]


def ref_cmac(data, key, fn="aes_cmac"):
    s = ref_sched(key)
    sk = ctypes.create_string_buffer(32)
    REF.aes_cmac_subkeys(s, sk)
    mac = ctypes.create_string_buffer(16)
    getattr(REF, fn)(data, ctypes.c_size_t(len(data)), s, sk, mac)
    return mac.raw


def ssl_cmac(data, key):
    SSL.CMAC_CTX_new.restype = ctypes.c_void_p
    SSL.EVP_aes_128_cbc.restype = ctypes.c_void_p
    ctx = ctypes.c_void_p(SSL.CMAC_CTX_new())
    assert SSL.CMAC_Init(ctx, key, ctypes.c_size_t(16), ctypes.c_void_p(SSL.EVP_aes_128_cbc()), None) == 1
    if data:
        assert SSL.CMAC_Update(ctx, data, ctypes.c_size_t(len(data))) == 1
    out = ctypes.create_string_buffer(16)
    olen = ctypes.c_size_t(0)
    assert SSL.CMAC_Final(ctx, out, ctypes.byref(olen)) == 1
    SSL.CMAC_CTX_free(ctx)
    return out.raw


def make_kat():
    msg = bytes.fromhex(CMAC_MSG)
    s = ref_sched(KEY_2B7E)
    assert list(np.frombuffer(s.raw, dtype="<u4")) == EXPANSION
    k1, k2 = ref_subkeys(s)
    for key, pt, ct in BLOCKS:
        out = ctypes.create_string_buffer(16)
        REF.aes_cypher(bytes.fromhex(pt), ref_sched(key), out)
        assert out.raw.hex() == ct
    cmac = []
    for L, words in CMAC_EXPECTED.items():
        exp = le_words_to_bytes(words)
        for fn in ("aes_cmac", "aes_cmac_no_loops"):
            assert ref_cmac(msg[:L], KEY_2B7E, fn) == exp, (fn, L)
        assert ssl_cmac(msg[:L], KEY_2B7E) == exp
        cmac.append({"len": L, "tag": exp.hex()})
    testpy = []
    for blk in TESTPY_BLOCKS:
        t = ref_cmac(bytes.fromhex(blk), KEY_2B7E)
        assert t == ssl_cmac(bytes.fromhex(blk), KEY_2B7E)
        testpy.append({"data": blk, "tag": t.hex()})
    # aes_cmac_no_loops silently processes at most 4 blocks (aes.c:394-431): record the
    # reference's own output for a few >64 B lengths so the restatement keeps the quirk.
    long_msg = bytes(range(200))
    quirk = [{"len": L, "tag": ref_cmac(long_msg[:L], KEY_2B7E, "aes_cmac_no_loops").hex(),
              "tag_full": ref_cmac(long_msg[:L], KEY_2B7E, "aes_cmac").hex()} for L in (65, 70, 80, 100, 128, 200)]
    # BR key convention and a worked hop-field sample
    hk = ctypes.create_string_buffer(192)
    REF.ref_hop_key(KEY_1111, hk)
    mi = bytes.fromhex("000012345f5e1000003f000100020000")
    tag1111 = ref_cmac(mi, KEY_1111)
    assert tag1111 == ssl_cmac(mi, KEY_1111)
    return {
        "source": "aes/src/test/aes_test.cpp:33-245, aes/test/test.py:122-126, br/test/run_tests:113",
        "key": KEY_2B7E.hex(),
        "expansion_le_words": [f"{w:08x}" for w in EXPANSION],
        "k1": k1.hex(), "k2": k2.hex(),
        "blocks": [{"key": k.hex(), "in": pt, "out": ct} for k, pt, ct in BLOCKS],
        "cmac_msg": CMAC_MSG,
        "cmac": cmac,
        "testpy_blocks": testpy,
        "no_loops_quirk": quirk,
        "br_key": {"base64": "MTExMTExMTExMTExMTExMQ==", "key": KEY_1111.hex(),
                   "hop_key": hk.raw.hex(), "macinput": mi.hex(), "tag": tag1111.hex(),
                   "zero_tag": ref_cmac(bytes(16), KEY_1111).hex()},
    }


def gen_records(n, keysel, hop_keys):
    recs = np.zeros((n, 64), dtype=np.uint8)
    kt = np.frombuffer(hop_keys, dtype=np.uint8)
    ORC.orc_gen_records(ctypes.c_void_p(recs.ctypes.data), ctypes.c_size_t(64), ctypes.c_size_t(n), ctypes.c_uint64(SEED_RECORDS),
                        ctypes.c_uint64(0), ctypes.c_void_p(kt.ctypes.data), ctypes.c_int(keysel))
    return recs


def make_hf(n, keysel, raw_keys):
    nkeys = len(raw_keys) // 16
    hop = bytearray()
    for k in range(nkeys):
        hk = ctypes.create_string_buffer(192)
        REF.ref_hop_key(raw_keys[16 * k:16 * k + 16], hk)
        hop += hk.raw
    orc_hop = bytearray()
    for k in range(nkeys):
        hk = ctypes.create_string_buffer(192)
        ORC.orc_hop_key_from_key(raw_keys[16 * k:16 * k + 16], hk)
        orc_hop += hk.raw
    assert bytes(hop) == bytes(orc_hop), "oracle hop_key != reference hop_key"
    hop_full = bytes(hop) + bytes(192 * (256 - nkeys))
    recs = gen_records(n, keysel, hop_full)
    valid = np.zeros(8, dtype=np.uint32)
    for k in range(nkeys):
        valid[k >> 5] |= np.uint32(1 << (k & 31))
    words = (n + 63) // 64
    bits = {}
    raw_full = raw_keys + bytes(16 * (256 - nkeys))
    for aesni in (0, 1):
        b = np.zeros(words, dtype=np.uint64)
        REF.ref_verify_records(ctypes.c_void_p(recs.ctypes.data), ctypes.c_size_t(64), ctypes.c_size_t(n), hop_full, raw_full,
                               ctypes.c_uint32(256), ctypes.c_void_p(valid.ctypes.data), ctypes.c_int(keysel), ctypes.c_void_p(b.ctypes.data),
                               ctypes.c_int(1), ctypes.c_int(aesni))
        bits[aesni] = b
    assert np.array_equal(bits[0], bits[1]), "reference soft vs AES-NI disagree"
    ob = np.zeros(words, dtype=np.uint64)
    ORC.orc_verify_records(ctypes.c_void_p(recs.ctypes.data), ctypes.c_size_t(64), ctypes.c_size_t(n), hop_full, ctypes.c_void_p(valid.ctypes.data),
                           ctypes.c_int(keysel), ctypes.c_void_p(ob.ctypes.data))
    assert np.array_equal(bits[0], ob), "oracle verify != reference verify"
    # per-record macinput / key index / full 16-byte tag via the reference aes_cmac
    mis = np.zeros((n, 16), dtype=np.uint8)
    kidx = np.zeros(n, dtype=np.uint8)
    tags = np.zeros((n, 16), dtype=np.uint8)
    for i in range(n):
        mi = ctypes.create_string_buffer(16)
        ORC.orc_macinput_ingress.restype = ctypes.c_uint64
        ORC.orc_macinput_ingress(recs[i, 40:48].tobytes(), recs[i, 48:60].tobytes(), mi)
        mis[i] = np.frombuffer(mi.raw, dtype=np.uint8)
        ORC.orc_record_key_index.restype = ctypes.c_uint32
        k = ORC.orc_record_key_index(recs[i].tobytes(), ctypes.c_int(keysel))
        kidx[i] = k
        key = raw_full[16 * k:16 * k + 16]
        t = ref_cmac(mi.raw, key)
        if i % 97 == 0:
            assert t == ssl_cmac(mi.raw, key)
        tags[i] = np.frombuffer(t, dtype=np.uint8)
    # the expected pass bit is exactly "no corruption" under a full key table
    expect = np.array([(tags[i, :6] == recs[i, 54:60]).all() for i in range(n)])
    got = np.array([(bits[0][i // 64] >> np.uint64(i % 64)) & np.uint64(1) for i in range(n)], dtype=bool)
    assert np.array_equal(expect, got)
    return dict(records=recs, pass_bits=bits[0], macinputs=mis, key_index=kidx, tags=tags,
                raw_keys=np.frombuffer(raw_full, dtype=np.uint8).reshape(256, 16),
                hop_keys=np.frombuffer(hop_full, dtype=np.uint8).reshape(256, 192),
                valid=valid, seed=np.uint64(SEED_RECORDS), keysel=np.int32(keysel), nkeys=np.int32(nkeys))


def main():
    kat = make_kat()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    single = make_hf(1000, 0, KEY_1111)
    np.savez_compressed(os.path.join(HERE, "hf_single.npz"), **single)
    keys = (ctypes.c_uint8 * (256 * 16))()
    ORC.orc_gen_key_table(ctypes.c_uint64(SEED_KEYS), ctypes.c_uint32(256), keys)
    multi = make_hf(1000, 1, bytes(keys))
    np.savez_compressed(os.path.join(HERE, "hf_ifid256.npz"), **multi)
    for name, d in (("single", single), ("ifid256", multi)):
        n = len(d["records"])
        passed = int(sum(bin(int(w)).count("1") for w in d["pass_bits"]))
        print(f"hf_{name}: {n} records, {passed} pass, {n - passed} fail")
    print("kat.json + hf_*.npz written; reference == oracle == OpenSSL on every vector")


if __name__ == "__main__":
    sys.exit(main())
