"""Runs the CPU checker's C code under AddressSanitizer + UBSan (host
sanitizers on the CPU restatement).  Started by tests/test_sanitize.py in a child process with
libasan preloaded and HFV_ORACLE_SO pointing at oracle/_san/libhfvoracle_san.so; any
out-of-bounds access or undefined behaviour aborts it.  Covers the AES/CMAC restatement (KATs,
random lengths incl. the aes_cmac_no_loops >64-byte quirk), the record generator and verifier
(both key-selection modes, ragged n), and the border-router restatement on PTF-derived fuzz
frames and on random garbage frames of every length up to the slot."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scion-xdp-br_amd"))
import br_fuzz as F  # noqa: E402
import br_topo as T  # noqa: E402
import orc  # noqa: E402

assert os.environ.get("HFV_ORACLE_SO", "").endswith("_san.so"), "expects the sanitizer build"


def aes_cmac():
    kat = json.load(open(os.path.join(HERE, "golden", "kat.json")))
    key, msg = bytes.fromhex(kat["key"]), bytes.fromhex(kat["cmac_msg"])
    for v in kat["cmac"]:   # RFC 4493 vectors (aes_test.cpp)
        assert orc.cmac(msg[:v["len"]], key).hex() == v["tag"]
        assert orc.cmac(msg[:v["len"]], key, no_loops=True).hex() == v["tag"]
    rng = np.random.default_rng(5)
    rkey = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    for length in range(0, 256):
        m = rng.integers(0, 256, length, dtype=np.uint8).tobytes()
        orc.cmac(m, rkey)
        orc.cmac(m, rkey, no_loops=True)
    return len(kat["cmac"])


def records():
    for keysel in (0, 1):
        raw = orc.gen_key_table(256) if keysel else orc.KEY_1111
        hk, valid = orc.key_table(raw)
        for n in (1, 63, 65, 4097, 100000):
            recs = orc.gen_records(n, hk, keysel)
            a = orc.verify_records(recs, hk, valid, keysel)
            b = orc.verify_records(recs, hk, valid, keysel, nthreads=4)
            assert np.array_equal(a, b) and a.any()


def router():
    mac = lambda k, m: orc.cmac(m, k)   # noqa: E731
    total = 0
    for v6 in (False, True):
        brs = {b: T.OracleBR(T.br_config(b, v6)) for b in ("br1", "br2", "br3")}
        hops = F.hop_inputs(brs, v6, mac)
        for br in ("br1", "br2", "br3"):
            frames, lens, ifidx = F.fuzz_batch(hops, br, v6, 3000, seed=77, payload_max=1500)
            orc.br_process(frames, lens, ifidx, T.br_config(br, v6), orc.hop_key(T.KEYS[1]))
            total += len(frames)
        # garbage: random bytes, every length 0..slot, random ingress interfaces
        rng = np.random.default_rng(99 + v6)
        n = 4096
        frames = rng.integers(0, 256, (n, T.SLOT), dtype=np.uint8)
        frames[::3, 12:14] = (0x08, 0x00) if not v6 else (0x86, 0xDD)   # many pass the EtherType
        lens = rng.integers(0, T.SLOT + 1, n).astype(np.uint16)
        ifidx = rng.integers(0, 70, n).astype(np.uint32)
        orc.br_process(frames, lens, ifidx, T.br_config("br1", v6), orc.hop_key(T.KEYS[1]))
        orc.br_process(frames, lens, ifidx, T.br_config("br2", v6), None)
        total += 2 * n
    return total


if __name__ == "__main__":
    k = aes_cmac()
    records()
    f = router()
    print(f"san ok: {k} CMAC KATs, random CMAC lengths 0..255, record batches, {f} router frames")
