"""ctypes access to the CPU checker (oracle/libhfvoracle.so) and, when it was built, the
reference's own AES compiled from /root/reference (oracle/_ref/libaesref.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# HFV_ORACLE_SO: another build of the same checker (the sanitizer build, tests/test_sanitize.py)
ORACLE_SO = os.environ.get("HFV_ORACLE_SO") or os.path.join(ORACLE_DIR, "libhfvoracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libaesref.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

SEED_RECORDS = 0x5C100001
SEED_KEYS = 0x5C100100
KEY_1111 = b"1111111111111111"

_orc = None
_ref = None


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data) if hasattr(a, "ctypes") else a


def oracle():
    global _orc
    if _orc is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", ORACLE_DIR, "libhfvoracle.so"], check=True, capture_output=True)
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_macinput_ingress.restype = ctypes.c_uint64
        L.orc_record_key_index.restype = ctypes.c_uint32
        L.orc_splitmix_at.restype = ctypes.c_uint64
        L.orc_splitmix_at.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        _orc = L
    return _orc


def reference():
    """The reference aes.c build, or None when it is not available (e.g. no /root/reference)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = ctypes.CDLL(REF_SO)
    return _ref


def hop_key(key: bytes) -> bytes:
    hk = ctypes.create_string_buffer(192)
    oracle().orc_hop_key_from_key(bytes(key), hk)
    return hk.raw


def cmac(data: bytes, key: bytes, no_loops=False) -> bytes:
    L = oracle()
    sched = ctypes.create_string_buffer(176)
    L.orc_key_expansion(bytes(key), sched)
    k1, k2 = ctypes.create_string_buffer(16), ctypes.create_string_buffer(16)
    L.orc_cmac_subkeys(sched, k1, k2)
    mac = ctypes.create_string_buffer(16)
    fn = L.orc_cmac_no_loops if no_loops else L.orc_cmac
    fn(bytes(data), ctypes.c_size_t(len(data)), sched, k1, k2, mac)
    return mac.raw


def key_table(raw_keys: bytes):
    """(hop_keys[256*192], valid[8]) for a list of raw 16-byte keys in slots 0..k-1."""
    nk = len(raw_keys) // 16
    hk = bytearray(256 * 192)
    valid = np.zeros(8, dtype=np.uint32)
    for k in range(nk):
        hk[192 * k:192 * k + 192] = hop_key(raw_keys[16 * k:16 * k + 16])
        valid[k >> 5] |= np.uint32(1 << (k & 31))
    return np.frombuffer(bytes(hk), dtype=np.uint8).copy(), valid


def gen_key_table(nkeys=256, seed=SEED_KEYS) -> bytes:
    buf = (ctypes.c_uint8 * (16 * nkeys))()
    oracle().orc_gen_key_table(ctypes.c_uint64(seed), ctypes.c_uint32(nkeys), buf)
    return bytes(buf)


def gen_records(n, hop_keys, keysel, seed=SEED_RECORDS, first_index=0, stride=64):
    recs = np.zeros((n, stride), dtype=np.uint8)
    oracle().orc_gen_records(_vp(recs), ctypes.c_size_t(stride), ctypes.c_size_t(n), ctypes.c_uint64(seed),
                             ctypes.c_uint64(first_index), _vp(hop_keys), ctypes.c_int(keysel))
    return recs


def verify_records(recs, hop_keys, valid, keysel, stride=64, n=None, nthreads=1):
    n = len(recs) if n is None else n
    bits = np.zeros((n + 63) // 64, dtype=np.uint64)
    oracle().orc_verify_records_mt(_vp(recs), ctypes.c_size_t(stride), ctypes.c_size_t(n), _vp(hop_keys), _vp(valid),
                                   ctypes.c_int(keysel), _vp(bits), ctypes.c_int(nthreads))
    return bits


def ref_verify_records(recs, raw_keys_256: bytes, hop_keys, valid, keysel, nthreads=1, aesni=0, stride=64, n=None):
    """Reference aes.c (soft) or AES-NI path over the same records; None if not built."""
    R = reference()
    if R is None:
        return None
    n = len(recs) if n is None else n
    bits = np.zeros((n + 63) // 64, dtype=np.uint64)
    R.ref_verify_records(_vp(recs), ctypes.c_size_t(stride), ctypes.c_size_t(n), _vp(hop_keys), bytes(raw_keys_256),
                         ctypes.c_uint32(256), _vp(valid), ctypes.c_int(keysel), _vp(bits), ctypes.c_int(nthreads),
                         ctypes.c_int(aesni))
    return bits


def macinputs_from_records(recs):
    """(macinput[n,16], expected u64[n], key_index_ifid u8[n]) via the oracle's rule."""
    L = oracle()
    n = len(recs)
    mi = np.zeros((n, 16), dtype=np.uint8)
    exp = np.zeros(n, dtype=np.uint64)
    kidx = np.zeros(n, dtype=np.uint8)
    buf = ctypes.create_string_buffer(16)
    for i in range(n):
        r = recs[i].tobytes()
        exp[i] = L.orc_macinput_ingress(r[40:48], r[48:60], buf)
        mi[i] = np.frombuffer(buf.raw, dtype=np.uint8)
        kidx[i] = L.orc_record_key_index(r, ctypes.c_int(1))
    return mi, exp, kidx


def expected_pass_rule(n, seed=SEED_RECORDS, first_index=0):
    """Generator-side truth: record i is corrupted iff r2 & 15 == 0, with
    r2 = splitmix64 draw 4i+2; numpy-vectorised so it scales to full bench sizes."""
    i = np.arange(first_index, first_index + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.uint64(4) * i + np.uint64(3)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(15)) != 0


BR_STATS_SHAPE = (64, 2, 11)   # HFV_BR_STATS_IFINDEX x (bytes, packets) x HFV_BR_COUNTERS


def br_process(frames, lens, ifidx, cfg, key0_hop_key=None, stats=None, hf_check=True, feat_off=0):
    """Oracle border router (hfv_br_oracle.c) over frames[n, slot] in place.
    Returns (action u8[n], verdict u8[n], egress i32[n], stats u64[64, 2, 11])."""
    n, slot = frames.shape
    assert frames.dtype == np.uint8 and frames.flags.c_contiguous
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    ifidx = np.ascontiguousarray(ifidx, dtype=np.uint32)
    action = np.zeros(n, dtype=np.uint8)
    verdict = np.zeros(n, dtype=np.uint8)
    egress = np.zeros(n, dtype=np.int32)
    if stats is None:
        stats = np.zeros(BR_STATS_SHAPE, dtype=np.uint64)
    key = ctypes.create_string_buffer(bytes(key0_hop_key), 192) if key0_hop_key is not None else None
    oracle().orc_br_process_feat(_vp(frames), ctypes.c_size_t(slot), _vp(lens), _vp(ifidx), ctypes.c_size_t(n),
                                 ctypes.byref(cfg), key, _vp(action), _vp(verdict), _vp(egress), _vp(stats),
                                 ctypes.c_int(1 if hf_check else 0), ctypes.c_uint32(feat_off))
    return action, verdict, egress, stats


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name)))
