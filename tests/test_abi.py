"""The C-ABI library loads and exports what include/*.h declares; the host-side
control-plane API (aes.h surface, base64 key decode, scalar verify_hop_field) matches the
reference's known answers.  CPU only: no compute call here touches a GPU."""
import ctypes
import errno
import json
import os
import re
import subprocess

import numpy as np
import pytest

import orc
import scion_hfv as hfv

ROOT = orc.ROOT
KAT = json.load(open(os.path.join(orc.GOLDEN, "kat.json")))


def declared_functions():
    names = set()
    for h in ("scion_hfv.h", "hfv_aes.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(\w+)\s*\([^;{]*\)\s*;", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_lib_exports_every_declared_symbol():
    names = declared_functions()
    assert {"hfv_verify_records", "hfv_key_add", "aes_cmac", "aes_key_expansion"} <= names
    out = subprocess.run(["nm", "-D", "--defined-only", hfv.LIB_PATH], check=True, capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = sorted(names - exported)
    assert not missing, missing
    assert "AES_SBox" in exported
    L = hfv.lib()
    assert L.hfv_abi_version() == 3


TEST_HOOKS = ("hfv_debug_loop_host_stage", "hfv_debug_publish_delay", "hfv_debug_relay_delay", "hfv_debug_br_grid",
              "hfv_debug_br_split")


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_test_hooks_only_in_the_test_build():
    """the hooks that change what the library does (a host callback in place
    of the router kernel, delays, launch-shape overrides) are compiled into the test build only;
    the product library exports none of them, and its diagnostics are read-only."""
    prod, test = _exports(hfv.LIB_PATH), _exports(hfv.TEST_LIB_PATH)
    assert not prod & set(TEST_HOOKS), sorted(prod & set(TEST_HOOKS))
    assert set(TEST_HOOKS) <= test
    assert declared_functions() <= test            # the test build is the product plus the hooks
    assert {s for s in prod if s.startswith("hfv_")} <= test
    # the spin kernel behind the publish delay lives in the test build's own object
    assert not [s for s in prod if "debug_spin" in s] and [s for s in test if "debug_spin" in s]


def test_exported_sbox():
    sbox = bytes((ctypes.c_uint8 * 256).in_dll(hfv.lib(), "AES_SBox"))
    L = orc.oracle()
    L.orc_sbox.restype = ctypes.POINTER(ctypes.c_uint8 * 256)
    assert sbox == bytes(L.orc_sbox().contents)


def test_host_aes_api_kats():
    key = bytes.fromhex(KAT["key"])
    sched = hfv.aes_key_expansion(key)
    assert [f"{w:08x}" for w in np.frombuffer(sched, dtype="<u4")] == KAT["expansion_le_words"]
    k1, k2 = hfv.aes_cmac_subkeys(sched)
    assert (k1.hex(), k2.hex()) == (KAT["k1"], KAT["k2"])
    for v in KAT["blocks"]:
        assert hfv.aes_cypher(bytes.fromhex(v["in"]), hfv.aes_key_expansion(bytes.fromhex(v["key"]))).hex() == v["out"]
    msg = bytes.fromhex(KAT["cmac_msg"])
    for v in KAT["cmac"]:
        assert hfv.aes_cmac(msg[: v["len"]], key).hex() == v["tag"]
        assert hfv.aes_cmac(msg[: v["len"]], key, no_loops=True).hex() == v["tag"]
    long_msg = bytes(range(200))
    for v in KAT["no_loops_quirk"]:
        assert hfv.aes_cmac(long_msg[: v["len"]], key, no_loops=True).hex() == v["tag"]
        assert hfv.aes_cmac(long_msg[: v["len"]], key).hex() == v["tag_full"]


def test_host_aes_api_random_vs_oracle():
    rng = np.random.default_rng(3)
    for _ in range(50):
        key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        assert hfv.hop_key(key) == orc.hop_key(key)
        for L in (0, 1, 15, 16, 17, 33, 64, 65, 100):
            data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
            assert hfv.aes_cmac(data, key) == orc.cmac(data, key)
            assert hfv.aes_cmac(data, key, no_loops=True) == orc.cmac(data, key, no_loops=True)


def test_decode_key_b64_br_convention():
    br = KAT["br_key"]
    assert hfv.decode_key_b64(br["base64"]).hex() == br["key"]
    assert hfv.decode_key_b64("MjIyMjIyMjIyMjIyMjIyMg==") == b"2222222222222222"
    with pytest.raises(hfv.HfvError) as e:
        hfv.decode_key_b64("MTEx")  # br_loader.cpp:70: "Key has invalid length"
    assert e.value.code == -errno.EINVAL
    with pytest.raises(hfv.HfvError):
        hfv.decode_key_b64("MTExMTExMTExMTExMTExM!==")


def test_scalar_verify_macinput():
    g = orc.load_golden("hf_single.npz")
    hk = g["hop_keys"][0].tobytes()
    truth = np.unpackbits(g["pass_bits"].view(np.uint8), bitorder="little")
    for i in range(200):
        expected = int.from_bytes(g["records"][i, 54:60].tobytes(), "little")
        assert hfv.verify_macinput(g["macinputs"][i].tobytes(), expected, hk) == bool(truth[i])
    assert not hfv.verify_macinput(g["macinputs"][0].tobytes(), 0, None)  # no key: fail closed


def test_ctx_without_gpu_reports_enodev():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(hfv.HfvError) as e:
        hfv.Ctx(0)
    assert e.value.code == -errno.ENODEV


def test_shard_ranges_cover_word_aligned():
    for n in (0, 1, 63, 64, 1000, 1 << 20, (1 << 20) + 5):
        for world in (1, 2, 3, 4, 8):
            cuts = [hfv.shard_range(n, world, r) for r in range(world)]
            assert cuts[0][0] == 0 and cuts[-1][1] == n
            for (a0, a1), (b0, b1) in zip(cuts, cuts[1:]):
                assert a1 == b0 and a0 % 64 == 0


def test_new_entry_points_reject_bad_arguments_without_gpu():
    """The round-2 entry points fail with -EINVAL on a NULL ctx or missing buffers before any
    device work (CPU; the GPU behaviour is in test_gpu_loop / test_gpu_service / test_gpu_parity)."""
    L = hfv.lib()
    cfg = hfv.LoopConfig()
    st = hfv.LoopStats()
    assert L.hfv_loop_run(None, ctypes.byref(cfg), ctypes.byref(st)) == -errno.EINVAL
    t = ctypes.c_uint64()
    ms = ctypes.c_float()
    assert L.hfv_service_run(None, None, 0, ctypes.byref(t), ctypes.byref(ms)) == -errno.EINVAL
    assert L.hfv_verdict_counters(None, None, 64, 1, None, None, None) == -errno.EINVAL
    assert "NULL" in L.hfv_last_error().decode() or "null" in L.hfv_last_error().decode()
    assert ctypes.sizeof(hfv.LoopStats) == 8 * (5 + hfv.BR_COUNTERS) + 8 * 5 + 8 * 2 + 16


def test_ctypes_layouts_match_the_c_header(tmp_path):
    """The ctypes mirrors of the public structs have the C header's size and field offsets
    (compiled with gcc against include/scion_hfv.h)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    checks = {"hfv_loop_config": (hfv.LoopConfig, ["rx_ifindex", "total", "dma", "stats", "rx_ifname", "idle_ms"]),
              "hfv_loop_stats": (hfv.LoopStats, ["verdict_pkts", "seconds", "rx_truncated", "tx_errors", "numa_node",
                                                 "threads", "threads_on_node"]),
              "hfv_br_config": (hfv.BrConfig, ["egress", "routes", "tx_ports"])}
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "scion_hfv.h"', "int main(void) {"]
    for st, (_, fields) in checks.items():
        src.append('printf("%%zu\\n", sizeof(struct %s));' % st)
        for f in fields:
            src.append('printf("%%zu\\n", offsetof(struct %s, %s));' % (st, f))
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(root, "include"), str(c), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = []
    for st, (cls, fields) in checks.items():
        want.append(ctypes.sizeof(cls))
        want += [getattr(cls, f).offset for f in fields]
    assert got == want


def test_loop_frame_digest_is_order_free():
    """hfv_loop_run's transmitted-frame digest (mirrored in scion_hfv.loop_frame_digest) depends
    on the bytes and the egress port, and sums order-independently."""
    a, b = bytes(range(138)), bytes(range(1, 139))
    da, db = hfv.loop_frame_digest(a, 3), hfv.loop_frame_digest(b, 3)
    assert da != db and hfv.loop_frame_digest(a, 1) != da
    assert (da + db) % 2**64 == (db + da) % 2**64
    assert hfv.loop_frame_digest(a[:137], 3) != da
