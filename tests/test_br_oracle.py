"""Config 4 on the CPU: the border-router oracle (oracle/hfv_br_oracle.c) against the
reference's own PTF expectations (br/test/ptf_tests/tests.py), re-derived from the SCION
path rules because scapy/scapy_scion/ptf are not installed; and the verdict of every
process_packet exit (br/src/bpf/xdp.c:98-283) on hand-made frames.

The BPF program itself cannot be built here (no clang BPF target / libbpf), so beyond the
PTF scenarios the oracle's quirk handling is pinned by reading xdp.c/parser.h/
path_processing.h/rewrite.h only ("parity partially pinned").
"""
import struct

import numpy as np
import pytest

import br_fuzz as F
import br_topo as T
import orc
import scion_hfv as hfv
from scion_hfv import packets as P

V = hfv.VERDICT
MAC = lambda k, m: orc.cmac(m, k)   # noqa: E731  checker-side AES for building test paths


@pytest.fixture(scope="module", params=[False, True], ids=["ipv4", "ipv6"])
def topo(request):
    v6 = request.param
    return v6, {b: T.OracleBR(T.br_config(b, v6)) for b in ("br1", "br2", "br3")}


def test_config_layout():
    import ctypes
    assert ctypes.sizeof(hfv.BrConfig) == 5076
    assert (ctypes.sizeof(hfv.BrIntIface), ctypes.sizeof(hfv.BrIngress), ctypes.sizeof(hfv.BrEgress),
            ctypes.sizeof(hfv.BrRoute)) == (28, 32, 48, 44)


def test_ptf_scenarios(topo):
    """DirectlyAttachedTest / ForwardToSiblingTest / IpForwardTest x down/up/core/seg_switch:
    egress frame byte-identical to the expected one, SCION_FORWARD counted on the first BR's
    ingress port with the frame length (tests.py:204-236)."""
    v6, brs = topo
    for name, kind, frame, first, ifi, want, veth_out in F.ptf_cases(v6, MAC):
        out, last, egress, trace = T.run_chain(brs, frame, first, ifi)
        assert out == want, (name, kind)
        assert egress == veth_out
        for br, a, v, _ in trace:
            assert (a, v) == (4, V["SCION_FORWARD"]), (name, kind, br)
        stats = trace[0][3]
        assert stats[ifi, 0, 1] == len(frame) and stats[ifi, 1, 1] == 1
        assert stats.sum() == len(frame) + 1


def _direct(v6=False, kind="down", seed=7):
    ing_enc, egr_enc, first, ifi = T.encaps(1, 2, v6)
    path = P.ptf_path(kind, 1, 2, T.KEYS, seed=seed, mac_fn=MAC)
    return ing_enc, path, ifi


def _run1(frame, ifi, br="br1", v6=False, key0=T.KEYS[1], cfg=None, ln=None):
    b = T.OracleBR(cfg or T.br_config(br, v6), key0=key0)
    buf, lens = T.to_slots([frame])
    if ln is not None:
        lens[0] = ln
    a, v, e, s = b.process(buf, lens, np.array([ifi], dtype=np.uint32))
    return int(a[0]), int(v[0]), int(e[0]), s, buf[0, :len(frame)].tobytes()


def test_not_scion_and_parse_errors():
    ing_enc, path, ifi = _direct()
    good = ing_enc.frame(P.scion_header(path.pack()))
    arp = good[:12] + b"\x08\x06" + good[14:]
    assert _run1(arp, ifi)[:2] == (2, V["NOT_SCION"])
    tcp = P.udp_ip_frame("02:00:00:00:00:01", "02:00:00:00:00:00", "10.1.1.1", "10.1.1.2", 50000, 50000,
                         P.scion_header(path.pack()), ip_proto=6)
    assert _run1(tcp, ifi)[:2] == (2, V["NOT_SCION"])
    assert _run1(good, ifi, ln=30)[:2] == (2, V["NOT_SCION"])            # truncated in IP
    assert _run1(good, ifi, ln=14 + 20 + 8 + 10)[:2] == (1, V["PARSE_ERROR"])   # truncated in SCION
    v1 = bytearray(good)
    v1[42] = 0x10                                                       # SCION version 1
    assert _run1(bytes(v1), ifi)[:2] == (2, V["NOT_IMPLEMENTED"])
    pt = bytearray(good)
    pt[42 + 8] = 2                                                      # path type EPIC
    assert _run1(bytes(pt), ifi)[:2] == (2, V["NOT_IMPLEMENTED"])


def test_interface_checks():
    ing_enc, path, ifi = _direct()
    good = ing_enc.frame(P.scion_header(path.pack()))
    assert _run1(good, 3)[:2] == (1, V["NO_INTERFACE"])                  # arrived on the wrong port
    other = P.ptf_path("down", 2, 1, T.KEYS, seed=7, mac_fn=MAC)            # HF says ingress 2
    assert _run1(ing_enc.frame(P.scion_header(other.pack())), ifi)[:2] == (1, V["NO_INTERFACE"])


def test_router_alert_and_last_hop():
    ing_enc, path, ifi = _direct()
    p = path.copy()
    p.hops[1].flags = 2
    assert _run1(ing_enc.frame(P.scion_header(p.pack())), ifi)[:2] == (2, V["ROUTER_ALERT"])
    p = path.copy()
    p.curr_hf = 2                                                       # last hop: local delivery
    p.hops[2].ing = 1
    assert _run1(ing_enc.frame(P.scion_header(p.pack())), ifi)[:2] == (2, V["NOT_IMPLEMENTED"])


def test_bad_mac_and_missing_key():
    ing_enc, path, ifi = _direct()
    p = path.copy()
    p.hops[1].mac = bytes([p.hops[1].mac[0] ^ 1]) + p.hops[1].mac[1:]
    a, v, e, s, out = _run1(ing_enc.frame(P.scion_header(p.pack())), ifi)
    assert (a, v) == (1, V["INVALID_HF"])
    assert e == 3            # the rewrite and next-hop decision happened before the check (xdp.c:242 vs 264)
    good = ing_enc.frame(P.scion_header(path.pack()))
    assert _run1(good, ifi, key0=None)[:2] == (1, V["INVALID_HF"])
    assert _run1(good, ifi, key0=T.KEYS[2])[:2] == (1, V["INVALID_HF"])


def test_hf_check_off_forwards_bad_macs():
    """ENABLE_HF_CHECK=OFF (br/CMakeLists.txt:8, path_processing.h:43, xdp.c:259-274): the same
    frame with a corrupted hop-field MAC, or with no key installed, is forwarded and rewritten
    exactly like the good frame with the check on."""
    ing_enc, path, ifi = _direct()
    good = ing_enc.frame(P.scion_header(path.pack()))
    p = path.copy()
    p.hops[1].mac = bytes([p.hops[1].mac[0] ^ 1]) + p.hops[1].mac[1:]
    bad = ing_enc.frame(P.scion_header(p.pack()))
    ref = _run1(good, ifi)
    import orc
    for frame, key0 in ((bad, T.KEYS[1]), (good, None)):
        buf, lens = T.to_slots([frame])
        hk = orc.hop_key(key0) if key0 is not None else None
        a, v, e, s = orc.br_process(buf, lens, np.array([ifi], dtype=np.uint32), T.br_config("br1"), hk,
                                    hf_check=False)
        assert (int(a[0]), int(v[0]), int(e[0])) == ref[:3] == (4, V["SCION_FORWARD"], 3)
        out = buf[0, :len(frame)].tobytes()
        if frame is good:
            assert out == ref[4]


def test_build_options():
    """ENABLE_IPV4 / ENABLE_IPV6 / ENABLE_SCION_PATH off (br/CMakeLists.txt:5-7): parse_underlay
    has no case for the family (parser.h:60,81) -> NOT_SCION, XDP_PASS, frame untouched;
    parse_scion has no case for the standard path (parser.h:140) -> NOT_IMPLEMENTED.  The loader
    check refuses tables holding an address of a switched-off family (maps.cpp:68-80)."""
    for v6 in (False, True):
        ing_enc, egr_enc, first, ifi = T.encaps(1, 2, v6)
        path = P.ptf_path("down", 1, 2, T.KEYS, seed=7, mac_fn=MAC)
        frame = ing_enc.frame(P.scion_header(path.pack()))
        cfg = T.br_config("br1", v6)
        for feat, want in ((hfv.BR_NO_IPV6 if v6 else hfv.BR_NO_IPV4, (2, V["NOT_SCION"])),
                           (hfv.BR_NO_SCION_PATH, (2, V["NOT_IMPLEMENTED"])),
                           (hfv.BR_NO_IPV4 if v6 else hfv.BR_NO_IPV6, (4, V["SCION_FORWARD"]))):
            buf, lens = T.to_slots([frame])
            a, v, e, s = orc.br_process(buf, lens, np.array([ifi], dtype=np.uint32), cfg, orc.hop_key(T.KEYS[1]),
                                        feat_off=feat)
            assert (int(a[0]), int(v[0])) == want, (v6, feat)
            if want[0] == 2:
                assert buf[0, :len(frame)].tobytes() == frame and int(e[0]) == -1
        other = hfv.BR_NO_IPV6 if v6 else hfv.BR_NO_IPV4
        with pytest.raises(hfv.HfvError, match="IPv%d support is deactivated" % (6 if v6 else 4)):
            hfv.br_config_check_options(cfg, other)
        hfv.br_config_check_options(cfg, hfv.BR_NO_SCION_PATH | (hfv.BR_NO_IPV4 if v6 else hfv.BR_NO_IPV6))


def test_unknown_egress_aborts_and_falls_through():
    """VERDICT_ABORT is XDP_ABORTED = 0, not > 0: the MAC check and the redirect still run and
    record a second verdict (xdp.c:194, 256-283)."""
    ing_enc, _, ifi = _direct()
    p = P.Path([P.InfoField(True)], [P.HopField(0, 1), P.HopField(1, 9), P.HopField(1, 0)], [3], mac_fn=MAC)
    p.init_macs([T.KEYS[2], T.KEYS[1], T.KEYS[3]], [5]).egress(T.KEYS[2], verify=True)
    frame = ing_enc.frame(P.scion_header(p.pack()))
    a, v, e, s, out = _run1(frame, ifi)
    assert (a, v, e) == (0, 0, -1)
    assert s[ifi, 1, 0] == 2 and s[ifi, 0, 0] == 2 * len(frame)
    assert out == frame                                                 # no rewrite


def test_fib_outcomes():
    ing_enc, path, ifi = _direct()
    frame = ing_enc.frame(P.scion_header(path.pack()))
    cfg = T.br_config("br1")
    cfg.n_routes = 0                                                    # no route: NOT_FWDED -> pass
    assert _run1(frame, ifi, cfg=cfg)[:2] == (2, V["FIB_LKUP_PASS"])
    cfg = T.br_config("br1")
    cfg.add_route("10.1.2.0", 24, 3, "02:00:00:00:00:03", "02:00:00:00:00:02", ret=1)   # shorter prefix loses
    assert _run1(frame, ifi, cfg=cfg)[:2] == (4, V["SCION_FORWARD"])
    cfg.add_route("10.1.2.1", 32, 3, "02:00:00:00:00:03", "02:00:00:00:00:02", ret=1)   # tie: first wins
    assert _run1(frame, ifi, cfg=cfg)[:2] == (4, V["SCION_FORWARD"])
    cfg = T.br_config("br1")
    cfg.routes[1].ret = 2                                               # BPF_FIB_LKUP_RET_UNREACHABLE
    assert _run1(frame, ifi, cfg=cfg)[:2] == (1, V["FIB_LKUP_DROP"])
    cfg = T.br_config("br1")
    cfg.n_tx_ports = 0                                                  # redirect target not in tx_port_map
    assert _run1(frame, ifi, cfg=cfg)[:3] == (0, 0, 3)


def test_underlay_mismatch():
    ing_enc, path, ifi = _direct()
    frame = ing_enc.frame(P.scion_header(path.pack()))
    cfg = T.br_config("br1")
    for i in range(cfg.n_egress):
        if cfg.egress[i].ifid == 2:
            cfg.egress[i].family = hfv.AF_INET6
    assert _run1(frame, ifi, cfg=cfg)[:2] == (2, V["UNDERLAY_MISMATCH"])


def test_fuzz_is_deterministic_and_covers_verdicts(topo):
    """The mutation generator used by the GPU parity test reaches every verdict."""
    v6, brs = topo
    hops = F.hop_inputs(brs, v6, MAC)
    seen = set()
    for br in ("br1", "br2", "br3"):
        frames, lens, ifidx = F.fuzz_batch(hops, br, v6, 3000, seed=11)
        f2, l2, i2 = F.fuzz_batch(hops, br, v6, 3000, seed=11)
        assert (frames == f2).all() and (lens == l2).all() and (ifidx == i2).all()
        a, v, e, s = brs[br].process(frames, lens, ifidx)
        seen |= set(int(x) for x in np.unique(v))
        assert s[:, 1, :].sum() >= len(frames)
    want = {V[k] for k in ("SCION_FORWARD", "PARSE_ERROR", "NOT_SCION", "NOT_IMPLEMENTED", "NO_INTERFACE",
                           "ROUTER_ALERT", "INVALID_HF", "ABORT")}
    assert want <= seen, sorted(want - seen)


@pytest.mark.parametrize("v6", [False, True], ids=["ipv4", "ipv6"])
def test_segid_rewrite_inside_checked_hop_field(v6):
    """CurrINF past the info fields: the SegID scion_as_egress rewrites is part of the hop field
    whose MAC is checked afterwards; the check uses the bytes read before the rewrite."""
    frame, first, ifi, want = F.overlap_frame(v6)
    br = T.OracleBR(T.br_config(first, v6))
    buf, lens = T.to_slots([frame])
    a, v, e, _ = br.process(buf, lens, np.array([ifi], dtype=np.uint32))
    assert (a[0], v[0]) == (4, V["SCION_FORWARD"])
    assert buf[0, :len(want)].tobytes() == want


def test_ipv4_options_move_fields_not_outcomes():
    """IPv4 options shift the SCION header by 4..40 bytes (parser.h:60-66 skips IHL * 4 - 20):
    every hop input of BR 1 gets the same action, verdict and egress with 0..10 option words
    (the GPU test of the same batch puts fields on both sides of the kernel's 128-byte window)."""
    brs = {b: T.OracleBR(T.br_config(b, False)) for b in ("br1", "br2", "br3")}
    frames, lens, ifidx, m = F.options_shift_batch(F.hop_inputs(brs, False, MAC))
    a, v, e, _ = orc.br_process(frames, lens, ifidx, T.br_config("br1"), orc.hop_key(T.KEYS[1]))
    a, v, e = (x.reshape(11, m) for x in (a, v, e))
    assert (a == a[0]).all() and (v == v[0]).all() and (e == e[0]).all()
    assert (v[0] == V["SCION_FORWARD"]).sum() >= m // 2
